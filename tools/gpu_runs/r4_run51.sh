#!/bin/bash
# end of round 4 (final tree): full GPU suite, headline bench, LoRA bench, recipe, default-step kernel profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4_51_tests.log 2>&1 || { tail -40 gpurun_out/r4_51_tests.log; exit 1; }
tail -1 gpurun_out/r4_51_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_51_bench.log 2>&1 || { tail -20 gpurun_out/r4_51_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_51_bench.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --freeze-policy lora > gpurun_out/r4_51_lora.log 2>&1 || { tail -20 gpurun_out/r4_51_lora.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_51_lora.log
timeout -k 10 600 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r4_51_recipe.log 2>&1 || { tail -30 gpurun_out/r4_51_recipe.log; exit 1; }
grep '"metric"' gpurun_out/r4_51_recipe.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof51 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r4_51_p.log 2>&1 || { tail -20 gpurun_out/r4_51_p.log; exit 1; }
db=$(ls /tmp/prof51/*/run_results.db /tmp/prof51/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r4_51_step_prof.md > /dev/null
head -12 gpurun_out/r4_51_step_prof.md
