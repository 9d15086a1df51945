#!/bin/bash
# recipe (reference parquet + evals), LoRA bench, default-step kernel profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r4_19_recipe.log 2>&1 || { tail -30 gpurun_out/r4_19_recipe.log; exit 1; }
grep '"metric"' gpurun_out/r4_19_recipe.log | cut -c1-400
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --freeze-policy lora > gpurun_out/r4_19_lora.log 2>&1 || { tail -20 gpurun_out/r4_19_lora.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/r4_19_lora.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof19 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r4_19_p.log 2>&1 || { tail -20 gpurun_out/r4_19_p.log; exit 1; }
db=$(ls /tmp/prof19/*/run_results.db /tmp/prof19/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 40 --out gpurun_out/r4_19_step_prof.md > /dev/null
head -30 gpurun_out/r4_19_step_prof.md
timeout -k 10 200 python -u tools/bench_down_pair.py > gpurun_out/r4_19_pair.log 2>&1 || { tail -20 gpurun_out/r4_19_pair.log; exit 1; }
cat gpurun_out/r4_19_pair.log
