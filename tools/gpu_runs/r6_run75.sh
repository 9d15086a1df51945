#!/bin/bash
# round 6 final validation (four-problem grids, unsplit partial round)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6_75_tests.log 2>&1 || { tail -40 gpurun_out/r6_75_tests.log; exit 1; }
tail -1 gpurun_out/r6_75_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_75_smoke.log 2>&1 || { tail -20 gpurun_out/r6_75_smoke.log; exit 1; }
tail -1 gpurun_out/r6_75_smoke.log
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [a-zA-Z0-9.-]*\|"train_pure_samples_per_second": [0-9.]*\|"peak_mem_gb": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py > gpurun_out/r6_75_bench$i.log 2>&1 || { tail -20 gpurun_out/r6_75_bench$i.log; exit 1; }
echo "headline $i: $(v gpurun_out/r6_75_bench$i.log)"
done
timeout -k 10 300 python -u bench.py --freeze-policy lora > gpurun_out/r6_75_lora.log 2>&1 || { tail -20 gpurun_out/r6_75_lora.log; exit 1; }
echo "lora: $(v gpurun_out/r6_75_lora.log)"
timeout -k 10 400 python -u bench.py --model llama3-8b --steps 10 --warmup 3 > gpurun_out/r6_75_llama.log 2>&1 || { tail -20 gpurun_out/r6_75_llama.log; exit 1; }
echo "llama: $(v gpurun_out/r6_75_llama.log)"
timeout -k 10 600 python -u bench.py --recipe --steps 40 > gpurun_out/r6_75_recipe.log 2>&1 || { tail -20 gpurun_out/r6_75_recipe.log; exit 1; }
echo "recipe: $(v gpurun_out/r6_75_recipe.log)"
