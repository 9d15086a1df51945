#!/bin/bash
# round 6: AdamW with nontemporal streams + one SR hash per element pair: kernel tests, bandwidth, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adamw" tests/test_trainer_gpu.py > gpurun_out/r6_12_tests.log 2>&1 || { tail -40 gpurun_out/r6_12_tests.log; exit 1; }
tail -2 gpurun_out/r6_12_tests.log
timeout -k 10 120 python -u tools/bench_adamw.py > gpurun_out/r6_12_adamw.log 2>&1 || { tail -20 gpurun_out/r6_12_adamw.log; exit 1; }
cat gpurun_out/r6_12_adamw.log | grep moments
for i in 1 2; do
timeout -k 10 300 python -u bench.py > gpurun_out/r6_12_bench$i.log 2>&1 || { tail -20 gpurun_out/r6_12_bench$i.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r6_12_bench$i.log | tr '\n' ' '; echo
done
