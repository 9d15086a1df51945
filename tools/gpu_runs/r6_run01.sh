#!/bin/bash
# round 6: the 4-wave ring with one LDS read / DMA piece per MFMA gap (cfg 14) vs the clumped ring (cfg 13):
# correctness, microbench, in-step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_4w_gpu.py > gpurun_out/r6_01_test.log 2>&1 || { tail -30 gpurun_out/r6_01_test.log; exit 1; }
tail -3 gpurun_out/r6_01_test.log
timeout -k 10 300 python -u tools/bench_wgrad.py --cfgs 13,14,15,16,1213,1214 --only gate_up,down,lm_head --no-blas > gpurun_out/r6_01_wgrad.log 2>&1 || { tail -30 gpurun_out/r6_01_wgrad.log; exit 1; }
grep shape gpurun_out/r6_01_wgrad.log
DGRAD_CFGS=13,14 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r6_01_dgrad.log 2>&1 || { tail -30 gpurun_out/r6_01_dgrad.log; exit 1; }
tail -8 gpurun_out/r6_01_dgrad.log
DGRAD_SHAPES=lm_head DGRAD_CFGS=13,14 timeout -k 10 300 python -u tools/bench_dgrad.py > gpurun_out/r6_01_dgrad_lm.log 2>&1 || { tail -30 gpurun_out/r6_01_dgrad_lm.log; exit 1; }
tail -5 gpurun_out/r6_01_dgrad_lm.log
for v in 13 14 13 14; do
  SFTAMD_G4_RING=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_01_bench_$v.log 2>&1 || { tail -20 gpurun_out/r6_01_bench_$v.log; exit 1; }
  echo "ring $v $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r6_01_bench_$v.log | tr '\n' ' ')"
done
