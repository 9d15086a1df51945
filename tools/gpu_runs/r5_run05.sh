#!/bin/bash
# round 5: dgrad2 SwiGLU-bwd with the gate / up prefetch (cfg 71-73) correctness + microbench; in-step A/B of the plain
# row-contiguous kernel for gate_up (+ the SwiGLU kernel), o_proj and the NoPE qkv vs hipBLASLt
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "dgrad" > gpurun_out/r5_05_tests.log 2>&1 || { tail -30 gpurun_out/r5_05_tests.log; exit 1; }
tail -1 gpurun_out/r5_05_tests.log
DGRAD_CFGS=7,71,72,73 timeout -k 10 300 python -u tools/bench_dgrad.py --rounds 3 > gpurun_out/r5_05_dgrad.log 2>&1 || { tail -20 gpurun_out/r5_05_dgrad.log; exit 1; }
grep swiglu gpurun_out/r5_05_dgrad.log
run() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_05_$n.log 2>&1 || { tail -20 gpurun_out/r5_05_$n.log; exit 1; }
  echo "$n $(grep -o '"value": [0-9.]*' gpurun_out/r5_05_$n.log)"
}
for r in 1 2; do
  run base$r SFTAMD_TN_CFG=11
  run gu$r SFTAMD_TN_CFG=11 SFTAMD_FWD_HIP_N=22016
  run guo$r SFTAMD_TN_CFG=11 SFTAMD_FWD_HIP_N=22016,2048,3072
done
