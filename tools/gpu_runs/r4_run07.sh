#!/bin/bash
# same-box interleaved A/B of the forward routing with the round-3 persistent kernel (cfg 164)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --fused-cfgs 11,50,164 > gpurun_out/r4_07_fused.log 2>&1 || { tail -20 gpurun_out/r4_07_fused.log; exit 1; }
cat gpurun_out/r4_07_fused.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_07_$tag.log 2>&1 || { tail -20 gpurun_out/r4_07_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4_07_$tag.log)"
}
for r in 1 2; do
  run base$r SFTAMD_X=0
  run gu$r SFTAMD_GATE_UP=164
  run fwd$r SFTAMD_FWD_GEMM=persist SFTAMD_PERSIST_CFG=164
  run both$r SFTAMD_GATE_UP=164 SFTAMD_FWD_GEMM=persist SFTAMD_PERSIST_CFG=164
done
