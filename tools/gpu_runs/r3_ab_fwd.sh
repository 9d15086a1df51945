#!/bin/bash
# End-to-end A/B of the forward GEMM routing (interleaved bench.py runs on one box):
#   base = hipBLASLt projections + SwiGLU kernel; gu12 / gu50 = gate_up GEMM with the SwiGLU epilogue on cfg 12 / 50;
#   p = plain projection forwards (o, down, lm_head) on the persistent cfg 50 as well
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_ab_$n.log 2>&1 || { tail -20 gpurun_out/r3_ab_$n.log; exit 1; }
  echo "$n: $(grep '"metric"' gpurun_out/r3_ab_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["final_loss"])')"
}
for r in 1 2; do
  run base_$r SFTAMD_GATE_UP=blas
  run gu12_$r SFTAMD_GATE_UP=12
  run gu50_$r SFTAMD_GATE_UP=50
  run gu12p_$r SFTAMD_GATE_UP=12 SFTAMD_FWD_GEMM=persist
done
