#!/bin/bash
# default-path test with the 4-wave backward routing, then an interleaved end-to-end A/B:
#   old = 8-wave wgrad rings + cfg 7 dgrads + hipBLASLt gate_up / lm_head dgrads; new = defaults (4-wave routing)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_default_path_gpu.py tests/test_gemm_4w_gpu.py \
  > gpurun_out/r3_16_test.log 2>&1 || { tail -40 gpurun_out/r3_16_test.log; exit 1; }
tail -2 gpurun_out/r3_16_test.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_ab_$n.log 2>&1 || { tail -20 gpurun_out/r3_ab_$n.log; exit 1; }
  echo "$n: $(grep '"metric"' gpurun_out/r3_ab_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["final_loss"])')"
}
for r in 1 2; do
  run old_$r SFTAMD_WGRAD_4W=0 SFTAMD_DGRAD_4W=0
  run new_$r
  run wg_$r SFTAMD_DGRAD_4W=0
  run dg_$r SFTAMD_WGRAD_4W=0
done
