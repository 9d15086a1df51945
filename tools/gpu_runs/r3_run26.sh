#!/bin/bash
# bisect the NaN of r3_run25: recipe 12 steps (no eval) with the 4-wave wgrad norm slots / down hybrid toggled
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rec() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --recipe --steps 12 --warmup 0 --eval-steps 1000 > gpurun_out/r3_26_$n.log 2>&1 || { tail -20 gpurun_out/r3_26_$n.log; exit 1; }
  echo "$n: $(grep '^\[step' gpurun_out/r3_26_$n.log | grep -o 'grad_norm=[^,]*' | tr '\n' ' ')"
}
rec default
rec nonorm SFTAMD_NORM_4W=0
rec nohybrid SFTAMD_WGRAD_HYBRID=0
rec neither SFTAMD_NORM_4W=0 SFTAMD_WGRAD_HYBRID=0
