#!/bin/bash
# fused gate_up + SwiGLU (cfg 50) vs hipBLASLt + SwiGLU kernel, with / without the AdamW-under-forward overlap
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env..., -- args
  local n=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r3_30_$n.log 2>&1 || { tail -20 gpurun_out/r3_30_$n.log; exit 1; }
  echo "$n: $(grep '"metric"' gpurun_out/r3_30_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
}
for r in 1 2; do
  run base_$r X=1 --
  run noov_$r X=1 -- --no-overlap
  run gu50_$r SFTAMD_GATE_UP=50 --
  run gu50noov_$r SFTAMD_GATE_UP=50 -- --no-overlap
done
