#!/bin/bash
# same-box A/B of the attention work: round-2 attention schedule (LEGWAIT=1, register staging) vs the default
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_42_$n.log 2>&1 || { tail -20 gpurun_out/r3_42_$n.log; exit 1; }
  echo "$n: $(grep '"metric"' gpurun_out/r3_42_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
}
for r in 1 2; do
  run old_$r SFTAMD_ATTN_LEGWAIT=1 SFTAMD_ATTN_FWD_DMA=0 SFTAMD_ATTN_BWD_DMA=0
  run new_$r X=1
done
