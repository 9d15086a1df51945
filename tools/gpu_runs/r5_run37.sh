#!/bin/bash
# recipe + headline: 4-wave read order (current) vs the previous one (SFTAMD_G4_OLD=1, temporary), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1 0 1; do
  SFTAMD_G4_OLD=$v timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r5_37_recipe$v.log 2>&1 || { tail -20 gpurun_out/r5_37_recipe$v.log; exit 1; }
  echo "recipe old=$v $(grep '"metric"' gpurun_out/r5_37_recipe$v.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r.get("train_pure_samples_per_second",""), r.get("final_loss", ""))')"
  SFTAMD_G4_OLD=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_37_bench$v.log 2>&1 || { tail -20 gpurun_out/r5_37_bench$v.log; exit 1; }
  echo "bench old=$v $(grep -o '"value": [0-9.]*\|"final_loss": [a-zA-Z0-9.]*' gpurun_out/r5_37_bench$v.log | tr '\n' ' ')"
done
