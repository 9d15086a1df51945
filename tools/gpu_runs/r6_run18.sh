#!/bin/bash
# round 6: cross-entropy occupancy cap (dynamic LDS per block) so the second pass re-reads rows from the Infinity Cache
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
for kb in 0 24 32 40 54 80; do
SFTAMD_CE_LDS_KB=$kb timeout -k 10 120 python -u tools/bench_ce.py > gpurun_out/r6_18_ce_$kb.log 2>&1 || { tail -20 gpurun_out/r6_18_ce_$kb.log; exit 1; }
echo "lds $kb KB: $(tail -1 gpurun_out/r6_18_ce_$kb.log)"
done; done
