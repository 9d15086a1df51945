#!/bin/bash
# round 6: the four-problem grid's 168 leftover tiles unsplit (default now) vs split 3 ways (SFTAMD_MULTI_SPLIT=3)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_default_path_gpu.py -m gpu > gpurun_out/r6_73_tests.log 2>&1 || { tail -40 gpurun_out/r6_73_tests.log; exit 1; }
tail -1 gpurun_out/r6_73_tests.log
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2 3; do
for s in d 3; do
if [ $s = d ]; then e=""; else e=3; fi
SFTAMD_MULTI_SPLIT=$e timeout -k 10 300 python -u bench.py --steps 20 > gpurun_out/r6_73_${s}_$i.log 2>&1 || { tail -20 gpurun_out/r6_73_${s}_$i.log; exit 1; }
echo "split=$s $i: $(v gpurun_out/r6_73_${s}_$i.log)"
done
done
