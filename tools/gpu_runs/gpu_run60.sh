#!/bin/bash
# Final same-box A/B (current default vs session-start commit) + rocprofv3 kernel trace of the default path.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/b60.log
for r in 1 2; do
  for t in new base; do
    if [ $t = new ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/_ab_base; fi
    v=$(cd $d && timeout -k 10 300 python bench.py 2>&1 | grep metric) || exit 1
    echo "$t $v" >> gpurun_out/b60.log
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/b60.log"):
    t, j = l.split(" ", 1)
    print(t, json.loads(j)["value"])
PY
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof60 -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/p60.log 2>&1 || { tail -20 gpurun_out/p60.log; exit 1; }
grep metric gpurun_out/p60.log | head -c 300
