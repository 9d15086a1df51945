#!/bin/bash
# Same-box A/B of the headline bench: current tree vs the session-start commit (11e9e90, built in _ab_base/).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/b56.log
for r in 1 2 3; do
  for t in new base; do
    if [ $t = new ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/_ab_base; fi
    v=$(cd $d && timeout -k 10 300 python bench.py 2>&1 | grep metric) || exit 1
    echo "$t $v" >> gpurun_out/b56.log
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/b56.log"):
    t, j = l.split(" ", 1)
    print(t, json.loads(j)["value"])
PY
