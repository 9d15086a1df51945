#!/bin/bash
# Bisect today's changes by their knobs on one box (interleaved, 2 rounds), plus the session-start commit.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/b57.log
run() {  # name, dir, env...
  local name=$1 d=$2; shift 2
  v=$(cd $d && env "$@" timeout -k 10 300 python bench.py 2>&1 | grep metric) || return 1
  echo "$name $v" >> gpurun_out/b57.log
}
for r in 1 2; do
  run new $GRAFT_REPO_ROOT A=1 || exit 1
  run base $GRAFT_REPO_ROOT/_ab_base A=1 || exit 1
  run no_tn_plain $GRAFT_REPO_ROOT SFTAMD_TN_PLAIN=0 || exit 1
  run no_small_tiles $GRAFT_REPO_ROOT SFTAMD_TN_SMALL_TILES=0 || exit 1
  run adam_unr1 $GRAFT_REPO_ROOT SFTAMD_ADAM_UNR=1 || exit 1
  run swiglu_unr1 $GRAFT_REPO_ROOT SFTAMD_SWIGLU_UNR=1 || exit 1
done
python - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/b57.log"):
    t, j = l.split(" ", 1)
    d[t].append(json.loads(j)["value"])
for t, v in d.items():
    print(f"{t:16s} {v}  mean {sum(v)/len(v):.2f}")
PY
