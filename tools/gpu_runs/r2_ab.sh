#!/bin/bash
# Same-box interleaved A/B: this tree ("new") vs the _ab_base worktree ("base"), default bench, R rounds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=${R:-2}
for r in $(seq $R); do
  for t in new base; do
    if [ $t = new ]; then d=$GRAFT_REPO_ROOT; else d=$GRAFT_REPO_ROOT/_ab_base; fi
    v=$(cd $d && timeout -k 10 300 python bench.py --steps 20 --warmup 5 $BENCH_ARGS 2>&1 | grep -o '"value": [0-9.]*') || exit 1
    echo "$t $v"
  done
done
