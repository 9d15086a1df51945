#!/bin/bash
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SFTAMD_ATTN_IMPL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11a -o run -- python3 tools/bench_attention.py > gpurun_out/p11a.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/p11a.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11b -o run -- python3 bench.py --steps 3 --warmup 2 --no-overlap > gpurun_out/p11b.log 2>&1; echo "rc=$?" >> gpurun_out/p11b.log
