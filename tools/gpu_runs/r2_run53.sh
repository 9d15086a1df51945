#!/bin/bash
# Peer-memory all-reduce latency, two ranks sharing one GPU (baseline: gloo).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python tools/bench_ipc_allreduce.py --world 2 > gpurun_out/r2_53_ipc.log 2>&1 || { tail -30 gpurun_out/r2_53_ipc.log; exit 1; }
grep bytes gpurun_out/r2_53_ipc.log
