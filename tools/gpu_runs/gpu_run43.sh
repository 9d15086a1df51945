#!/bin/bash
# Rehearse bench.py's multi-rank path (torchrun, ZeRO-1 reduce-scatter/all-gather, timing MAX-reduce,
# JSON line) with 2 ranks sharing the single GPU over gloo — numbers meaningless, control flow real.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SFTAMD_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/b43_2rank.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/b43_2rank.log
