#!/bin/bash
# Validation after moving the ZeRO-1 update + gathers to a side stream (overlapped with the next forward):
# 2-rank ZeRO-1 bench path (gloo, both ranks on the one GPU) that exercises the in-flight count.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t62.log 2>&1 || { tail -30 gpurun_out/t62.log; exit 1; }
tail -2 gpurun_out/t62.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s62.log 2>&1 || { tail -20 gpurun_out/s62.log; exit 1; }
tail -1 gpurun_out/s62.log
SFTAMD_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/b62_2rank.log 2>&1 || { tail -20 gpurun_out/b62_2rank.log; exit 1; }
grep metric gpurun_out/b62_2rank.log
