#!/bin/bash
# Validation after the async token-count change: GPU test suite, smoke(), 1-GPU bench, and the
# 2-rank ZeRO-1 bench path (gloo, both ranks on the one GPU) that exercises the in-flight count.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t61.log 2>&1 || { tail -30 gpurun_out/t61.log; exit 1; }
tail -2 gpurun_out/t61.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/s61.log 2>&1 || { tail -20 gpurun_out/s61.log; exit 1; }
tail -1 gpurun_out/s61.log
timeout -k 10 300 python bench.py > gpurun_out/b61.log 2>&1 || { tail -20 gpurun_out/b61.log; exit 1; }
grep metric gpurun_out/b61.log
SFTAMD_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/b61_2rank.log 2>&1 || { tail -20 gpurun_out/b61_2rank.log; exit 1; }
grep metric gpurun_out/b61_2rank.log
