#!/bin/bash
# Full GPU suite, headline bench, rocprofv3 kernel trace of the current default path.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t51.log 2>&1 || { tail -30 gpurun_out/t51.log; exit 1; }
tail -2 gpurun_out/t51.log
timeout -k 10 300 python bench.py > gpurun_out/b51.log 2>&1 || { tail -20 gpurun_out/b51.log; exit 1; }
grep metric gpurun_out/b51.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof51 -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/p51.log 2>&1 || { tail -20 gpurun_out/p51.log; exit 1; }
ls gpurun_out/prof51 | head
