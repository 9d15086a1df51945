#!/bin/bash
# round 5: dgrad cfg 8 (4-wave 256 x 128 workgroups, two per CU) for the SwiGLU-backward down dgrad
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "dgrad" > gpurun_out/r5_12_tests.log 2>&1 || { tail -30 gpurun_out/r5_12_tests.log; exit 1; }
tail -1 gpurun_out/r5_12_tests.log
DGRAD_CFGS=7,8,2 timeout -k 10 300 python -u tools/bench_dgrad.py --rounds 3 > gpurun_out/r5_12_dgrad.log 2>&1 || { tail -20 gpurun_out/r5_12_dgrad.log; exit 1; }
grep -v TunableOp gpurun_out/r5_12_dgrad.log | cut -c1-300
