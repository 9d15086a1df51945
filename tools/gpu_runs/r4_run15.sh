#!/bin/bash
# attention kernels after the buffer-descriptor DMA / V-image / AGPR-pinned dK-dV changes: tests, then A/B bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "attention or flash or attn" > gpurun_out/r4_15_attn.log 2>&1 || { tail -40 gpurun_out/r4_15_attn.log; exit 1; }
tail -2 gpurun_out/r4_15_attn.log
B=16 CFGS=ds,fwd16,dkdv5 timeout -k 10 300 python -u tools/bench_attention.py > gpurun_out/r4_15_bench.log 2>&1 || { tail -20 gpurun_out/r4_15_bench.log; exit 1; }
cat gpurun_out/r4_15_bench.log
