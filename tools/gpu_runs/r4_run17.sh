#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "varlen_gqa" > gpurun_out/r4_17_attn.log 2>&1; grep -E "passed|failed|Error:" gpurun_out/r4_17_attn.log | head -40
