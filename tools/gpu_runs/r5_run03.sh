#!/bin/bash
# round 5: default-path numerics report (SmolLM3 + Llama-3-8B widths; per-parameter gradient errors for the test
# bounds), then the end-to-end A/B of the row-contiguous forward GEMM routing (interleaved x2) + a step profile
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
DEFAULT_PATH_REPORT=$PWD/gpurun_out/r5_03_default_path.jsonl timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_default_path_gpu.py > gpurun_out/r5_03_tests.log 2>&1
tail -5 gpurun_out/r5_03_tests.log
bash tools/gpu_runs/r5_run02.sh
