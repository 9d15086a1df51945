#!/bin/bash
# final sanity of the in-tree extension: smoke() and the 4-wave / kernel / default-path GPU tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3_52_smoke.log 2>&1 || { tail -20 gpurun_out/r3_52_smoke.log; exit 1; }
tail -1 gpurun_out/r3_52_smoke.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_kernels_gpu.py tests/test_default_path_gpu.py \
  > gpurun_out/r3_52_test.log 2>&1 || { tail -40 gpurun_out/r3_52_test.log; exit 1; }
tail -1 gpurun_out/r3_52_test.log
