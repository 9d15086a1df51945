#!/bin/bash
# Round 2: model/trainer GPU tests on the new MLP backward + same-box A/B of the fused path.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_09_tests.log 2>&1 || { tail -40 gpurun_out/r2_09_tests.log; exit 1; }
tail -1 gpurun_out/r2_09_tests.log
b() { timeout -k 10 300 env "$@" python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1; }
for r in 1 2; do
  echo "new $(b SFTAMD_X=1)"
  echo "no_fused_down $(b SFTAMD_SWIGLU_DOWN=0)"
  echo "dgrad_blas $(b SFTAMD_DGRAD=blas SFTAMD_SWIGLU_DOWN=0)"
done
