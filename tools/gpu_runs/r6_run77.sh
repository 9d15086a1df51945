#!/bin/bash
# round 6: nontemporal gate / up loads in the SwiGLU-backward dgrad epilogue — tests, step vs the previous build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_default_path_gpu.py -m gpu > gpurun_out/r6_77_tests.log 2>&1 || { tail -40 gpurun_out/r6_77_tests.log; exit 1; }
tail -1 gpurun_out/r6_77_tests.log
v() { grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [0-9.]*' $1 | tr '\n' ' '; echo; }
for i in 1 2 3; do
for lib in new old; do
l=llm_fine_tune_distributed_amd/_C.so; [ $lib = old ] && l=llm_fine_tune_distributed_amd/_C_ab_old.so
SFTAMD_LIB=$l timeout -k 10 300 python -u bench.py --steps 20 > gpurun_out/r6_77_${lib}_$i.log 2>&1 || { tail -20 gpurun_out/r6_77_${lib}_$i.log; exit 1; }
echo "$lib $i: $(v gpurun_out/r6_77_${lib}_$i.log)"
done
done
