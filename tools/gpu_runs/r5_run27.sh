#!/bin/bash
# power-of-two row pitch: the same GEMMs with padded operand pitches; then the Llama-3-8B kernel table (r5_run25)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_ld.py > gpurun_out/r5_27_ld.log 2>&1 || { tail -20 gpurun_out/r5_27_ld.log; exit 1; }
grep -v "amdgpu.ids\|TunableOp" gpurun_out/r5_27_ld.log
bash tools/gpu_runs/r5_run25.sh
