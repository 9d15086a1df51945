#!/bin/bash
# Round 2: kernel trace of the default step (fused down dgrad) and of SFTAMD_SWIGLU_DOWN=0 SFTAMD_DGRAD=blas.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in a b; do
  if [ $v = b ]; then export SFTAMD_SWIGLU_DOWN=0 SFTAMD_DGRAD=blas; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_r2_10$v -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/r2_10$v.log 2>&1 || { tail -20 gpurun_out/r2_10$v.log; exit 1; }
  python tools/prof_summary.py $(find /tmp/prof_r2_10$v -name "*.db" | head -1) --top 40 > gpurun_out/r2_10$v.md
done
echo ok
