#!/bin/bash
# round 6: SwiGLU forward walking its input from the end (Infinity Cache residency of the gate_up output), micro + step
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r6_36.log; : > $out
for r in 0 1 0 1; do
  SFTAMD_SWIGLU_REV=$r timeout -k 10 120 python -u tools/bench_after_producer.py 2>&1 | grep rev >> $out || { echo fail; exit 1; }
done
for r in 1 0 1 0; do
  SFTAMD_SWIGLU_REV=$r timeout -k 10 300 python bench.py --steps 20 > gpurun_out/r6_36_b.log 2>&1 || { tail -20 gpurun_out/r6_36_b.log; exit 1; }
  echo "rev=$r $(tail -1 gpurun_out/r6_36_b.log | cut -c60-140)" >> $out
done
cat $out
