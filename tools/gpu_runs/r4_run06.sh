#!/bin/bash
# forward GEMMs on the persistent kernel (nt stores + K stagger) end to end: interleaved A/B on one box
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 50,164 --plain-only > gpurun_out/r4_06_gemm8k.log 2>&1 || { tail -20 gpurun_out/r4_06_gemm8k.log; exit 1; }
cat gpurun_out/r4_06_gemm8k.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --fused-cfgs 50,164 > gpurun_out/r4_06_fused.log 2>&1 || { tail -20 gpurun_out/r4_06_fused.log; exit 1; }
cat gpurun_out/r4_06_fused.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_06_base$r.log 2>&1 || { tail -20 gpurun_out/r4_06_base$r.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/r4_06_base$r.log | sed "s/^/base $r /"
  SFTAMD_FWD_GEMM=persist timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_06_fwd$r.log 2>&1 || { tail -20 gpurun_out/r4_06_fwd$r.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/r4_06_fwd$r.log | sed "s/^/persist $r /"
  SFTAMD_FWD_GEMM=persist SFTAMD_GATE_UP=50 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_06_gu$r.log 2>&1 || { tail -20 gpurun_out/r4_06_gu$r.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/r4_06_gu$r.log | sed "s/^/persist+gu50 $r /"
done
