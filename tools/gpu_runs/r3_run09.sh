#!/bin/bash
# persistent cfg 50 with the next tile's K0 + K1 issued before the epilogue stores (first boundary waits only for
# K1): correctness, GEMM timing vs hipBLASLt / cfg 12, fused epilogues, then one round of the end-to-end A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn_4wave" \
  > gpurun_out/r3_09_test.log 2>&1 || { tail -40 gpurun_out/r3_09_test.log; exit 1; }
tail -2 gpurun_out/r3_09_test.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --cfgs 12,50 --plain-only --iters 30 \
  --shapes gate_up:22016:2048,lm_head:128256:2048,down:2048:11008,o:2048:2048,qkv:3072:2048,gu1k:22016:1024,gu4k:22016:4096 > gpurun_out/r3_09.log 2>&1 || { tail -30 gpurun_out/r3_09.log; exit 1; }
cat gpurun_out/r3_09.log
timeout -k 10 200 python -u tools/bench_gemm_tn.py --fused-cfgs 11,12,50 --iters 30 > gpurun_out/r3_09f.log 2>&1 || { tail -30 gpurun_out/r3_09f.log; exit 1; }
cat gpurun_out/r3_09f.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_ab_$n.log 2>&1 || { tail -20 gpurun_out/r3_ab_$n.log; exit 1; }
  echo "$n: $(grep '"metric"' gpurun_out/r3_ab_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["final_loss"])')"
}
run base SFTAMD_GATE_UP=blas
run gu12 SFTAMD_GATE_UP=12
run gu50 SFTAMD_GATE_UP=50
run gu12p SFTAMD_GATE_UP=12 SFTAMD_FWD_GEMM=persist
