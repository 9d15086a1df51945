#!/bin/bash
# tn5 variants (per-tile 51, dynamic tile queue 165): tests, microbench, end-to-end A/B against the overlapped AdamW;
# LoRA on the hand-written path (tests, bench, profile)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_tn_4wave or dynamic_queue or lora" > gpurun_out/r4_11_tests.log 2>&1 || { tail -30 gpurun_out/r4_11_tests.log; exit 1; }
tail -2 gpurun_out/r4_11_tests.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 51,164,165 --plain-only > gpurun_out/r4_11_plain.log 2>&1 || { tail -20 gpurun_out/r4_11_plain.log; exit 1; }
cat gpurun_out/r4_11_plain.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --fused-cfgs 51,164,165 > gpurun_out/r4_11_fused.log 2>&1 || { tail -20 gpurun_out/r4_11_fused.log; exit 1; }
cat gpurun_out/r4_11_fused.log
run() {  # tag, bench args...; env via BENV
  local tag=$1; shift
  env $BENV timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r4_11_$tag.log 2>&1 || { tail -20 gpurun_out/r4_11_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4_11_$tag.log)"
}
for r in 1 2; do
  BENV="SFTAMD_X=0" run base$r
  BENV="SFTAMD_GATE_UP=165 SFTAMD_FWD_GEMM=persist SFTAMD_PERSIST_CFG=165" run dyn$r
  BENV="SFTAMD_GATE_UP=51 SFTAMD_FWD_GEMM=persist SFTAMD_PERSIST_CFG=51" run tile$r
  BENV="SFTAMD_X=0" run base_noov$r --no-overlap
  BENV="SFTAMD_GATE_UP=164 SFTAMD_FWD_GEMM=persist SFTAMD_PERSIST_CFG=164" run pers_noov$r --no-overlap
done
bash tools/gpu_runs/r4_run09.sh
