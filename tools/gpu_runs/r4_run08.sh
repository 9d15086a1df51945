#!/bin/bash
# persistent GEMMs vs the overlapped AdamW: one-tile-per-workgroup launches (cfg 51), and the no-overlap control
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --fused-cfgs 51,164 > gpurun_out/r4_08_fused.log 2>&1 || { tail -20 gpurun_out/r4_08_fused.log; exit 1; }
cat gpurun_out/r4_08_fused.log
timeout -k 10 300 python -u tools/bench_gemm_tn.py --m 8192 --cfgs 51,164 --plain-only > gpurun_out/r4_08_plain.log 2>&1 || { tail -20 gpurun_out/r4_08_plain.log; exit 1; }
cat gpurun_out/r4_08_plain.log
run() {  # tag, bench args..., then env via BENV
  local tag=$1; shift
  env $BENV timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r4_08_$tag.log 2>&1 || { tail -20 gpurun_out/r4_08_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/r4_08_$tag.log)"
}
for r in 1 2; do
  BENV="SFTAMD_X=0" run base$r
  BENV="SFTAMD_GATE_UP=51 SFTAMD_FWD_GEMM=persist SFTAMD_PERSIST_CFG=51" run tile$r
  BENV="SFTAMD_X=0" run base_noov$r --no-overlap
  BENV="SFTAMD_GATE_UP=164 SFTAMD_FWD_GEMM=persist SFTAMD_PERSIST_CFG=164" run pers_noov$r --no-overlap
done
