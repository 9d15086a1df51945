#!/bin/bash
# round 6: where the 4-wave ring's cycles go (gate_up wgrad at T = 8192): cfg 14 vs the timing-only diagnostics 17 (no
# DMA in the loop) / 18 (no K-step barrier); wall time interleaved, then SQ wait / issue counters
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r6_06_ab.log
timeout -k 10 300 python -u tools/bench_ab.py wgrad gate_up,lm_head 14,17,18 --rounds 5 > $L 2>&1 || { tail -30 $L; exit 1; }
cat $L
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d /tmp/pmc06 -o run -- python3 tools/bench_ab.py wgrad gate_up 14,17,18 --rounds 1 --iters 2 > gpurun_out/r6_06_pmc.log 2>&1 || { tail -20 gpurun_out/r6_06_pmc.log; exit 1; }
python tools/pmc_csv.py $(find /tmp/pmc06 -name "*counter_collection.csv") --match "g4_kernel<1, 1, 0, 4>,g4_kernel<1, 1, 0, 8>,g4_kernel<1, 1, 0, 12>" | tee gpurun_out/r6_06_pmc.txt
