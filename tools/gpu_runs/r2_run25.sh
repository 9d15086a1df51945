#!/bin/bash
# Ping-pong TN GEMM: cost of the epilogue stores (cfg 99 = cfg 11 without them) over a K sweep.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_gemm_tn.py --cfgs 11,99 --plain-only --shapes gu1k:22016:1024,gu2k:22016:2048,gu4k:22016:4096,gate_up:22016:2048,down:2048:11008 2>&1 | tee gpurun_out/r2_25.md
