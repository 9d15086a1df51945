#!/bin/bash
# r3_run07 (persistent 4-wave GEMM) + r3_run06 (default-path test, IPC, fused epilogues) in one box
cd $GRAFT_REPO_ROOT
bash tools/gpu_runs/r3_run07.sh && bash tools/gpu_runs/r3_run06.sh
