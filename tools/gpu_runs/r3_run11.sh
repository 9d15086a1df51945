#!/bin/bash
# attention v6 forward (r3_run10), then the persistent GEMM + forward-routing A/B (r3_run09)
cd $GRAFT_REPO_ROOT
bash tools/gpu_runs/r3_run10.sh && bash tools/gpu_runs/r3_run09.sh
