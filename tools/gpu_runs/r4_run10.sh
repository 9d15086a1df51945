#!/bin/bash
# r4_run08 (persistent GEMMs vs the overlapped AdamW) + r4_run09 (LoRA baseline profile) in one call
cd $GRAFT_REPO_ROOT
bash tools/gpu_runs/r4_run08.sh && bash tools/gpu_runs/r4_run09.sh
