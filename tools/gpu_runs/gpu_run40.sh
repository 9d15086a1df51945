#!/bin/bash
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/attn_ablate.py > gpurun_out/ab40.log 2>&1; echo "rc=$?" >> gpurun_out/ab40.log
