#!/bin/bash
# round 6: localise the cfg 14 (interleaved 4-wave ring) error
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/debug/g4_il_diag.py 2>&1 | tee gpurun_out/r6_02_diag.log
