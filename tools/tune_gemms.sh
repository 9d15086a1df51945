#!/bin/bash
# Tune hipBLASLt/rocBLAS selections (PyTorch TunableOp) for the GEMM shapes of one bench config and merge
# them into a copy of the shipped selection file. Run on an MI355X box:
#     bash tools/tune_gemms.sh OUT.csv [bench.py args ...]
# TunableOp appends the device ordinal to the file name (OUT0.csv); copy that over
# tuning/tunableop_results_mi355x.csv after checking it.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/tune.csv}
shift || true
cp tuning/tunableop_results_mi355x.csv "$OUT"
# tuning one shape can take minutes without output: a heartbeat line every 60 s keeps the run visibly alive
( while sleep 60; do echo "[tune_gemms] still tuning $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME="$OUT" \
    python bench.py --steps 2 --warmup 1 --tunableop off "$@"
