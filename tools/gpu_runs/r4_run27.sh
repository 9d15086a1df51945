#!/bin/bash
# TunableOp selections for the LoRA bench's hipBLASLt/rocBLAS shapes (dxa = s dy B_blockdiag, the small adapter GEMMs)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 bash tools/tune_gemms.sh gpurun_out/tune_lora.csv --freeze-policy lora > gpurun_out/r4_27_tune.log 2>&1 || { tail -20 gpurun_out/r4_27_tune.log; exit 1; }
tail -3 gpurun_out/r4_27_tune.log
ls gpurun_out/tune_lora*.csv
