#!/bin/bash
# (1) recipe (reference parquet, 8 x GA 2 merged, evals every 10 steps): hipBLASLt forwards vs the persistent HIP
#     forward GEMM for the ragged-M projections; (2) chunked LM head + CE at the bench shape: peak memory / samples/s
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
rec() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r3_19_rec_$n.log 2>&1 || { tail -20 gpurun_out/r3_19_rec_$n.log; exit 1; }
  echo "rec $n: $(grep '"metric"' gpurun_out/r3_19_rec_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["train_pure_samples_per_second"], d["train_tokens_per_second"], d["eval_runtime_s"], d["peak_mem_gb"])')"
}
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r3_19_$n.log 2>&1 || { tail -20 gpurun_out/r3_19_$n.log; exit 1; }
  echo "$n: $(grep '"metric"' gpurun_out/r3_19_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["final_loss"])')"
}
rec base
rec persist SFTAMD_FWD_GEMM=persist SFTAMD_GATE_UP=50
run base
run chunk1k --lm-head-chunk 1024
run chunk2k --lm-head-chunk 2048
run base2
