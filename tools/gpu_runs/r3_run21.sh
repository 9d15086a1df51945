#!/bin/bash
# padding-free default: trainer GPU tests; recipe pf on / off (+ persistent forward GEMMs); bench pf auto / off
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_trainer_gpu.py > gpurun_out/r3_21_test.log 2>&1 || { tail -30 gpurun_out/r3_21_test.log; exit 1; }
tail -2 gpurun_out/r3_21_test.log
rec() {  # name, env / args...
  local n=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 $RA > gpurun_out/r3_21_rec_$n.log 2>&1 || { tail -20 gpurun_out/r3_21_rec_$n.log; exit 1; }
  echo "rec $n: $(grep '"metric"' gpurun_out/r3_21_rec_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["train_pure_samples_per_second"], d["train_tokens_per_second"], d["eval_runtime_s"], d["final_eval_loss"], d["peak_mem_gb"])')"
}
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r3_21_$n.log 2>&1 || { tail -20 gpurun_out/r3_21_$n.log; exit 1; }
  echo "$n: $(grep '"metric"' gpurun_out/r3_21_$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"], d["final_loss"])')"
}
RA="--padding-free off" rec pad
rec pf
rec pf_persist SFTAMD_FWD_GEMM=persist SFTAMD_GATE_UP=50
run auto
run off --padding-free off
