#!/bin/bash
# parked norm-slot fix: 4-wave tests, recipe grad norms (default vs the no-hybrid reference), bench x2, full recipe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_4w_gpu.py tests/test_default_path_gpu.py > gpurun_out/r3_27_test.log 2>&1 || { tail -30 gpurun_out/r3_27_test.log; exit 1; }
tail -2 gpurun_out/r3_27_test.log
rec() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --recipe --steps 12 --warmup 0 --eval-steps 1000 > gpurun_out/r3_27_$n.log 2>&1 || { tail -20 gpurun_out/r3_27_$n.log; exit 1; }
  echo "$n: $(grep '^\[step' gpurun_out/r3_27_$n.log | grep -o 'grad_norm=[^,]*' | tr '\n' ' ')"
}
rec default
rec nohybrid SFTAMD_WGRAD_HYBRID=0
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_27_bench$r.log 2>&1 || { tail -20 gpurun_out/r3_27_bench$r.log; exit 1; }
grep '"metric"' gpurun_out/r3_27_bench$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], d["final_loss"])'
done
timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r3_27_rec.log 2>&1 || { tail -20 gpurun_out/r3_27_rec.log; exit 1; }
grep '"metric"' gpurun_out/r3_27_rec.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rec", d["value"], d["train_pure_samples_per_second"], d["train_tokens_per_second"], d["eval_runtime_s"], d["final_eval_loss"])'
