#!/bin/bash
# routing update (down wgrad hybrid 1213, fused norm slots for the 4-wave wgrads): default-path + trainer tests, bench x2, recipe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_default_path_gpu.py tests/test_trainer_gpu.py > gpurun_out/r3_25_test.log 2>&1 || { tail -30 gpurun_out/r3_25_test.log; exit 1; }
tail -2 gpurun_out/r3_25_test.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_25_bench$r.log 2>&1 || { tail -20 gpurun_out/r3_25_bench$r.log; exit 1; }
grep '"metric"' gpurun_out/r3_25_bench$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"])'
done
timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r3_25_rec.log 2>&1 || { tail -20 gpurun_out/r3_25_rec.log; exit 1; }
grep '"metric"' gpurun_out/r3_25_rec.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rec", d["value"], d["train_pure_samples_per_second"], d["train_tokens_per_second"], d["eval_runtime_s"], d["final_eval_loss"])'
