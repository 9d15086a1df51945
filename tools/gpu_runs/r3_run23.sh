#!/bin/bash
# dgrad hybrid split-K for partial rounds: tests, M = 10240 microbench (split on / off), recipe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_4w_gpu.py > gpurun_out/r3_23_test.log 2>&1 || { tail -30 gpurun_out/r3_23_test.log; exit 1; }
tail -2 gpurun_out/r3_23_test.log
DGRAD_CFGS=12,13 timeout -k 10 300 python -u tools/bench_dgrad.py --tokens 10240 > gpurun_out/r3_23_dg.log 2>&1 || { tail -20 gpurun_out/r3_23_dg.log; exit 1; }
grep '^{' gpurun_out/r3_23_dg.log
SFTAMD_DGRAD_SPLITK=0 DGRAD_CFGS=12,13 timeout -k 10 300 python -u tools/bench_dgrad.py --tokens 10240 > gpurun_out/r3_23_dg0.log 2>&1 || { tail -20 gpurun_out/r3_23_dg0.log; exit 1; }
grep '^{' gpurun_out/r3_23_dg0.log
DGRAD_SHAPES=lm_head DGRAD_CFGS=13 timeout -k 10 300 python -u tools/bench_dgrad.py --tokens 10240 > gpurun_out/r3_23_dg2.log 2>&1 || { tail -20 gpurun_out/r3_23_dg2.log; exit 1; }
grep '^{' gpurun_out/r3_23_dg2.log
timeout -k 10 400 python -u bench.py --recipe --steps 40 --warmup 0 > gpurun_out/r3_23_rec.log 2>&1 || { tail -20 gpurun_out/r3_23_rec.log; exit 1; }
grep '"metric"' gpurun_out/r3_23_rec.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("rec", d["value"], d["train_pure_samples_per_second"], d["train_tokens_per_second"], d["eval_runtime_s"], d["final_eval_loss"])'
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_23_bench.log 2>&1 || { tail -20 gpurun_out/r3_23_bench.log; exit 1; }
grep '"metric"' gpurun_out/r3_23_bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"])'
