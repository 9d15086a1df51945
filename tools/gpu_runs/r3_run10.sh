#!/bin/bash
# attention forward v6 (GQA-stacked, glds K/V): correctness, then fwd/bwd timing vs v3 at B 16 x 512 and a kernel
# profile of the two forwards
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "fwd6 or bwd6 or flash_bwd_rope or flash_attention_smollm3 or deferred_rescale" \
  > gpurun_out/r3_10_test.log 2>&1 || { tail -40 gpurun_out/r3_10_test.log; exit 1; }
tail -2 gpurun_out/r3_10_test.log
B=16 ATTN_FWD=1 timeout -k 10 200 python -u tools/bench_attention.py > gpurun_out/r3_10_bench.log 2>&1 || { tail -30 gpurun_out/r3_10_bench.log; exit 1; }
cat gpurun_out/r3_10_bench.log
cd /tmp && B=16 ATTN_FWD=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3_10_prof -o prof -- python -u $GRAFT_REPO_ROOT/tools/bench_attention.py > $GRAFT_REPO_ROOT/gpurun_out/r3_10_prof.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/r3_10_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/r3_10_prof -name "*.db" -o -name "*kernel_stats.csv" | sort | tail -1)
python tools/prof_summary.py "$f" --top 25 --out gpurun_out/r3_10_prof.md > /dev/null && cat gpurun_out/r3_10_prof.md
