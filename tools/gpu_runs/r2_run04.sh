#!/bin/bash
# Round 2: full GPU tests, bench variants (bf16 vs fp32 moments, 8xGA2 merged vs two passes), profile of the default.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_04_tests.log 2>&1 || { tail -40 gpurun_out/r2_04_tests.log; exit 1; }
tail -2 gpurun_out/r2_04_tests.log
: > gpurun_out/r2_04_bench.jsonl
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/r2_04_$tag.log 2>&1 || { tail -20 gpurun_out/r2_04_$tag.log; exit 1; }
  grep metric gpurun_out/r2_04_$tag.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); r['tag']='$tag'; print(json.dumps(r))" >> gpurun_out/r2_04_bench.jsonl
  tail -1 gpurun_out/r2_04_bench.jsonl | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['tag'], r['value'], r['ms_per_step'], r['peak_mem_gb'])"
}
run default
run fp32_moments --optim-state fp32
run ga2_merged --micro-batch 8 --ga 2
run ga2_two_passes --micro-batch 8 --ga 2 --ga-merge-max-tokens 0
run default_again
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2_04 -o run -- python bench.py --steps 4 --warmup 2 > gpurun_out/r2_04_p.log 2>&1 || { tail -20 gpurun_out/r2_04_p.log; exit 1; }
echo done
