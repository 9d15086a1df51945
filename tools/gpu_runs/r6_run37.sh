#!/bin/bash
# round 6: end-of-session kernel tables: headline step and LoRA step (rocprofv3 kernel trace)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof37 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r6_37_ps.log 2>&1 || { tail -20 gpurun_out/r6_37_ps.log; exit 1; }
db=$(ls /tmp/prof37/*/run_results.db /tmp/prof37/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 50 --out gpurun_out/r6_37_step_prof.md > /dev/null
python tools/prof_timeline.py $db > gpurun_out/r6_37_timeline.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof37l -o run -- python bench.py --freeze-policy lora --steps 6 --warmup 2 > gpurun_out/r6_37_psl.log 2>&1 || { tail -20 gpurun_out/r6_37_psl.log; exit 1; }
db=$(ls /tmp/prof37l/*/run_results.db /tmp/prof37l/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 50 --out gpurun_out/r6_37_lora_prof.md > /dev/null
head -30 gpurun_out/r6_37_step_prof.md
head -30 gpurun_out/r6_37_lora_prof.md
