#!/bin/bash
# round 6: GPU busy / idle gaps over the timed steps of the headline bench (serial AdamW default)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof19 -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/r6_19_ps.log 2>&1 || { tail -20 gpurun_out/r6_19_ps.log; exit 1; }
grep '"metric"' gpurun_out/r6_19_ps.log | grep -o '"ms_per_step": [0-9.]*'
db=$(ls /tmp/prof19/*/run_results.db /tmp/prof19/run_results.db 2>/dev/null | head -1)
python - "$db" <<'PY' > gpurun_out/r6_19_window.txt
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
rows = c.execute("select start, end from kernels order by start").fetchall()
# the timed window: find the adamw kernels (one per step, serial) and take the span of the last 8 steps
names = c.execute(f"select {'kernel_name' if 'kernel_name' in cols else 'name'}, start, end from kernels order by start").fetchall()
ad = [s for n, s, e in names if "adamw_kernel" in n]
print("adamw launches", len(ad))
PY
python tools/prof_timeline.py $db --window-ms 1200 --out gpurun_out/r6_19_timeline.md > /dev/null
head -40 gpurun_out/r6_19_timeline.md
