#!/bin/bash
# round 6 session 2 baseline: full GPU suite + smoke + headline bench; kernel table + PMC of the step (cfg 14 ring)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6_03_tests.log 2>&1 || { tail -40 gpurun_out/r6_03_tests.log; exit 1; }
tail -2 gpurun_out/r6_03_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_03_smoke.log 2>&1 || { tail -20 gpurun_out/r6_03_smoke.log; exit 1; }
tail -1 gpurun_out/r6_03_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r6_03_bench.log 2>&1 || { tail -20 gpurun_out/r6_03_bench.log; exit 1; }
grep '"metric"' gpurun_out/r6_03_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof03 -o run -- python bench.py --steps 6 --warmup 2 > gpurun_out/r6_03_ps.log 2>&1 || { tail -20 gpurun_out/r6_03_ps.log; exit 1; }
db=$(ls /tmp/prof03/*/run_results.db /tmp/prof03/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $db --top 45 --out gpurun_out/r6_03_step_prof.md > /dev/null
head -40 gpurun_out/r6_03_step_prof.md
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc03a -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r6_03_pmca.log 2>&1 || { tail -20 gpurun_out/r6_03_pmca.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc03b -o run -- python bench.py --steps 2 --warmup 1 > gpurun_out/r6_03_pmcb.log 2>&1 || { tail -20 gpurun_out/r6_03_pmcb.log; exit 1; }
python tools/pmc_step.py /tmp/pmc03a /tmp/pmc03b --out gpurun_out/r6_03_step_pmc.md > /dev/null
head -40 gpurun_out/r6_03_step_pmc.md
