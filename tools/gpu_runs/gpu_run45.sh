#!/bin/bash
# Full GPU test suite on the rebuilt extension (BK64 config generalised over 4/8 waves), a smoke step on the
# device-assert debug build (_C_debug.so), the per-step ATen copy/fill audit, and a default bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t45.log 2>&1 || { tail -30 gpurun_out/t45.log; exit 1; }
tail -3 gpurun_out/t45.log
SFTAMD_DEBUG=1 timeout -k 10 300 python -c "import __graft_entry__ as g, torch; g.smoke(); from llm_fine_tune_distributed_amd.ops import _ext; print('lib', _ext.lib_path())" > gpurun_out/dbg45.log 2>&1 || { tail -30 gpurun_out/dbg45.log; exit 1; }
tail -2 gpurun_out/dbg45.log
timeout -k 10 300 python tools/copy_audit.py > gpurun_out/copy_audit45.txt 2>&1 || { tail -30 gpurun_out/copy_audit45.txt; exit 1; }
head -3 gpurun_out/copy_audit45.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/b45.log 2>&1 || { tail -20 gpurun_out/b45.log; exit 1; }
grep metric gpurun_out/b45.log
