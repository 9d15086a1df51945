#!/bin/bash
# Full-size 2-rank rehearsal on ONE GPU over gloo (RCCL refuses two ranks on one device): SmolLM3-3B, ZeRO-1 with the
# sparse tied-embedding exchange, then DDP; checks the N = 2 code path end to end at real sizes (numbers are not
# throughput evidence: gloo stages every collective through the host).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export SFTAMD_DIST_BACKEND=gloo
timeout -k 10 600 python bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/r2_49_zero.log 2>&1 || { tail -30 gpurun_out/r2_49_zero.log; exit 1; }
tail -1 gpurun_out/r2_49_zero.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print({k: r[k] for k in ("value","final_loss","optimizer_sharding","bucket_plan","comm_probe","dist")})'
timeout -k 10 600 python bench.py --gpus 2 --steps 2 --warmup 1 --zero 0 > gpurun_out/r2_49_ddp.log 2>&1 || { tail -30 gpurun_out/r2_49_ddp.log; exit 1; }
tail -1 gpurun_out/r2_49_ddp.log | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print({k: r[k] for k in ("value","final_loss","optimizer_sharding","bucket_plan")})'
