#!/usr/bin/env python3
"""RCCL (xGMI) bucket all-reduce sweep: bus bandwidth vs bucket size.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py

busbw = algbw * 2 (N-1) / N (nccl-tests convention). Use it to pick ddp_bucket_cap_mb: the
smallest size whose busbw is within ~10% of the plateau keeps per-call latency amortised while
still letting the first buckets start early in backward.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from llm_fine_tune_distributed_amd.parallel.process_group import setup_distributed  # noqa: E402


def main():
    st = setup_distributed(verbose=False)
    n = st.world_size
    sizes_mb = [1, 4, 16, 32, 64, 128, 256, 512]
    res = []
    for mb in sizes_mb:
        x = torch.ones(mb * 1024 * 1024 // 2, dtype=torch.bfloat16, device=st.device)
        for _ in range(3):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        iters = max(5, min(50, 2000 // mb))
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        alg = mb * 2**20 / dt / 1e9
        res.append({"size_mb": mb, "us": round(dt * 1e6, 1), "algbw_GBs": round(alg, 1),
                    "busbw_GBs": round(alg * 2 * (n - 1) / n, 1)})
    if st.is_main:
        print(json.dumps({"world_size": n, "dtype": "bf16", "results": res}, indent=1))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
