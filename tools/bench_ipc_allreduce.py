"""Latency of the peer-memory one-shot all-reduce (csrc/ipc_allreduce.hip) vs the process group's all_reduce.

    python tools/bench_ipc_allreduce.py [--world 2]

Ranks go to GPU (rank % device_count): on one GPU both ranks share it (the process group is then gloo, which only
carries the handle exchange and the baseline); on a multi-GPU node every rank has its own GPU and the baseline is
RCCL over xGMI. Prints one JSON line per message size (median us over 200 calls, rank 0)."""
import argparse
import json
import os
import socket
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _worker(rank, world, port, sizes, iters):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(rank % ndev)
    backend = "nccl" if ndev >= world else "gloo"
    dist.init_process_group(backend, rank=rank, world_size=world)
    from llm_fine_tune_distributed_amd.parallel.ipc_allreduce import IPCAllReduce
    ar = IPCAllReduce(max_bytes=max(sizes))
    for nbytes in sizes:
        x = torch.ones(nbytes // 4, device="cuda")
        res = {}
        for name, fn in (("ipc", lambda: ar.all_reduce_(x)), (backend, lambda: dist.all_reduce(x))):
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            ts = []
            for _ in range(iters):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn()
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            res[f"{name}_us"] = round(statistics.median(ts), 1)
        if rank == 0:
            print(json.dumps({"world": world, "devices": min(world, ndev), "bytes": nbytes, **res,
                              "error_word": ar.check()}), flush=True)
    ar.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--sizes", default="16,4096,65536,1048576")
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    sizes = [int(v) for v in a.sizes.split(",")]
    mp.spawn(_worker, args=(a.world, port, sizes, a.iters), nprocs=a.world, join=True)


if __name__ == "__main__":
    main()
