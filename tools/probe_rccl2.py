"""Can RCCL (torch.distributed "nccl") form a 2-rank communicator on ONE MI355X? (The 1-GPU box is the only GPU this
build loop can run on; the 8-GPU scaling run is the driver's.) Two spawned ranks on cuda:0: init, all_reduce,
reduce_scatter, all_gather; prints what happens.

    python tools/probe_rccl2.py

Result (r5_run34): RCCL refuses it ("Duplicate GPU detected", ncclInvalidUsage) — profiles/r5_rccl_probe.md.
"""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                      NCCL_DEBUG="WARN")
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", init_method="env://", world_size=2, rank=rank, device_id=dev)
        x = torch.full((1 << 20,), float(rank + 1), device=dev)
        dist.all_reduce(x)
        y = torch.empty(1 << 19, device=dev)
        dist.reduce_scatter_tensor(y, x)
        z = torch.empty(1 << 20, device=dev)
        dist.all_gather_into_tensor(z, y)
        torch.cuda.synchronize()
        q.put((rank, f"ok all_reduce={x[0].item()} reduce_scatter={y[0].item()} all_gather={z[-1].item()}"))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - report whatever RCCL says
        q.put((rank, f"error {type(e).__name__}: {str(e)[:400]}"))


def main():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    [p.start() for p in ps]
    for _ in range(2):
        try:
            print(q.get(timeout=120), flush=True)
        except Exception:  # noqa: BLE001
            print("no answer within 120 s", flush=True)
            break
    for p in ps:
        p.join(timeout=30)
        if p.exitcode is None:
            p.kill()
        print("exit", p.exitcode, flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
