"""RCCL INFO log of a world-size-1 communicator on one MI355X, through parallel/rccl_info.py: what summarize() reads
from a real RCCL log (init_ok, nranks, version, channels). The raw log is kept in gpurun_out/rccl_info_probe/.

    python tools/probe_rccl_info.py
"""
import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    d = os.path.abspath("gpurun_out/rccl_info_probe")
    from llm_fine_tune_distributed_amd.parallel import rccl_info
    rccl_info.enable(d)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="env://", world_size=1, rank=0, device_id=torch.device("cuda", 0))
    x = torch.ones(1 << 20, device="cuda")
    dist.all_reduce(x)
    dist.barrier()
    torch.cuda.synchronize()
    summ = rccl_info.summarize(d)
    print(json.dumps(summ), flush=True)
    print(rccl_info.dist_warnings([summ], 1), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
