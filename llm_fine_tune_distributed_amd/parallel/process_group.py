"""Process bootstrap: env-var contract, device binding, RCCL/gloo process group.

Same env contract and defaults as the reference's ``setup_distributed`` (``training.py:16-42``):
``WORLD_SIZE=1, RANK=0, LOCAL_RANK=0, MASTER_ADDR=localhost, MASTER_PORT=23456``. Unlike the
reference (which binds every rank to ``cuda:0``, ``training.py:85``) the local rank is bound to
its own GPU *before* any allocation, and the process group is actually initialised here:
``nccl`` (= RCCL on ROCm, xGMI peer-to-peer) when GPUs are present, ``gloo`` on CPU.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistState:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_STATE: Optional[DistState] = None


def read_env():
    ws = int(os.getenv("WORLD_SIZE", "1"))
    rank = int(os.getenv("RANK", "0"))
    lr = int(os.getenv("LOCAL_RANK", os.getenv("RANK", "0")))
    os.environ.setdefault("MASTER_ADDR", "localhost")
    os.environ.setdefault("MASTER_PORT", "23456")
    return ws, rank, lr


def nccl_options():
    """RCCL process-group options: collectives on a HIGH-PRIORITY HIP stream. The bucket reduce-scatters / all-reduces (backward) and the ZeRO-1 all-gathers (forward)
    are meant to run under the compute kernels; on a busy device a high-priority queue gets their
    kernels dispatched as soon as CUs free up instead of behind the queued GEMMs."""
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except (AttributeError, RuntimeError):
        return None


def setup_distributed(backend: Optional[str] = None, timeout_s: float = 1800.0, device: Optional[str] = None,
                      verbose: bool = True) -> DistState:
    """Initialise (once) and return the distributed state."""
    global _STATE
    if _STATE is not None:
        return _STATE
    ws, rank, local_rank = read_env()
    # dmabuf IPC for RCCL / CUDA-tensor sharing between ranks. Why it is on by default: the MI355X hosts this runs on
    # ship a kernel driver that supports ONLY dmabuf IPC — with the legacy mode, hipIpcGetMemHandle fails with
    # "invalid argument", which is what RCCL's intra-node P2P/IPC transport (and any CUDA-tensor sharing between
    # ranks) calls at communicator setup; dmabuf is also the upstream ROCm 7 default path. An explicit setting in the
    # environment wins (setdefault). The HSA runtime reads it once, when it initialises, which
    # torch.cuda.is_available() below triggers — so it must be in the environment before that call.
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    use_gpu = (device != "cpu") and torch.cuda.is_available()
    if use_gpu:
        n = torch.cuda.device_count()
        torch.cuda.set_device(local_rank % n)
        dev = torch.device("cuda", local_rank % n)
    else:
        dev = torch.device("cpu")
    be = backend or os.environ.get("SFTAMD_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if ws > 1 and not dist.is_initialized():
        # RCCL: keep peer-to-peer (xGMI) on; async error handling = watchdog aborts on hangs.
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = dict(backend=be, init_method="env://", world_size=ws, rank=rank,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = dev
            opts = nccl_options()
            if opts is not None:
                kw["pg_options"] = opts
        dist.init_process_group(**kw)
        if verbose and rank == 0:
            print(f"[dist] {be} world_size={ws} master={os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}",
                  flush=True)
    elif ws == 1 and verbose:
        print("[dist] single-process mode", flush=True)
    _STATE = DistState(ws, rank, local_rank, dev, be if ws > 1 else None)
    return _STATE


def get_state() -> DistState:
    return _STATE if _STATE is not None else setup_distributed(verbose=False)


def barrier():
    if dist.is_available() and dist.is_initialized():
        st = get_state()
        if st.backend == "nccl" and st.device.type == "cuda":
            dist.barrier(device_ids=[st.device.index])
        else:
            dist.barrier()


def cleanup_distributed():
    """Explicit barrier + destroy (the reference only prints, training.py:44-47)."""
    global _STATE
    if dist.is_available() and dist.is_initialized():
        try:
            barrier()
        finally:
            dist.destroy_process_group()
    _STATE = None


def all_reduce_sum_(t: torch.Tensor) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


class PendingCount:
    """A count whose all-reduce is in flight; ``resolve()`` makes the current stream wait for it (once)
    and returns it clamped to >= 1, times ``scale``."""

    def __init__(self, t: torch.Tensor, work=None, scale: float = 1.0):
        self._t, self._work, self._done, self._scale = t, work, None, scale

    def resolve(self) -> torch.Tensor:
        if self._done is None:
            if self._work is not None:
                self._work.wait()
            self._done = self._t.clamp(min=1.0)
            if self._scale != 1.0:
                self._done = self._done * self._scale
        return self._done


def all_reduce_sum_async(t: torch.Tensor, group=None, scale: float = 1.0) -> PendingCount:
    """In-place SUM all-reduce of ``t`` (over ``group``, default the world) issued without blocking the compute
    stream (a group of one: nothing in flight); the resolved count is multiplied by ``scale``."""
    work = None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        work = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True)
    return PendingCount(t, work, scale)


def broadcast_object(obj, src: int = 0):
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        lst = [obj]
        dist.broadcast_object_list(lst, src=src)
        return lst[0]
    return obj
