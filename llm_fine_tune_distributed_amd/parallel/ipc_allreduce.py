"""One-shot peer-memory all-reduce for small messages, csrc/ipc_allreduce.hip.

RCCL's ring / tree all-reduce pays several kernel-to-kernel hops per call; for a few KB (the step's token count,
the clip norm, metrics) a single kernel that reads every peer's copy over xGMI and sums them locally is latency-
bound instead. Each rank registers one device region, the regions are exchanged as HIP IPC (dmabuf) handles over the
existing process group, and every call is one kernel on the caller's stream:

    ar = IPCAllReduce(max_bytes=1 << 20)          # collective: every rank of the group
    ar.all_reduce_(t)                              # in place, SUM, bf16 / fp32, numel * esz % 16 == 0
    assert ar.check() == 0                         # 1 = a bounded wait timed out (a peer never arrived)

Every rank sums the ranks' chunks in rank order, so the result is bitwise identical on all ranks. Waits are bounded
(2 s) so a missing peer reports an error instead of hanging the device; the timed-out call's output is poisoned with
NaN, and ``raise_if_failed()`` (non-blocking: it reads a pinned copy of the error word written behind each call)
raises on the next use. Opt-in (`SFTAMD_IPC_ALLREDUCE=1` routes the trainer's scalar all-reduces through it) and
UNVALIDATED across GPUs: the only test runs two ranks on one GPU (shared L2); the region is allocated uncached so that
cross-GPU polling cannot read stale lines, but no multi-GPU run has exercised it yet.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import _ext


class IPCAllReduce:
    def __init__(self, max_bytes: int = 1 << 20, group=None, blocks: int = 16):
        if not _ext.load():
            raise RuntimeError(f"IPCAllReduce needs the HIP extension: {_ext.load_error()}")
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.max_bytes = (int(max_bytes) + 15) // 16 * 16
        self.blocks = blocks
        ops = _ext.ops()
        self.ctx = ops.ipc_ar_create(self.max_bytes, self.world, self.rank)
        handle = list(ops.ipc_ar_handle(self.ctx))
        handles = [handle]
        if self.world > 1:
            handles = [None] * self.world
            dist.all_gather_object(handles, handle, group=group)
        ops.ipc_ar_open(self.ctx, [w for h in handles for w in h])
        if self.world > 1:
            dist.barrier(group=group)  # every peer has opened every region before the first call
        self.round = 0

    def fits(self, t: torch.Tensor) -> bool:
        n = t.numel() * t.element_size()
        return (t.is_cuda and t.is_contiguous() and t.dtype in (torch.bfloat16, torch.float32) and n <= self.max_bytes
                and n % 16 == 0)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM over the group on the current stream (every rank must call, in the same order)."""
        if not self.fits(t):
            raise ValueError(f"IPCAllReduce: {t.dtype} x {t.numel()} does not fit ({self.max_bytes} B, 16-B multiple)")
        self.round += 1
        _ext.ops().ipc_ar_allreduce(t, self.ctx, self.round, self.blocks)
        return t

    def check(self) -> int:
        """Synchronises the device; 0 = every wait completed, 1 = a wait timed out."""
        return int(_ext.ops().ipc_ar_check(self.ctx))

    def poll(self) -> int:
        """Error word of the last finished call without waiting: -1 still running, 0 ok, 1 a wait timed out."""
        return int(_ext.ops().ipc_ar_poll(self.ctx))

    def raise_if_failed(self):
        if self.poll() > 0:
            raise RuntimeError("IPCAllReduce: a peer did not arrive within the bounded wait (output poisoned with NaN); "
                               "unset SFTAMD_IPC_ALLREDUCE to use the process group's all-reduce")

    @property
    def uncached(self) -> bool:
        return bool(_ext.ops().ipc_ar_uncached(self.ctx))

    def close(self):
        if self.ctx is not None:
            if self.world > 1:
                dist.barrier(group=self.group)  # no peer still reads this region
            _ext.ops().ipc_ar_destroy(self.ctx)
            self.ctx = None
