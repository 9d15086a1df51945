"""Step-phase timing and trace ranges.

* ``StepTimer``: GPU-event timing of named phases (data, fwd, bwd, comm wait, optimizer) without
  host syncs inside the step; ``summary()`` syncs once and returns milliseconds per phase.
* ``range(name)``: roctx range (visible in ``rocprofv3 --marker-trace`` / torch profiler) when
  available, a no-op otherwise.
* ``torch_profile(...)``: torch.profiler with ROCm activities, Chrome trace export.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict

import torch


@contextlib.contextmanager
def range(name: str):
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)  # maps to roctx on ROCm builds
            pushed = True
        except Exception:
            pass
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


class StepTimer:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._ev = defaultdict(list)
        self._cpu = defaultdict(float)

    @contextlib.contextmanager
    def phase(self, name: str, host: bool = False):
        """Time ``name``: device time between two events on the current stream (no sync), or host wall time
        when the timer is disabled / ``host=True`` (e.g. data loading, which runs on the CPU)."""
        if not self.enabled or host:
            t = time.perf_counter()
            with range(name):
                yield
            self._cpu[name] += time.perf_counter() - t
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        with range(name):
            yield
        e.record()
        self._ev[name].append((s, e))

    def summary(self, reset: bool = True) -> Dict[str, float]:
        out = {}
        if self.enabled:
            torch.cuda.synchronize()
            for k, lst in self._ev.items():
                out[k] = sum(s.elapsed_time(e) for s, e in lst)
        for k, v in self._cpu.items():
            out[k] = out.get(k, 0.0) + v * 1e3
        if reset:
            self._ev.clear()
            self._cpu.clear()
        return out


def torch_profile(out_path: str, steps: int = 3):
    from torch.profiler import ProfilerActivity, profile, schedule
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    return profile(activities=acts, schedule=schedule(wait=0, warmup=1, active=steps),
                   on_trace_ready=lambda p: p.export_chrome_trace(out_path), record_shapes=True)
