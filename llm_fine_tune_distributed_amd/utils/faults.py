"""Fault injection for failure-detection / resume tests.

``SFTAMD_FAULT_INJECT="rank:step[:code]"`` makes that rank exit abruptly (``os._exit``) when it
reaches that optimizer step — the launcher must then tear the group down and, with
``--max-restarts``, restart it so the trainer resumes from the latest checkpoint. Only the first
attempt injects (``SFTAMD_RESTART_COUNT == 0``).

``SFTAMD_FAULT_INJECT="rank:step:hang"`` makes that rank stop making progress instead (it sleeps forever without
exiting, like a rank stuck in a driver call): the other ranks then block in their next collective, and only the
heartbeat watchdogs (utils/heartbeat.py, launch.py ``--hang-timeout``) end the run.

``SFTAMD_FAULT_INJECT="rank:step:nan"`` poisons one parameter of that rank with a NaN before that step
(bench.py; the non-finite loss must fail the run instead of producing a throughput record).
"""
from __future__ import annotations

import os
import sys
import time


def maybe_inject(rank: int, step: int) -> None:
    spec = os.environ.get("SFTAMD_FAULT_INJECT")
    if not spec or os.environ.get("SFTAMD_RESTART_COUNT", "0") != "0":
        return
    parts = spec.split(":")
    r, s = int(parts[0]), int(parts[1])
    if rank != r or step != s:
        return
    if len(parts) > 2 and parts[2] == "nan":
        return  # (nan_injection: the caller poisons a parameter)
    if len(parts) > 2 and parts[2] == "hang":
        print(f"[fault] injecting a hang on rank {rank} at step {step}", file=sys.stderr, flush=True)
        while True:
            time.sleep(3600)
    code = int(parts[2]) if len(parts) > 2 else 17
    print(f"[fault] injecting failure on rank {rank} at step {step}", file=sys.stderr, flush=True)
    os._exit(code)


def nan_injection(rank: int, step: int) -> bool:
    """True when ``SFTAMD_FAULT_INJECT="rank:step:nan"`` names this rank and step (first attempt only)."""
    spec = os.environ.get("SFTAMD_FAULT_INJECT")
    if not spec or os.environ.get("SFTAMD_RESTART_COUNT", "0") != "0":
        return False
    parts = spec.split(":")
    return len(parts) > 2 and parts[2] == "nan" and int(parts[0]) == rank and int(parts[1]) == step
