"""Single-node multi-GPU launcher (replaces the reference's Kubeflow PyTorchJob).

    python -m llm_fine_tune_distributed_amd.launch --nproc-per-node 8 train_script.py [args...]
    python -m llm_fine_tune_distributed_amd.launch --nproc-per-node 8 -m llm_fine_tune_distributed_amd.cli.train

One process per GPU; each child gets the torchrun env contract (``WORLD_SIZE, RANK, LOCAL_RANK,
LOCAL_WORLD_SIZE, MASTER_ADDR, MASTER_PORT``) plus ``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC for
RCCL over xGMI). The launcher never touches the GPU itself.

Failure detection: the launcher polls its children; when one exits non-zero the others are
terminated (SIGTERM, then SIGKILL after ``--grace``) instead of blocking in a collective until
the watchdog timeout (the reference's "workers hang until NCCL timeout"). With
``--max-restarts K`` the whole group is restarted (``SFTAMD_RESTART_COUNT`` is exported) and the
training script resumes from its latest checkpoint (``--resume auto``).

Hang detection: every rank writes a one-line heartbeat (step, phase, last gradient bucket launched) into
``$SFTAMD_HEARTBEAT_DIR/rank<r>.hb`` (utils/heartbeat.py). With ``--hang-timeout S`` a rank whose heartbeat has
not changed for S seconds (or that wrote none within ``--startup-timeout``) is declared hung; ``--deadline S``
bounds the whole run. Either way — and on any failing rank — the launcher prints the last heartbeat of EVERY rank
before tearing the group down, and exits with 124 for a hang / deadline.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import shutil
import subprocess
import sys
import tempfile
import threading
import time
from typing import List, Tuple


def _free_port(addr: str) -> int:
    s = socket.socket()
    s.bind((addr, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _die_with_parent():
    """Child pre-exec: SIGTERM this rank when the launcher dies (PR_SET_PDEATHSIG), so a launcher killed by
    a time limit never leaves ranks holding GPUs."""
    try:
        import ctypes
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # 1 = PR_SET_PDEATHSIG
    except Exception:
        pass


def _spawn(n: int, cmd: List[str], addr: str, port: int, restart: int, node_rank: int, nnodes: int,
           new_session: bool = True, hb_dir: str = "") -> List[subprocess.Popen]:
    procs = []
    for lr in range(n):
        env = dict(os.environ)
        env.update(WORLD_SIZE=str(n * nnodes), RANK=str(node_rank * n + lr), LOCAL_RANK=str(lr),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK=str(node_rank), MASTER_ADDR=addr, MASTER_PORT=str(port),
                   SFTAMD_RESTART_COUNT=str(restart), SFTAMD_LAUNCHER="sftamd", SFTAMD_HEARTBEAT_DIR=hb_dir)
        # dmabuf IPC (the only IPC mode the hosts' driver supports; rationale: parallel/process_group.py) unless the
        # caller set the mode explicitly
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        env.setdefault("OMP_NUM_THREADS", "1")
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=new_session, preexec_fn=_die_with_parent))
    return procs


class _ExitLog:
    """Children's exits in ARRIVAL order: one reaper thread per child blocks in its waitpid and appends
    (local rank, code) the moment that child exits. A polling loop that collects every exit seen in one interval
    and takes the lowest rank misattributes a failure when the faulting rank's peer dies on the broken collective
    inside the same interval (rank 1 exits 23, rank 0 then exits 1: the group must be reported as failed by rank 1)."""

    def __init__(self, procs: List[subprocess.Popen]):
        self._lock = threading.Lock()
        self.order: List[Tuple[int, int]] = []
        self._threads = [threading.Thread(target=self._reap, args=(i, p), daemon=True) for i, p in enumerate(procs)]
        for t in self._threads:
            t.start()

    def _reap(self, i: int, p: subprocess.Popen):
        code = p.wait()
        with self._lock:
            self.order.append((i, code))

    def first_failure(self):
        with self._lock:
            for i, c in self.order:
                if c != 0:
                    return i, c
        return None

    def count(self) -> int:
        with self._lock:
            return len(self.order)


def _signal(p: subprocess.Popen, sig, group: bool):
    try:
        if group:
            os.killpg(p.pid, sig)
        else:
            p.send_signal(sig)
    except ProcessLookupError:
        pass


def _terminate(procs: List[subprocess.Popen], grace: float, group: bool = True):
    for p in procs:
        if p.poll() is None:
            _signal(p, signal.SIGTERM, group)
    t0 = time.time()
    while time.time() - t0 < grace and any(p.poll() is None for p in procs):
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            _signal(p, signal.SIGKILL, group)
    for p in procs:
        p.wait()


def _heartbeats(hb_dir: str, n: int, node_rank: int):
    """Last heartbeat line of each local rank (read without importing the package: no torch in the launcher)."""
    out = []
    now = time.time()
    for lr in range(n):
        r = node_rank * n + lr
        p = os.path.join(hb_dir, f"rank{r}.hb")
        try:
            with open(p) as f:
                out.append((lr, f.read().strip(), now - os.path.getmtime(p)))
        except OSError:
            out.append((lr, None, None))
    return out


def _print_heartbeats(hb_dir: str, n: int, node_rank: int):
    for lr, line, age in _heartbeats(hb_dir, n, node_rank):
        if line is None:
            print(f"[launch] local rank {lr}: no heartbeat", file=sys.stderr, flush=True)
        else:
            print(f"[launch] local rank {lr} last heartbeat ({age:.1f} s ago): {line}", file=sys.stderr, flush=True)


def _hung(hb_dir: str, n: int, node_rank: int, procs, started: float, hang_timeout: float, startup: float):
    """(local rank, reason) of the first live rank whose heartbeat is stale, else None."""
    if hang_timeout <= 0:
        return None
    now = time.time()
    for (lr, line, age), p in zip(_heartbeats(hb_dir, n, node_rank), procs):
        if p.poll() is not None:
            continue
        if line is None:
            if now - started > startup:
                return lr, f"no heartbeat within {startup:.0f} s of the start"
            continue
        try:
            rec = json.loads(line)
        except ValueError:
            rec = {}
        if rec.get("paused"):  # outside the training loop (utils/heartbeat.py pause())
            continue
        limit = max(hang_timeout, float(rec.get("limit_s", 0) or 0))  # a slow phase under Heartbeat.hold
        if age > limit:
            return lr, f"heartbeat unchanged for {age:.0f} s (hang limit {limit:.0f} s)"
    return None


def run(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node-rank", type=int, default=0)
    ap.add_argument("--master-addr", "--master_addr", default=os.environ.get("MASTER_ADDR", "127.0.0.1"))
    ap.add_argument("--master-port", "--master_port", type=int, default=int(os.environ.get("MASTER_PORT", "0")))
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("--grace", type=float, default=10.0)
    ap.add_argument("--monitor-interval", type=float, default=0.5)
    ap.add_argument("--hang-timeout", type=float, default=float(os.environ.get("SFTAMD_HANG_TIMEOUT_S", "0") or 0),
                    help="seconds without a heartbeat change after which a rank counts as hung (0 = off)")
    ap.add_argument("--startup-timeout", type=float, default=900.0,
                    help="seconds a rank may take to write its first heartbeat (first import of torch, model build)")
    ap.add_argument("--deadline", type=float, default=0.0, help="wall-clock limit of the whole run in seconds (0 = none)")
    ap.add_argument("--heartbeat-dir", default=os.environ.get("SFTAMD_HEARTBEAT_DIR", ""))
    ap.add_argument("--same-session", action="store_true",
                    help="keep the ranks in the launcher's process group (a signal to the group reaches them)")
    ap.add_argument("-m", dest="module", default=None, help="run a module (like python -m)")
    ap.add_argument("script", nargs="?")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.module:
        cmd = [sys.executable, "-u", "-m", a.module] + ([a.script] if a.script else []) + a.args
    elif a.script:
        cmd = [sys.executable, "-u", a.script] + a.args
    else:
        ap.error("need a script or -m module")
    own_dir = not a.heartbeat_dir
    hb_dir = a.heartbeat_dir or tempfile.mkdtemp(prefix="sftamd_hb_")
    os.makedirs(hb_dir, exist_ok=True)
    try:
        return _run_group(a, cmd, hb_dir)
    finally:
        if own_dir:
            shutil.rmtree(hb_dir, ignore_errors=True)


def _run_group(a, cmd, hb_dir: str) -> int:
    restart = 0
    t_run = time.time()
    n = a.nproc_per_node
    while True:
        port = a.master_port or _free_port(a.master_addr)
        for r in range(a.node_rank * n, (a.node_rank + 1) * n):  # this node's ranks restart with no heartbeats
            try:  # (a shared directory also holds the other nodes' files: leave those)
                os.remove(os.path.join(hb_dir, f"rank{r}.hb"))
            except OSError:
                pass
        started = time.time()
        procs = _spawn(a.nproc_per_node, cmd, a.master_addr, port, restart, a.node_rank, a.nnodes,
                       new_session=not a.same_session, hb_dir=hb_dir)
        grp = not a.same_session
        exits = _ExitLog(procs)
        failed = None
        try:
            while True:
                bad = exits.first_failure()
                if bad is not None:
                    failed = bad
                    break
                if exits.count() == len(procs):
                    return 0
                if a.deadline > 0 and time.time() - t_run > a.deadline:
                    failed = (-1, 124, f"deadline of {a.deadline:.0f} s exceeded")
                    break
                h = _hung(hb_dir, a.nproc_per_node, a.node_rank, procs, started, a.hang_timeout,
                          max(a.startup_timeout, a.hang_timeout))
                if h is not None:
                    failed = (h[0], 124, h[1])
                    break
                time.sleep(a.monitor_interval)
        except KeyboardInterrupt:
            _terminate(procs, a.grace, grp)
            return 130
        if len(failed) == 3:
            rank, code, why = failed
            who = "the run" if rank < 0 else f"local rank {rank}"
            print(f"[launch] hang: {who}: {why}; terminating all ranks", file=sys.stderr, flush=True)
        else:
            rank, code = failed
            print(f"[launch] local rank {rank} exited with code {code}; terminating the other ranks", file=sys.stderr,
                  flush=True)
        _print_heartbeats(hb_dir, a.nproc_per_node, a.node_rank)
        _terminate(procs, a.grace, grp)
        if restart >= a.max_restarts:
            return code if code > 0 else 1
        restart += 1
        print(f"[launch] restarting group (attempt {restart}/{a.max_restarts})", file=sys.stderr, flush=True)


def main():
    sys.exit(run())


if __name__ == "__main__":
    main()
