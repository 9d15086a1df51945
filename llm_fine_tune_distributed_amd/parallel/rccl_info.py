"""RCCL topology / transport capture for the first multi-GPU run ("verify channel count with
NCCL_DEBUG=INFO"; the reference's job runs with ``NCCL_DEBUG=INFO``, ``deploy/pytorchjob.yaml:51-64``).

``enable(dir)`` (before the process group exists) points RCCL's INFO log of this process at a file of its own
(``NCCL_DEBUG=INFO``, ``NCCL_DEBUG_FILE=<dir>/rccl.<pid>.log``, ``NCCL_DEBUG_SUBSYS=INIT,GRAPH,ENV``);
``summarize(path)`` reduces it to what a scaling run needs to be explained:

* ``p2p_transport``: the distinct ``via ...`` transports of the ring / tree connections (``P2P/IPC``,
  ``P2P/direct pointer``, ``SHM``, ``NET/...``) — over xGMI every peer should be P2P;
* ``n_channels``: the number of channels of the communicator (``Channel xx/NN`` lines; RCCL stripes a collective
  over them, so on an 8-GPU mesh it should be well above one ring per link);
* ``coll_channels`` / ``p2p_channels``: from the ``N coll channels, ... M p2p channels`` summary line;
* ``version``: the ``RCCL version`` line; ``init_ok``: an ``Init COMPLETE`` line was seen; ``nranks``: the rank
  count of the communicator (``comm ... nranks N`` lines) — must equal WORLD_SIZE.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Dict, Optional

_CHAN = re.compile(r"Channel (\d+)/(\d+)")
_VIA = re.compile(r"via ((?:P2P|SHM|NET|NVLS|COLLNET)[^\s,]*(?: pointer)?(?:/read)?)")
_SUMMARY = re.compile(r"(\d+) coll channels.*?(\d+) p2p channels")
_VERSION = re.compile(r"RCCL version[^\d]*([\d.]+)|NCCL version[^\d]*([\d.]+)")
_NRANKS = re.compile(r"nranks (\d+)")


def enable(directory: str) -> str:
    """Route this process's RCCL INFO log to ``directory`` (call before init_process_group). Returns the pattern."""
    os.makedirs(directory, exist_ok=True)
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,GRAPH,ENV")
    pat = os.path.join(directory, "rccl.%p.log")
    os.environ["NCCL_DEBUG_FILE"] = pat
    return pat


def summarize_text(text: str) -> Dict:
    chans, via = set(), set()
    nmax = 0
    coll = p2p = None
    version = None
    nranks = None
    for line in text.splitlines():
        if "NCCL INFO" not in line and "RCCL" not in line:
            continue
        m = _CHAN.search(line)
        if m:
            chans.add(int(m.group(1)))
            nmax = max(nmax, int(m.group(2)))
        for v in _VIA.findall(line):
            via.add(v.strip())
        m = _SUMMARY.search(line)
        if m:
            coll, p2p = int(m.group(1)), int(m.group(2))
        m = _NRANKS.search(line)
        if m:
            nranks = max(nranks or 0, int(m.group(1)))
        m = _VERSION.search(line)
        if m and version is None:
            version = m.group(1) or m.group(2)
    n = max(len(chans), nmax)
    return {"p2p_transport": sorted(via) or None, "n_channels": n or None, "coll_channels": coll,
            "p2p_channels": p2p, "version": version, "init_ok": "Init COMPLETE" in text, "nranks": nranks}


def summarize(directory: str, pid: Optional[int] = None) -> Optional[Dict]:
    """Summary of this process's (``pid``, default os.getpid()) RCCL log in ``directory``; None if absent."""
    pid = os.getpid() if pid is None else pid
    files = glob.glob(os.path.join(directory, f"rccl.{pid}.log")) or glob.glob(os.path.join(directory, "rccl.*.log"))
    if not files:
        return None
    text = ""
    for f in files[:1]:
        try:
            with open(f, errors="replace") as fh:
                text = fh.read()
        except OSError:
            return None
    return summarize_text(text)


def dist_warnings(per_rank, world_size: int):
    """(warnings, fatal) for the multi-GPU record from every rank's ``summarize`` result (None = no log).

    Fatal = positive evidence of a degraded collective path: a non-P2P transport (SHM / NET instead of xGMI P2P),
    a communicator that saw a different rank count, an init that never completed, or fewer channels than peer links
    (world_size - 1: one xGMI link per GPU pair on an MI355X node). A missing log is a (non-fatal) warning: nothing is
    known about that rank."""
    warnings, fatal = [], False
    for r, s in enumerate(per_rank):
        if not s:
            warnings.append(f"rank {r}: no RCCL INFO log (transport unknown)")
            continue
        bad = [t for t in (s.get("p2p_transport") or []) if not str(t).startswith("P2P")]
        if bad:
            warnings.append(f"rank {r}: transport {','.join(bad)} (expected P2P over xGMI)")
            fatal = True
        if s.get("nranks") is not None and s["nranks"] != world_size:
            warnings.append(f"rank {r}: communicator saw {s['nranks']} ranks, WORLD_SIZE={world_size}")
            fatal = True
        if s.get("init_ok") is False:
            warnings.append(f"rank {r}: no 'Init COMPLETE' in the RCCL log")
            fatal = True
        nch = s.get("n_channels")
        if nch is not None and nch < world_size - 1:
            warnings.append(f"rank {r}: {nch} channels < {world_size - 1} peer links")
            fatal = True
    return warnings, fatal
