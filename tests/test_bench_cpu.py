"""bench.py as the driver runs it, rehearsed on CPU/gloo: ``python bench.py --gpus N`` with no external
launcher spawns N ranks itself (the parent never imports torch), rank 0 prints ONE JSON line with the
driver contract fields plus the multi-GPU diagnostics, and a failing rank tears the group down."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--device", "cpu", "--model", "tiny", "--steps", "2", "--warmup", "1", "--micro-batch", "2", "--seq", "32"]


def _bench(n, extra=(), env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)] + SMALL + list(extra),
                          env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{") and '"metric"' in l]


@pytest.mark.parametrize("n", [1, 2, 4])
def test_bench_self_launches_n_ranks(n):
    r = _bench(n, ["--baseline-1gpu", "10"])
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout  # exactly one JSON line, from rank 0
    rec = recs[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["n_gpus"] == n and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["global_batch"] == 2 * n and rec["config"]["parallelism"] == f"dp{n}"
    assert rec["dist"]["world_size"] == n and rec["dist"]["consistent"]
    assert len(rec["per_rank"]) == n
    if n > 1:
        assert rec["dist"]["backend"] == "gloo" and rec["dist"]["launcher"] == "sftamd"
        assert rec["optimizer_sharding"] == "zero1"
    assert rec["bucket_plan"]["count"] >= 1
    assert rec["scaling_efficiency"] == pytest.approx(rec["value"] / (n * 10), rel=1e-3)
    assert rec["value"] > 0 and rec["final_loss"] > 0


def test_bench_replicated_ddp_path():
    r = _bench(2, ["--zero", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert _json_lines(r.stdout)[0]["optimizer_sharding"] == "none"


def test_bench_failing_rank_tears_down_the_group():
    r = _bench(2, env_extra={"SFTAMD_FAULT_INJECT": "1:2:23"}, timeout=200)
    assert r.returncode == 23, (r.returncode, r.stderr[-2000:])
    assert "terminating the other ranks" in r.stderr
    assert not _json_lines(r.stdout)
