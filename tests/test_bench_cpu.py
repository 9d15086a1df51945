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


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_bench_self_launches_n_ranks(n):
    """n = 8 rehearses the driver's scaling run (bench.py --gpus 8) end to end on gloo: pad unit, shard sizes, the
    sparse tied-embedding exchange, sparse_cap and the probe-planned buckets all take their 8-rank values."""
    r = _bench(n, ["--baseline-1gpu", "10"], timeout=600)
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
    for k in ("rccl_info", "p2p_transport", "n_channels", "n_channels_per_rank", "rccl_nranks_per_rank",
              "rccl_saw_all_ranks", "link_probe"):
        assert k in rec["dist"], k  # the multi-GPU record explains itself (None / [] where it cannot apply)
    for k in ("plan_source", "alpha_us", "link_gbps"):
        assert k in rec["bucket_plan"], k
    assert rec["dist"]["params_equal_across_ranks"] and rec["dist"]["warnings"] == []
    assert rec["loss_finite"] is True  # a NaN run's throughput is void (bench.py flags it)
    if n > 1:
        assert rec["dist"]["strict"] is True
        assert rec["bucket_plan"]["tied_sparse"]  # tiny ties its embedding: the sparse exchange ran
        assert rec["dist"]["backend"] == "gloo" and rec["dist"]["launcher"] == "sftamd"
        assert rec["optimizer_sharding"] == "zero1"
        # gloo rehearsal: no RCCL log to read, but the startup link probe ran and planned the buckets
        assert rec["dist"]["rccl_info"] is False and len(rec["dist"]["n_channels_per_rank"]) == n
        assert rec["bucket_plan"]["plan_source"] == "probe" and len(rec["dist"]["link_probe"]) == 2
        assert rec["bucket_plan"]["alpha_us"] >= 1.0 and rec["bucket_plan"]["link_gbps"] >= 1.0
    else:
        assert rec["bucket_plan"]["plan_source"] == "model" and rec["dist"]["link_probe"] == []
    assert rec["bucket_plan"]["count"] >= 1
    assert rec["scaling_efficiency"] == pytest.approx(rec["value"] / (n * 10), rel=1e-3)
    assert rec["value"] > 0 and rec["final_loss"] > 0


def test_bench_replicated_ddp_path():
    r = _bench(2, ["--zero", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert _json_lines(r.stdout)[0]["optimizer_sharding"] == "none"


@pytest.mark.parametrize("n", [1, 2])
def test_bench_nonfinite_loss_fails_the_run(n):
    """A NaN parameter (injected before step 2) makes the loss non-finite: the record is still printed for the
    post-mortem (loss_finite false) but the run exits non-zero, so its throughput can never pass as a measurement."""
    r = _bench(n, env_extra={"SFTAMD_FAULT_INJECT": "0:2:nan"}, timeout=300)
    assert r.returncode == 4, (r.returncode, r.stderr[-2000:])
    recs = _json_lines(r.stdout)
    assert len(recs) == 1 and recs[0]["loss_finite"] is False
    assert "throughput is void" in r.stderr


def test_bench_failing_rank_tears_down_the_group():
    r = _bench(2, env_extra={"SFTAMD_FAULT_INJECT": "1:2:23"}, timeout=200)
    assert r.returncode == 23, (r.returncode, r.stderr[-2000:])
    assert "terminating the other ranks" in r.stderr
    assert not _json_lines(r.stdout)


def test_bench_hang_is_detected_and_reported():
    """A rank that stops making progress (not an exit: it sleeps inside step 2) while its peer blocks in the next
    collective: the heartbeat watchdogs end the run with 124 well inside the bench timeout and print the last
    heartbeat (rank, step, phase, last gradient bucket) of the hung rank."""
    import time
    t0 = time.time()
    r = _bench(2, ["--timeout-s", "150", "--hang-timeout-s", "12"], env_extra={"SFTAMD_FAULT_INJECT": "1:2:hang"},
               timeout=240)
    assert r.returncode == 124, (r.returncode, r.stderr[-3000:])
    assert time.time() - t0 < 150
    assert "injecting a hang on rank 1" in r.stderr
    assert "last heartbeat" in r.stderr and '"rank":1' in r.stderr, r.stderr[-3000:]
    assert '"bucket"' in r.stderr  # the DDP engine's position rides in every heartbeat
    assert not _json_lines(r.stdout)


def test_dist_warnings_fail_loud_on_degraded_transport():
    from llm_fine_tune_distributed_amd.parallel.rccl_info import dist_warnings
    ok = {"p2p_transport": ["P2P/IPC"], "n_channels": 16, "nranks": 8, "init_ok": True}
    assert dist_warnings([ok] * 8, 8) == ([], False)
    w, fatal = dist_warnings([ok] * 7 + [dict(ok, p2p_transport=["SHM/direct/direct"])], 8)
    assert fatal and "rank 7" in w[0] and "SHM" in w[0]
    assert dist_warnings([ok] * 7 + [dict(ok, nranks=4)], 8)[1]
    assert dist_warnings([dict(ok, n_channels=4)] * 8, 8)[1]
    assert dist_warnings([dict(ok, n_channels=1, nranks=2)] * 2, 2) == ([], False)  # one link per GPU pair
    w, fatal = dist_warnings([ok] * 7 + [None], 8)  # no log: unknown, not degraded
    assert not fatal and "no RCCL INFO log" in w[0]


def test_rccl_info_summary_parser():
    from llm_fine_tune_distributed_amd.parallel.rccl_info import summarize_text
    log = "\n".join([
        "host:1:1 [0] NCCL INFO RCCL version : 2.22.3-develop",
        "host:1:1 [0] NCCL INFO Channel 00/32 :    0   1   2   3   4   5   6   7",
        "host:1:1 [0] NCCL INFO Channel 31/32 :    0   7   6   5   4   3   2   1",
        "host:1:1 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC",
        "host:1:1 [0] NCCL INFO Channel 01/0 : 0[0] -> 7[7] via P2P/direct pointer",
        "host:1:1 [0] NCCL INFO 32 coll channels, 32 collnet channels, 0 nvls channels, 32 p2p channels, 4 p2p "
        "channels per peer",
        "host:1:1 [0] NCCL INFO comm 0x1 rank 0 nranks 8 cudaDev 0 busId 1000 - Init COMPLETE"])
    s = summarize_text(log)
    assert s["nranks"] == 8
    assert s["n_channels"] == 32 and s["coll_channels"] == 32 and s["p2p_channels"] == 32
    assert s["p2p_transport"] == ["P2P/IPC", "P2P/direct pointer"] and s["init_ok"] and s["version"] == "2.22.3"
    assert summarize_text("")["n_channels"] is None
