"""Failure detection + elastic-lite restart: kill rank 1 at step 3 (gloo, 2 ranks); the launcher must
tear the group down, restart it, and the trainer must resume from checkpoint-2 and finish identically
to an uninterrupted run."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(out, env_extra, restarts):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    env.pop("SFTAMD_RESTART_COUNT", None)
    cmd = [sys.executable, "-m", "llm_fine_tune_distributed_amd.launch", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--max-restarts", str(restarts), "--grace", "5",
           os.path.join(ROOT, "tests", "_fault_worker.py"), out]
    return subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)


def test_failure_is_detected_without_restart():
    out = tempfile.mkdtemp()
    r = _launch(out, {"SFTAMD_FAULT_INJECT": "1:3"}, restarts=0)
    assert r.returncode == 17, r.stderr[-2000:]
    assert "terminating the other ranks" in r.stderr


def test_restart_resumes_from_checkpoint():
    ref = tempfile.mkdtemp()
    r0 = _launch(ref, {}, restarts=0)
    assert r0.returncode == 0, r0.stderr[-2000:]
    out = tempfile.mkdtemp()
    r = _launch(out, {"SFTAMD_FAULT_INJECT": "1:3"}, restarts=1)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.load(open(os.path.join(out, "result.json")))
    base = json.load(open(os.path.join(ref, "result.json")))
    assert res["step"] == 6 and res["restart"] == "1"
    assert abs(res["checksum"] - base["checksum"]) < 1e-6 * max(1.0, abs(base["checksum"]))


def _launch_n(out, env_extra, restarts, n):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    env.pop("SFTAMD_RESTART_COUNT", None)
    cmd = [sys.executable, "-m", "llm_fine_tune_distributed_amd.launch", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--max-restarts", str(restarts), "--grace", "5",
           os.path.join(ROOT, "tests", "_fault_worker.py"), out]
    return subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)


import pytest  # noqa: E402
import torch  # noqa: E402


@pytest.mark.parametrize("n", [2, 4])
def test_zero1_checkpoint_kill_resume_is_bit_exact(n):
    """ZeRO-1 (sharded AdamW) with save_steps=2: every rank joins the optimizer-state gather at save time (no
    deadlock), a rank killed at step 3 is torn down, the group restarts from checkpoint-2 and finishes with
    parameters bit-identical to an uninterrupted run. train_loss averages the steps run after the resume."""
    env = {"SFTAMD_TEST_SHARD": "1"}
    ref = tempfile.mkdtemp()
    r0 = _launch_n(ref, env, 0, n)
    assert r0.returncode == 0, r0.stderr[-3000:]
    out = tempfile.mkdtemp()
    r = _launch_n(out, dict(env, SFTAMD_FAULT_INJECT="1:3"), 1, n)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.load(open(os.path.join(out, "result.json")))
    base = json.load(open(os.path.join(ref, "result.json")))
    assert res["optimizer"] == base["optimizer"] == "ShardedAdamW"
    assert res["step"] == 6 and res["restart"] == "1"
    assert torch.equal(torch.load(os.path.join(out, "params.pt")), torch.load(os.path.join(ref, "params.pt")))
    assert res["log"][-4:] == base["log"][-4:]
    # resumed call ran steps 3..6: its train_loss is their mean (not a sum over 4 steps divided by 6)
    assert abs(res["train_loss"] - sum(res["log"][-4:]) / 4) < 1e-6
    assert abs(base["train_loss"] - sum(base["log"][-6:]) / 6) < 1e-6


def test_launcher_reports_the_first_rank_to_fail(tmp_path):
    """Rank 1 exits 23; rank 0 dies with 1 a moment later (as on a broken collective) — both inside ONE monitor
    interval. The launcher must blame rank 1 and return 23 (arrival order), not the lowest failing rank index."""
    script = tmp_path / "two_failures.py"
    script.write_text(
        "import os, sys, time\n"
        "r = int(os.environ['RANK'])\n"
        "time.sleep(0.5 if r == 1 else 0.9)\n"
        "sys.exit(23 if r == 1 else 1)\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "llm_fine_tune_distributed_amd.launch", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--monitor-interval", "3", "--grace", "2", str(script)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 23, (r.returncode, r.stderr[-2000:])
    assert "local rank 1 exited with code 23" in r.stderr
