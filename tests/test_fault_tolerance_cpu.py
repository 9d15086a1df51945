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
