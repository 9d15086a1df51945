"""Heartbeat slow-phase limits seen by the launcher's watchdog (utils/heartbeat.py, launch.py): a phase under
``Heartbeat.hold`` must be allowed its slow-phase limit even when the rank runs no in-process watchdog (the
launcher-only configuration: ``launch.py --hang-timeout`` without ``SFTAMD_HANG_TIMEOUT_S`` in the children), and a
hold lifts ``pause()`` so a stuck final save is still bounded."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HB = os.path.join(ROOT, "llm_fine_tune_distributed_amd", "utils", "heartbeat.py")


def _load():
    import importlib.util
    spec = importlib.util.spec_from_file_location("_hb_under_test", HB)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _rec(d):
    with open(os.path.join(d, "rank0.hb")) as f:
        return json.loads(f.read())


def test_hold_writes_limit_without_inprocess_watchdog(tmp_path, monkeypatch):
    monkeypatch.delenv("SFTAMD_HANG_TIMEOUT_S", raising=False)
    hb = _load().Heartbeat(0, directory=str(tmp_path), stderr_every_s=0, hang_timeout_s=0)
    hb.beat(1, "step")
    assert "limit_s" not in _rec(tmp_path)
    with hb.hold("save", timeout_s=77):
        assert _rec(tmp_path)["limit_s"] == 77
    assert "limit_s" not in _rec(tmp_path)
    with hb.hold("load"):
        assert _rec(tmp_path)["limit_s"] == hb.slow_timeout >= 1800
    hb.close()


def test_hold_lifts_pause(tmp_path):
    hb = _load().Heartbeat(0, directory=str(tmp_path), stderr_every_s=0, hang_timeout_s=5)
    hb.pause()
    assert _rec(tmp_path).get("paused")
    with hb.hold("final_save", timeout_s=40):
        r = _rec(tmp_path)
        assert not r.get("paused") and r["limit_s"] == 40
        assert hb._limit == 40  # the in-process watchdog applies the hold's limit too
    assert _rec(tmp_path).get("paused") and hb._limit == 5
    hb.close()


CHILD = textwrap.dedent("""
    import importlib.util, sys, time
    spec = importlib.util.spec_from_file_location("hb", {hb!r})
    hb = importlib.util.module_from_spec(spec); spec.loader.exec_module(hb)
    h = hb.Heartbeat(0, stderr_every_s=0)
    h.beat(1, "step")
    if sys.argv[1] == "hold":
        with h.hold("checkpoint_save", timeout_s=60):
            time.sleep(7)
    else:
        time.sleep(7)
    h.beat(2, "step")
""")


@pytest.mark.parametrize("mode,code", [("hold", 0), ("bare", 124)])
def test_launcher_honours_hold_limit(tmp_path, mode, code):
    script = tmp_path / "child.py"
    script.write_text(CHILD.format(hb=HB))
    env = dict(os.environ)
    env.pop("SFTAMD_HANG_TIMEOUT_S", None)
    env["PYTHONPATH"] = ROOT
    r = subprocess.run([sys.executable, "-m", "llm_fine_tune_distributed_amd.launch", "--nproc-per-node", "1",
                        "--hang-timeout", "3", "--grace", "2", str(script), mode],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == code, r.stderr[-2000:]
