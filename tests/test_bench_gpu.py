"""bench.py's self-launch on the GPU box: ``python bench.py --gpus 2`` with no external launcher spawns two
ranks (sharing the one MI355X of a test box; gloo transport because RCCL refuses two ranks on one device),
runs the HIP training step on both and prints ONE JSON line with the multi-GPU diagnostics."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("zero", ["1", "0"])
def test_bench_self_launch_two_ranks_on_gpu(zero):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["SFTAMD_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "tiny-gpu",
                        "--steps", "2", "--warmup", "1", "--micro-batch", "2", "--seq", "128", "--zero", zero,
                        "--tunableop", "off"], env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(recs) == 1
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["dist"]["world_size"] == 2 and rec["dist"]["consistent"]
    assert rec["dist"]["launcher"] == "sftamd" and rec["optimizer_sharding"] == ("zero1" if zero == "1" else "none")
    assert all(p["device"].startswith("cuda") for p in rec["per_rank"])
    assert rec["value"] > 0 and rec["peak_mem_gb"] > 0 and rec["final_loss"] > 0
