"""Deployment artifacts: manifests parse, point at entry points that exist, mount what the
trainer writes, and the helper scripts are valid shell. The reference ships the equivalent PyTorchJob / Aim
manifests and kubectl scripts (deploy/*.yaml, deploy/*.sh, aim/*.yaml there)."""
import os
import subprocess

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEPLOY = os.path.join(ROOT, "deploy")


def _docs(name):
    with open(os.path.join(DEPLOY, name)) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def _containers(doc):
    return doc["spec"]["template"]["spec"]["containers"]


def test_manifests_parse_and_reference_real_entry_points():
    for name in ("job-single-node.yaml", "job-multi-node.yaml"):
        jobs = [d for d in _docs(name) if d["kind"] == "Job"]
        assert len(jobs) == 1, name
        c = _containers(jobs[0])[0]
        cmd = " ".join(c.get("command", []) + c.get("args", []))
        assert "llm_fine_tune_distributed_amd.launch" in cmd and "training.py" in cmd
        assert os.path.exists(os.path.join(ROOT, "training.py"))
        assert os.path.exists(os.path.join(ROOT, "llm_fine_tune_distributed_amd", "launch.py"))
        env = {e["name"]: e["value"] for e in c["env"]}
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"  # dmabuf IPC for RCCL across processes
        assert c["resources"]["limits"]["amd.com/gpu"] == 8
        mounts = {m["mountPath"] for m in c["volumeMounts"]}
        assert env["OUTPUT_DIR"].startswith("/persistent") and "/persistent" in mounts and "/dev/shm" in mounts
    # multi-node: node rank from the indexed Job, rendezvous on pod 0 behind the headless Service
    mn = _docs("job-multi-node.yaml")
    svc = next(d for d in mn if d["kind"] == "Service")
    job = next(d for d in mn if d["kind"] == "Job")
    assert svc["spec"]["clusterIP"] == "None" and job["spec"]["template"]["spec"]["subdomain"] == svc["metadata"]["name"]
    args = " ".join(_containers(job)[0]["args"])
    assert "--node-rank $JOB_COMPLETION_INDEX" in args and f"--nnodes {job['spec']['completions']}" in args


def test_aim_server_and_storage():
    aim = _docs(os.path.join("aim", "aim.yaml"))
    kinds = {d["kind"]: d for d in aim}
    assert set(kinds) == {"PersistentVolumeClaim", "Deployment", "Service"}
    port = _containers(kinds["Deployment"])[0]["ports"][0]["containerPort"]
    assert kinds["Service"]["spec"]["ports"][0]["targetPort"] == port == 43800
    claim = kinds["PersistentVolumeClaim"]["metadata"]["name"]
    # the trainer job mounts the same Aim volume at AIM_REPO
    job = _docs("job-single-node.yaml")[0]
    vols = {v["name"]: v for v in job["spec"]["template"]["spec"]["volumes"]}
    c = _containers(job)[0]
    aim_mount = next(m for m in c["volumeMounts"] if m["mountPath"] == "/aim")
    assert vols[aim_mount["name"]]["persistentVolumeClaim"]["claimName"] == claim
    assert {e["name"]: e["value"] for e in c["env"]}["AIM_REPO"] == "/aim"
    pvc = _docs("storage.yaml")[0]
    assert vols["models"]["persistentVolumeClaim"]["claimName"] == pvc["metadata"]["name"]


def test_scripts_are_valid_shell():
    for s in ("deploy.sh", "monitor.sh", "cleanup.sh"):
        p = os.path.join(DEPLOY, s)
        assert os.access(p, os.X_OK), s
        subprocess.run(["bash", "-n", p], check=True)
