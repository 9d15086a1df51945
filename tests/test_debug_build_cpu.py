"""The device-assert debug build: every kernel source must still compile for gfx950 with
``-DSFTAMD_DEBUG`` (``build_ext.py --debug``). Host+device syntax check only; hipcc cross-compiles without a
GPU, so this runs here."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which("g++") is None, reason="no hipcc")
def test_debug_asserts_compile():
    import torch
    tdir = os.path.dirname(torch.__file__)
    srcs = [p for p in sorted(glob.glob(os.path.join(ROOT, "csrc", "*.hip"))) if "SFT_DASSERT" in open(p).read()]
    assert len(srcs) >= 3, srcs
    inc = [f"-I{tdir}/include", f"-I{tdir}/include/torch/csrc/api/include", f"-I{ROOT}/csrc"]
    for src in srcs:
        r = subprocess.run([HIPCC, "-fsyntax-only", src, "--offload-arch=gfx950", "-O1", "-DSFTAMD_DEBUG",
                            "-std=c++17", "-DUSE_ROCM=1"] + inc, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, f"{os.path.basename(src)}:\n{r.stderr[-3000:]}"


def test_debug_library_selection(monkeypatch):
    from llm_fine_tune_distributed_amd.ops import _ext
    monkeypatch.setenv("SFTAMD_DEBUG", "1")
    assert _ext._select_lib().endswith("_C_debug.so")
    monkeypatch.setenv("SFTAMD_DEBUG", "0")
    assert _ext._select_lib().endswith(os.sep + "_C.so")
