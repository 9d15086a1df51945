"""Host sanitizers. GPU AddressSanitizer / XNACK builds are not available on the MI355X pool, so the
native HOST code is checked here instead: the collator core (csrc/collate_core.h, the loops behind the
``sftamd::pad_batch`` / ``pack_sequences`` ops) is compiled with -fsanitize=address,undefined into a standalone
driver (tools/debug/collate_sanitize.cpp) that runs randomised corpora into exactly-sized buffers and checks the
outputs against the HF padding / packing semantics."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_collator_core_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "collate_sanitize")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "csrc"),
                    os.path.join(ROOT, "tools", "debug", "collate_sanitize.cpp"), "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "1500"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "clean" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_ddp_reducer_core_under_asan_ubsan(tmp_path):
    """The DDP bucket planner / ready tracker core (csrc/ddp_reducer_core.h, behind the ``sftamd::ddp_*`` ops) under
    AddressSanitizer + UBSan, with the layout and launch-order invariants checked on random parameter lists."""
    exe = str(tmp_path / "reducer_sanitize")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "csrc"),
                    os.path.join(ROOT, "tools", "debug", "reducer_sanitize.cpp"), "-o", exe], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe, "1500"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "clean" in r.stdout
