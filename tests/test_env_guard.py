"""The test session must run the shipped default dispatch: no SFTAMD_* override may be set when it starts (the
GPU kernels read several of them per call, csrc/attention.hip attn_impl() and friends). conftest.py restores the
environment after every test, so overrides a test sets stay inside that test."""
import os

from conftest import START_SFTAMD_ENV


def test_no_dispatch_overrides_at_session_start():
    assert not START_SFTAMD_ENV, f"SFTAMD_* set when the session started: {sorted(START_SFTAMD_ENV)}"


def test_environment_restored_between_tests_part1():
    os.environ["SFTAMD_ENV_GUARD_PROBE"] = "1"


def test_environment_restored_between_tests_part2():
    assert "SFTAMD_ENV_GUARD_PROBE" not in os.environ
