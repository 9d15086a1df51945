"""Loader for the in-tree HIP extension (``csrc/*.hip`` -> ``_C.so``, gfx950).

The extension registers its kernels as torch custom ops in the ``sftamd`` namespace
(``torch.ops.sftamd.*``). It is built by ``build_ext.py`` (``__graft_entry__.build``).

Policy: on a GPU process the HIP path is *mandatory* — if the .so is missing or fails to
load and a CUDA(HIP) tensor reaches an op, we raise instead of silently running the
PyTorch reference (set ``SFTAMD_ALLOW_FALLBACK=1`` to opt in to the fallback, or
``SFTAMD_DISABLE_HIP=1`` to force the reference path for A/B numerics). ``SFTAMD_DEBUG=1`` loads
``_C_debug.so`` instead (``build_ext.py --debug``: -O1 -g, device asserts on).
"""
from __future__ import annotations

import os
import threading

import torch

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _select_lib() -> str:
    if os.environ.get("SFTAMD_LIB"):  # an alternative build (A/B tooling: tools/bench_attention.py old vs new)
        return os.path.abspath(os.environ["SFTAMD_LIB"])
    return os.path.join(_PKG, "_C_debug.so" if os.environ.get("SFTAMD_DEBUG", "0") == "1" else "_C.so")


_LIB_PATH = _select_lib()
_lock = threading.Lock()
_loaded = None  # None = not tried, True/False afterwards
_error = None


def lib_path() -> str:
    return _LIB_PATH


def load() -> bool:
    global _loaded, _error
    if _loaded is not None:
        return _loaded
    with _lock:
        if _loaded is not None:
            return _loaded
        if not os.path.exists(_LIB_PATH):
            flag = " --debug" if _LIB_PATH.endswith("_debug.so") else ""
            _loaded, _error = False, f"extension not built: {_LIB_PATH} (run python build_ext.py{flag})"
            return False
        try:
            torch.ops.load_library(_LIB_PATH)
            _loaded = True
        except Exception as e:  # pragma: no cover - depends on environment
            _loaded, _error = False, f"failed to load {_LIB_PATH}: {e}"
    return _loaded


def load_error() -> str | None:
    load()
    return _error


def hip_disabled() -> bool:
    return os.environ.get("SFTAMD_DISABLE_HIP", "0") == "1"


def use_hip(t: torch.Tensor) -> bool:
    """True if the HIP kernel must be used for tensor ``t``.

    CPU tensors always take the reference path. GPU tensors take the HIP path unless it is
    explicitly disabled; a missing extension on a GPU is an error unless fallback is allowed.
    """
    if not t.is_cuda or hip_disabled():
        return False
    if load():
        return True
    if os.environ.get("SFTAMD_ALLOW_FALLBACK", "0") == "1":
        return False
    raise RuntimeError(f"HIP extension required on GPU but unavailable: {_error}")


def ops():
    load()
    return torch.ops.sftamd
