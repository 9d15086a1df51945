"""hipBLASLt/rocBLAS kernel selection for the plain projection GEMMs (PyTorch TunableOp).

The fused/hot non-GEMM ops are hand-written HIP; the plain library GEMMs (q/k/v, o, gate/up, down,
lm_head: fwd, dgrad, wgrad) go to hipBLASLt/rocBLAS. TunableOp benchmarks every candidate solution
of both libraries per GEMM shape on the actual MI355X and records the fastest. We ship the selections
for the SmolLM3-3B training shapes in ``tuning/tunableop_results_mi355x.csv`` (produced on MI355X with
``tools/tune_gemms.sh``) and load them read-only at start-up, so no tuning happens in timed runs.
Shapes missing from the file fall back to the library default heuristics.
"""
from __future__ import annotations

import os
from typing import Optional

_DEFAULT = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tuning",
                        "tunableop_results_mi355x.csv")


def enable_tuned_gemms(path: Optional[str] = None, tune: bool = False, verbose: bool = False) -> bool:
    import torch
    if not torch.cuda.is_available():
        return False
    path = path or os.environ.get("SFTAMD_GEMM_TUNING_FILE", _DEFAULT)
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(bool(tune))
    if tune:
        tun.set_filename(path, insert_device_ordinal=False)
    else:  # read-only: no per-rank tunableop_results<N>.csv dumped into the working directory at exit
        try:
            tun.write_file_on_exit(False)
        except AttributeError:  # older torch
            pass
    ok = False
    if os.path.exists(path):
        ok = bool(tun.read_file(path))
    _TUNED[0] = _tuned_tn(path) if ok else frozenset()
    if verbose:
        print(f"[gemm] TunableOp enabled (tuning={tune}) selections={path if ok else 'none'}", flush=True)
    return ok


_TUNED = [frozenset()]


def _tuned_tn(path: str) -> frozenset:
    """(N, M, K) of every contiguous bf16 TN GEMM (y[M, N] = x[M, K] W[N, K]^T, torch's column-major naming
    ``tn_N_M_K_ld_K_K_N``) with a selection in the TunableOp file. Only ``GemmTunableOp_BFloat16_TN`` rows count: an
    fp16 / fp32 selection of the same shape says nothing about the bf16 projection. The set is read once, at
    enable_tuned_gemms: shapes tuned in-process (tune=True) route to hipBLASLt from the next start on."""
    out = set()
    try:
        with open(path) as f:
            for line in f:
                parts = line.split(",")
                if len(parts) < 2 or parts[0] != "GemmTunableOp_BFloat16_TN" or not parts[1].startswith("tn_"):
                    continue
                f_ = parts[1].split("_")  # tn, N, M, K, ld, lda, ldb, ldc
                try:
                    n, m, k, lda, ldb, ldc = (int(f_[i]) for i in (1, 2, 3, 5, 6, 7))
                except (ValueError, IndexError):
                    continue
                if lda == k and ldb == k and ldc == n:
                    out.add((n, m, k))
    except OSError:
        pass
    return frozenset(out)


def tuned_tn_shapes() -> frozenset:
    """The forward-projection GEMM shapes hipBLASLt has a TunableOp selection for (empty until enable_tuned_gemms)."""
    return _TUNED[0]
