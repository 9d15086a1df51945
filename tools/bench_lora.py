"""LoRA GEMM-layout microbench (SmolLM3-3B shapes, T = 8192): wide (K+R) GEMMs vs base GEMM + rank-R
updates, plus the dropout/widen kernels. Run under TunableOp tuning to compare tuned selections:
    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/lora_tune.csv \\
        python tools/bench_lora.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1000, 1)  # us


def main():
    assert _ext.load(), _ext.load_error()
    ops = _ext.ops()
    T = 8192
    for name, K, n, R in (("qkv", 2048, 3072, 48), ("o", 2048, 2048, 16), ("gate_up", 2048, 22016, 32),
                          ("down", 11008, 2048, 16)):
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        wide = torch.randn(n, K + R, device="cuda", dtype=torch.bfloat16) * 0.02
        W, Bd = wide[:, :K], wide[:, K:]
        X = torch.randn(T, K + R, device="cuda", dtype=torch.bfloat16)
        xa = X[:, K:].contiguous()
        dy = torch.randn(T, n, device="cuda", dtype=torch.bfloat16)
        Wc = W.contiguous()
        rec = {"module": name, "K": K, "n": n, "R": R}
        rec["fwd_plain_us"] = timeit(lambda: torch.mm(x, Wc.t()))
        rec["fwd_wide_us"] = timeit(lambda: torch.mm(X, wide.t()))
        rec["fwd_base_view_us"] = timeit(lambda: torch.mm(x, W.t()))
        y = torch.mm(x, W.t())
        rec["fwd_rank_update_us"] = timeit(lambda: y.addmm_(xa, Bd.t()))
        rec["dgrad_plain_us"] = timeit(lambda: torch.mm(dy, Wc))
        rec["dgrad_wide_us"] = timeit(lambda: torch.mm(dy, wide))
        rec["dgrad_base_view_us"] = timeit(lambda: torch.mm(dy, W))
        rec["dxa_skinny_us"] = timeit(lambda: torch.mm(dy, Bd))
        rec["dB_skinny_us"] = timeit(lambda: torch.mm(dy.t(), X[:, K:]))
        rec["xa_skinny_us"] = timeit(lambda: torch.mm(x, xa[:R].t() if False else W[:R].t()))
        rec["widen_drop_us"] = timeit(lambda: ops.lora_widen(x, R, 0.05, 3))
        rec["dropout_add_us"] = timeit(lambda: ops.dropout_add(X[:, :K], x, 0.05, 3))
        print(json.dumps(rec), flush=True)
        del x, wide, X, xa, dy, Wc, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
