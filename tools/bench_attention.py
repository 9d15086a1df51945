"""Micro-benchmark of the flash-attention kernels (SmolLM3 shape: 8 x 512 tokens, 16q/4kv, d128).
Interleaves implementations in one process (CDNA guide rule 24) and reports median TFLOP/s."""
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
B, T, NQ, NKV, D = int(os.environ.get("B", 8)), int(os.environ.get("T", 512)), 16, 4, 128
M = B * T
cu = torch.arange(0, (B + 1) * T, T, dtype=torch.int32, device="cuda")
if os.environ.get("RAGGED"):  # the recipe's padding-free batches: B sequences of 553..754 tokens (mean ~621)
    g = torch.Generator().manual_seed(0)
    lens = torch.randint(553, 755, (B,), generator=g)
    T = int(lens.max())
    cu = torch.cat([torch.zeros(1, dtype=torch.long), lens.cumsum(0)]).to(torch.int32).cuda()
    M = int(lens.sum())
    print(f"ragged: {B} sequences, {M} tokens, max {T}")
qkv = torch.randn(M, (NQ + 2 * NKV) * D, device="cuda", dtype=torch.bfloat16)
dout = torch.randn(M, NQ * D, device="cuda", dtype=torch.bfloat16)
sc = 1 / math.sqrt(D)
flops_f = 4.0 * B * NQ * T * T * D / 2  # causal
if os.environ.get("RAGGED"):
    flops_f = sum(4.0 * NQ * int(n) ** 2 * D / 2 for n in (cu[1:] - cu[:-1]).tolist())
ops = _ext.ops()


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


# "ds": the default backward (materialised dS^T + dq32) incl. the delta kernel; "dsd": the same with delta given;
# "dq3": the recompute path used past the dS^T budget
CFGS = os.environ.get("CFGS", "ds,dq3").split(",")
res = {}
ref = None
for rnd in range(int(os.environ.get("ROUNDS", 3))):
    for cfg in CFGS:
        os.environ["SFTAMD_ATTN_DS_MB"] = "0" if cfg == "dq3" else ""
        out, lse = ops.flash_fwd(qkv, cu, T, NQ, NKV, D, sc, True)
        dq = ops.flash_bwd(dout, qkv, out, lse, cu, T, NQ, NKV, D, sc, True)
        if ref is None:
            ref = (out.float(), dq.float())
        else:
            eo = ((out.float() - ref[0]).norm() / ref[0].norm()).item()
            ed = ((dq.float() - ref[1]).norm() / ref[1].norm()).item()
            assert eo < 1e-2 and ed < 1e-2, (cfg, eo, ed)
        tf = timeit(lambda: ops.flash_fwd(qkv, cu, T, NQ, NKV, D, sc, True))
        # "dsd": delta precomputed (the default training path: dgrad_gemm_delta's epilogue makes it), not timed here
        dl = (dout.float() * out.float()).view(M, NQ, D).sum(-1).t().contiguous() if cfg == "dsd" else None
        tb = timeit(lambda: ops.flash_bwd(dout, qkv, out, lse, cu, T, NQ, NKV, D, sc, True, dl))
        res.setdefault(cfg, []).append((tf, tb))
for cfg, v in res.items():
    tf = statistics.median(x[0] for x in v)
    tb = statistics.median(x[1] for x in v)
    print(f"{cfg}: fwd {tf*1e3:.1f} us ({flops_f/tf/1e9:.0f} TFLOP/s)  bwd {tb*1e3:.1f} us "
          f"({2.5*flops_f/tb/1e9:.0f} TFLOP/s)")
