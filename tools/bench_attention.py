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


# suffix ",serial": dq3 after dK/dV on one stream; ",ds": v4 backward (materialised dS^T + dq4, the default)
# ",ds,perhead": the v4 backward with per-query-head dK/dV + fp32 partials + reduce (SFTAMD_ATTN_GQA=0)
CFGS = [("1", ""), ("2", "8,1"), ("3", "8,1"), ("3", "4,1"), ("4", ""), ("3", "8,1,serial"), ("3", "8,1,ds"),
        ("3", "8,1,ds,perhead")]
if os.environ.get("ATTN_QUICK"):
    CFGS = [("3", "8,1,serial"), ("3", "8,1,ds,perhead"), ("3", "8,1,ds,nosplit"), ("3", "8,1,ds")]
if os.environ.get("ATTN_FWD"):  # ",fwd6": the GQA-stacked v6 forward (SFTAMD_ATTN_FWD6=1); ",dq6": v6 backward
    CFGS = [("3", "8,1,ds"), ("3", "8,1,ds,fwd6"), ("3", "8,1,ds,fwd6,dq6")]
if os.environ.get("ATTN_LEG"):  # ",leg": the round-2 instruction schedule (SFTAMD_ATTN_LEGWAIT=1) vs the default
    CFGS = [("3", "8,1,ds,leg"), ("3", "8,1,ds"), ("3", "8,1,ds,dma3")]
res = {}
ref = None
for rnd in range(int(os.environ.get("ROUNDS", 3))):
    for impl, cfg in CFGS:
        os.environ["SFTAMD_ATTN_IMPL"] = impl
        os.environ["SFTAMD_ATTN_GQA"] = "0" if cfg.endswith(",perhead") else "1"
        os.environ["SFTAMD_ATTN_GQA_SPLIT"] = "0" if cfg.endswith(",nosplit") else "1"
        os.environ["SFTAMD_ATTN_FWD6"] = "1" if ",fwd6" in cfg else "0"
        os.environ["SFTAMD_ATTN_DQ6"] = "1" if ",dq6" in cfg else "0"
        os.environ["SFTAMD_ATTN_LEGWAIT"] = "1" if ",leg" in cfg else "0"
        os.environ["SFTAMD_ATTN_FWD7"] = "1" if ",fwd7" in cfg else "0"
        os.environ["SFTAMD_ATTN_FWD_DMA3"] = "1" if ",dma3" in cfg else "0"
        os.environ["SFTAMD_ATTN_FWD_DMA"] = "0" if ",nodma" in cfg else "1"
        os.environ["SFTAMD_ATTN_BWD_DMA"] = "0" if ",nodma" in cfg or ",nobdma" in cfg else "1"
        tag = cfg
        cfg = cfg.replace(",leg", "").replace(",nodma", "").replace(",nobdma", "").replace(",fwd7", "").replace(",dma3", "").replace(",perhead", "").replace(",nosplit", "").replace(",fwd6", "").replace(",dq6", "")
        os.environ["SFTAMD_ATTN_CFG"] = cfg.replace(",serial", "").replace(",ds", "")
        os.environ["SFTAMD_ATTN_CONC"] = "0" if cfg.endswith("serial") or cfg.endswith("ds") else "1"
        os.environ["SFTAMD_ATTN_DS_MB"] = "" if cfg.endswith("ds") else "0"
        out, lse = ops.flash_fwd(qkv, cu, T, NQ, NKV, D, sc, True)
        dq = ops.flash_bwd(dout, qkv, out, lse, cu, T, NQ, NKV, D, sc, True)
        if ref is None:
            ref = (out.float(), dq.float())
        else:
            eo = ((out.float() - ref[0]).norm() / ref[0].norm()).item()
            ed = ((dq.float() - ref[1]).norm() / ref[1].norm()).item()
            assert eo < 1e-2 and ed < 1e-2, (impl, cfg, eo, ed)
        tf = timeit(lambda: ops.flash_fwd(qkv, cu, T, NQ, NKV, D, sc, True))
        tb = timeit(lambda: ops.flash_bwd(dout, qkv, out, lse, cu, T, NQ, NKV, D, sc, True))
        res.setdefault(impl + ":" + tag, []).append((tf, tb))
for impl, v in res.items():
    tf = statistics.median(x[0] for x in v)
    tb = statistics.median(x[1] for x in v)
    print(f"impl {impl}: fwd {tf*1e3:.1f} us ({flops_f/tf/1e9:.0f} TFLOP/s)  bwd {tb*1e3:.1f} us "
          f"({2.5*flops_f/tb/1e9:.0f} TFLOP/s)")
