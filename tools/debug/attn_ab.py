"""A/B of the attention backward paths on one input: the 32x32 kernels (default) vs dkdv5 + dq4
(SFTAMD_ATTN_DKDV5=1), twice each (determinism), per gradient block and per sequence."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from llm_fine_tune_distributed_amd.ops import _ext  # noqa: E402

assert _ext.load(), _ext.load_error()
ops = _ext.ops()
D = 128
for lens, nq, nkv in (([100, 255, 64, 1, 300, 129], 8, 2), ([512, 511, 7], 16, 4), ([200, 65], 12, 3)):
    torch.manual_seed(0)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    M = int(cu[-1])
    qkv = torch.randn(M, (nq + 2 * nkv) * D, device="cuda", dtype=torch.bfloat16)
    sc = 1 / math.sqrt(D)
    out, lse = ops.flash_fwd(qkv, cu, max(lens), nq, nkv, D, sc, True)
    dout = torch.randn_like(out)
    res = {}
    for cfg in ("", "1", "", "1"):
        os.environ["SFTAMD_ATTN_DKDV5"] = cfg
        res.setdefault(cfg, []).append(ops.flash_bwd(dout, qkv, out, lse, cu, max(lens), nq, nkv, D, sc, True).float())
    a, b = res[""][0], res["1"][0]
    from llm_fine_tune_distributed_amd.ops import reference as ref
    q32 = qkv.float().requires_grad_(True)
    o_ref = ref.attention(q32, nq, nkv, D, cu, sc, True)
    (g_ref,) = torch.autograd.grad(o_ref, q32, dout.float())
    for s in range(len(lens)):
        r0, r1 = int(cu[s]), int(cu[s + 1])
        eo = ((out[r0:r1].float() - o_ref[r0:r1].float()).norm() / o_ref[r0:r1].float().norm()).item()
        eg = [((a[r0:r1, sl] - g_ref[r0:r1, sl]).norm() / (g_ref[r0:r1, sl].norm() + 1e-9)).item()
              for sl in (slice(0, nq * D), slice(nq * D, (nq + nkv) * D), slice((nq + nkv) * D, None))]
        print(f"  seq {s} len {r1 - r0}: out {eo:.3g} dq/dk/dv vs fp32 {eg[0]:.3g} {eg[1]:.3g} {eg[2]:.3g}")
    print(f"lens {lens} nq {nq} nkv {nkv}: deterministic new {torch.equal(res[''][0], res[''][1])} old "
          f"{torch.equal(res['1'][0], res['1'][1])}")
    for name, sl in (("dq", slice(0, nq * D)), ("dk", slice(nq * D, (nq + nkv) * D)), ("dv", slice((nq + nkv) * D, None))):
        for s in range(len(lens)):
            r0, r1 = int(cu[s]), int(cu[s + 1])
            x, y = a[r0:r1, sl], b[r0:r1, sl]
            e = ((x - y).norm() / (y.norm() + 1e-9)).item()
            bad = (~torch.isfinite(x)).sum().item()
            if e > 1e-2 or bad:
                rows = ((x - y).abs().amax(1) > 0.05 * y.abs().max()).nonzero().flatten().tolist()
                print(f"  {name} seq {s} (len {r1 - r0}): rel {e:.3g} nonfinite {bad} bad rows {rows[:12]}")
