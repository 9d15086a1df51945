#!/bin/bash
# cross-entropy with the VALU-lean passes: numerics tests + standalone timing at the bench's [8192, 128256]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py -k "cross_entropy or ce or lm_head or loss" \
  > gpurun_out/r3_53_test.log 2>&1 || { tail -40 gpurun_out/r3_53_test.log; exit 1; }
tail -1 gpurun_out/r3_53_test.log
timeout -k 10 120 python -u - > gpurun_out/r3_53_t.log 2>&1 <<'PY' || { tail -20 gpurun_out/r3_53_t.log; exit 1; }
import torch, statistics
from llm_fine_tune_distributed_amd.ops import _ext
assert _ext.load(), _ext.load_error()
M, V = 8192, 128256
lg0 = (3 * torch.randn(M, V, device="cuda")).to(torch.bfloat16)
lab = torch.randint(0, V, (M,), device="cuda")
inv = torch.tensor([1.0 / M], device="cuda")
ts = []
for it in range(12):
    lg = lg0.clone()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record(); _ext.ops().ce_fwd(lg, lab, inv, True); e.record(); torch.cuda.synchronize()
    if it >= 2: ts.append(s.elapsed_time(e))
print(f"ce_fwd [8192 x 128256] write_grad: {statistics.median(ts):.3f} ms (median of 10)")
PY
cat gpurun_out/r3_53_t.log | grep ce_fwd
