import os, sys, json, statistics
sys.path.insert(0, os.getcwd())
import torch
from llm_fine_tune_distributed_amd.ops import _ext
from llm_fine_tune_distributed_amd.utils.gemm_tuning import enable_tuned_gemms
assert _ext.load(), _ext.load_error()
enable_tuned_gemms()
T = 8192
def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it
for name, (N, K) in {"o": (2048, 2048), "down": (2048, 11008)}.items():
    x = (0.05 * torch.randn(T, K, device="cuda")).to(torch.bfloat16)
    w = (0.02 * torch.randn(N, K, device="cuda")).to(torch.bfloat16)
    r = torch.randn(T, N, device="cuda").to(torch.bfloat16)
    res = {"mm": [], "addmm": [], "mm+add": []}
    for _ in range(7):
        res["mm"].append(t(lambda: torch.mm(x, w.t())))
        res["addmm"].append(t(lambda: torch.addmm(r, x, w.t())))
        res["mm+add"].append(t(lambda: torch.mm(x, w.t()).add_(r)))
    d = (torch.addmm(r, x, w.t()).float() - (torch.mm(x, w.t()).float() + r.float())).abs().max().item()
    print(json.dumps({"shape": name, **{k: round(statistics.median(v), 4) for k, v in res.items()}, "maxdiff": d}), flush=True)
