"""hipGraph-captured decode == eager decode == full re-forward (greedy) on MI355X."""
import pytest
import torch

from llm_fine_tune_distributed_amd.inference.generation import generate
from llm_fine_tune_distributed_amd.models import build_model, tiny

pytestmark = pytest.mark.gpu


def test_graph_decode_matches_eager():
    torch.manual_seed(0)
    cfg = tiny(hidden_size=512, num_attention_heads=4, num_key_value_heads=2, head_dim=128, intermediate_size=1024,
               vocab_size=1024, num_hidden_layers=4)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=3)
    prompt = torch.randint(0, 1024, (37,)).tolist()
    a = generate(m, prompt, max_new_tokens=12, do_sample=False, repetition_penalty=1.0, use_graph=True)
    b = generate(m, prompt, max_new_tokens=12, do_sample=False, repetition_penalty=1.0, use_graph=False)
    assert a == b
    seq = list(prompt)
    for _ in range(4):
        with torch.no_grad():
            lg = m(torch.tensor(seq, device="cuda")[None], return_logits=True).logits
        seq.append(int(lg[-1].float().argmax()))
    assert a[:4] == seq[len(prompt):]


def test_device_sampling_greedy_matches_host():
    torch.manual_seed(0)
    cfg = tiny(hidden_size=512, num_attention_heads=4, num_key_value_heads=2, head_dim=128, intermediate_size=1024,
               vocab_size=1024, num_hidden_layers=2)
    m = build_model(cfg, device="cuda", dtype=torch.bfloat16, seed=5)
    prompt = torch.randint(0, 1024, (21,)).tolist()
    for rp in (1.0, 1.3):
        host = generate(m, prompt, max_new_tokens=40, do_sample=False, repetition_penalty=rp, device_sampling=False)
        dev = generate(m, prompt, max_new_tokens=40, do_sample=False, repetition_penalty=rp, device_sampling=True)
        eager = generate(m, prompt, max_new_tokens=40, do_sample=False, repetition_penalty=rp, device_sampling=True,
                         use_graph=False)
        assert dev == host == eager
    # EOS stops the device loop at the same place
    eos = host[7]
    d2 = generate(m, prompt, max_new_tokens=40, do_sample=False, repetition_penalty=1.3, device_sampling=True,
                  eos_token_id=eos)
    h2 = generate(m, prompt, max_new_tokens=40, do_sample=False, repetition_penalty=1.3, device_sampling=False,
                  eos_token_id=eos)
    assert d2 == h2 and d2[-1] == eos


def test_fused_sampler_distribution():
    """Frequencies of the fused sampler over many draws match penalty -> temperature -> top-k -> top-p
    softmax computed in PyTorch (same rules as generation.sample_next)."""
    from llm_fine_tune_distributed_amd.ops import _ext
    torch.manual_seed(0)
    V, K, T, P, RP = 5000, 12, 0.7, 0.9, 1.2
    logits = torch.randn(V, device="cuda") * 2
    hist = torch.tensor([3, 17, 17, 400], device="cuda")
    logits[hist] += 3.0  # make the penalised tokens competitive
    import numpy as np
    words = np.zeros((V + 31) // 32, dtype=np.uint32)
    for t in hist.tolist():
        words[t >> 5] |= np.uint32(1 << (t & 31))
    base = torch.from_numpy(words.view(np.int32).copy()).cuda()
    # reference distribution
    lg = logits.clone()
    sc = lg[hist]
    lg[hist] = torch.where(sc < 0, sc * RP, sc / RP)
    lg = lg / T
    kth = torch.topk(lg, K).values[-1]
    lg[lg < kth] = -float("inf")
    sl, si = torch.sort(lg, descending=True)
    cp = sl.softmax(-1).cumsum(-1)
    rem = cp > P
    rem[1:] = rem[:-1].clone()
    rem[0] = False
    lg[si[rem]] = -float("inf")
    pref = lg.softmax(-1)
    state = torch.zeros(4, dtype=torch.long, device="cuda")
    n = 6000
    counts = torch.zeros(V, device="cuda")
    for _ in range(n):
        pres = base.clone()
        _ext.ops().sample_token(logits, pres, state, None, None, None, None, T, K, P, RP, True, 1234)
        counts[state[1]] += 1
    assert int(state[0]) == n
    freq = counts / n
    support = pref > 0
    assert (freq[~support] == 0).all()
    assert (freq - pref).abs().max().item() < 0.03
    # greedy = argmax of the penalised logits
    g_state = torch.zeros(4, dtype=torch.long, device="cuda")
    _ext.ops().sample_token(logits.to(torch.bfloat16), base.clone(), g_state, None, None, None, None, T, K, P, RP,
                            False, 0)
    lgb = logits.to(torch.bfloat16).float()
    sc = lgb[hist]
    lgb[hist] = torch.where(sc < 0, sc * RP, sc / RP)
    assert int(g_state[1]) == int(lgb.argmax())
