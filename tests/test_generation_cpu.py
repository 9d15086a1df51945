"""KV-cache decode == full re-forward (greedy), sampling processors."""
import torch

from llm_fine_tune_distributed_amd.inference.generation import generate, sample_next
from llm_fine_tune_distributed_amd.models import build_model, tiny


def test_greedy_cache_matches_full_forward():
    torch.manual_seed(0)
    m = build_model(tiny(), dtype=torch.float32, seed=2)
    prompt = torch.randint(0, 512, (9,)).tolist()
    out = generate(m, prompt, max_new_tokens=6, do_sample=False, repetition_penalty=1.0)
    seq = list(prompt)
    for _ in range(6):
        with torch.no_grad():
            lg = m(torch.tensor(seq)[None], return_logits=True).logits
        seq.append(int(lg[-1].argmax()))
    assert out == seq[len(prompt):]


def test_sampling_processors():
    lg = torch.tensor([1.0, 5.0, 3.0, 4.9, -2.0])
    assert sample_next(lg, torch.tensor([], dtype=torch.long), do_sample=False) == 1
    # repetition penalty demotes token 1 below token 3
    assert sample_next(lg, torch.tensor([1]), repetition_penalty=1.1, do_sample=False) == 3
    g = torch.Generator().manual_seed(0)
    picks = {sample_next(lg, torch.tensor([], dtype=torch.long), top_k=2, generator=g) for _ in range(50)}
    assert picks <= {1, 3}


def test_static_decoder_matches_cached_forward_cpu():
    from llm_fine_tune_distributed_amd.inference.generation import GraphDecoder, KVCache, forward_cached
    torch.manual_seed(0)
    m = build_model(tiny(), dtype=torch.float32, seed=2)
    prompt = torch.randint(0, 512, (7,))
    c1 = KVCache(m.config, 16, "cpu", torch.float32)
    c2 = KVCache(m.config, 16, "cpu", torch.float32)
    forward_cached(m, prompt, c1, prefill=True)
    forward_cached(m, prompt, c2, prefill=True)
    dec = GraphDecoder(m, c2)
    for t in (5, 9, 11):
        a = forward_cached(m, torch.tensor([t]), c1, prefill=False)
        b = dec.step(t, c2.len, use_graph=False)
        c2.len += 1
        assert torch.allclose(a, b, atol=1e-4)
