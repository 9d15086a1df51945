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
