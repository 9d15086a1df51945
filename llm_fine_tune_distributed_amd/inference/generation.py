"""KV-cache text generation (reference I1/I2: ``model.generate`` in ask_tuned_model.py:55-65).

Prefill runs the training kernels (fused RMSNorm, packed QKV GEMM, in-place RoPE, the varlen
flash-attention forward) over the prompt and stores K/V in a preallocated cache sized for the
whole generation (288 GB of HBM: no paging needed at this scale). On the GPU the decode step is
shape-static — the token, its position and the live cache length sit in device tensors, the KV
append is an ``index_copy_`` and attention is the HIP split-K decode kernel that reads the
length from device memory — so ONE decode step is captured into a hipGraph and replayed per
token (no per-layer launch overhead, no host sync inside the step). On CPU the same step runs
eagerly. Sampling matches HF's logits-processor order: repetition penalty -> temperature ->
top-k -> top-p -> multinomial.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch

from .. import ops


class KVCache:
    def __init__(self, cfg, max_len: int, device, dtype=torch.bfloat16):
        L = cfg.num_hidden_layers
        self.k = torch.empty(L, max_len, cfg.num_key_value_heads, cfg.head_dim, device=device, dtype=dtype)
        self.v = torch.empty_like(self.k)
        self.len = 0


@torch.no_grad()
def _layer(model, li, x, residual, cache: KVCache, pos: torch.Tensor, prefill: bool):
    cfg = model.config
    layer = model.model.layers[li]
    at = layer.self_attn
    nq, nkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    h, residual = ops.add_rms_norm(x, residual, layer.input_layernorm.weight, cfg.rms_norm_eps)
    qkv = ops.linear(h, at.qkv_proj) if at.lora is None else ops.lora_linear(h, at.qkv_proj, at.lora["qkv"])
    if at.use_rope:
        cos, sin = model.rope_tables(pos)
        ops.rope_(qkv, cos, sin, nq, nkv, D)
    M = qkv.shape[0]
    k = qkv[:, nq * D:(nq + nkv) * D].view(M, nkv, D)
    v = qkv[:, (nq + nkv) * D:].view(M, nkv, D)
    s = cache.len
    cache.k[li, s:s + M] = k
    cache.v[li, s:s + M] = v
    if prefill:
        cu = torch.tensor([0, M], dtype=torch.int32, device=x.device)
        a = ops.flash_attention(qkv.contiguous(), cu, M, nq, nkv, D)
    else:
        q = qkv[:, :nq * D].view(nq, D).float()
        K = cache.k[li, :s + 1].float()  # [S, nkv, D]
        V = cache.v[li, :s + 1].float()
        rep = nq // nkv
        qg = q.view(nkv, rep, D)
        att = torch.einsum("grd,sgd->grs", qg, K) / math.sqrt(D)
        p = att.softmax(-1)
        a = torch.einsum("grs,sgd->grd", p, V).reshape(1, nq * D).to(x.dtype)
    o = ops.linear(a, at.o_proj) if at.lora is None else ops.lora_linear(a, at.o_proj, at.lora["o"])
    h, residual = ops.add_rms_norm(o, residual, layer.post_attention_layernorm.weight, cfg.rms_norm_eps)
    return layer.mlp(h), residual


@torch.no_grad()
def forward_cached(model, ids: torch.Tensor, cache: KVCache, prefill: bool) -> torch.Tensor:
    """ids: [M] tokens appended at positions cache.len ... Returns last-token logits [V] (fp32)."""
    M = ids.numel()
    pos = torch.arange(cache.len, cache.len + M, device=ids.device)
    x = ops.embedding(ids, model.model.embed_tokens)
    residual = None
    for li in range(model.config.num_hidden_layers):
        x, residual = _layer(model, li, x, residual, cache, pos, prefill)
    cache.len += M
    n = model.model.norm
    h, _ = ops.add_rms_norm(x[-1:], residual[-1:], n.weight, model.config.rms_norm_eps)
    return torch.nn.functional.linear(h, model.lm_head_weight).float()[0]


def sample_next(logits: torch.Tensor, history: torch.Tensor, temperature: float = 0.6, top_k: int = 40,
                top_p: float = 0.95, repetition_penalty: float = 1.1, do_sample: bool = True,
                generator: Optional[torch.Generator] = None) -> int:
    logits = logits.clone()
    if repetition_penalty and repetition_penalty != 1.0 and history.numel():
        sc = logits[history]
        logits[history] = torch.where(sc < 0, sc * repetition_penalty, sc / repetition_penalty)
    if not do_sample:
        return int(logits.argmax())
    logits = logits / max(temperature, 1e-5)
    if top_k and top_k > 0:
        kth = torch.topk(logits, min(top_k, logits.numel())).values[-1]
        logits[logits < kth] = -float("inf")
    if top_p is not None and top_p < 1.0:
        sl, si = torch.sort(logits, descending=True)
        cp = sl.softmax(-1).cumsum(-1)
        remove = cp > top_p
        remove[1:] = remove[:-1].clone()
        remove[0] = False
        logits[si[remove]] = -float("inf")
    p = logits.softmax(-1)
    return int(torch.multinomial(p, 1, generator=generator))


class DeviceSampler:
    """GPU-resident sampling state of one sequence for the fused HIP sampler (csrc/sampler.hip): the
    history as a presence bitmask (repetition penalty is a set operation), a step counter that keys the
    counter-based RNG, the running position / KV length, and a device log of the generated tokens."""

    def __init__(self, vocab_size: int, device, history_ids, max_new_tokens: int, seed: Optional[int],
                 temperature: float, top_k: int, top_p: Optional[float], repetition_penalty: float, do_sample: bool):
        import numpy as np
        words = np.zeros((vocab_size + 31) // 32, dtype=np.uint32)
        ids = np.asarray(list(history_ids), dtype=np.int64)
        np.bitwise_or.at(words, ids >> 5, (np.uint32(1) << (ids & 31).astype(np.uint32)))
        self.presence = torch.from_numpy(words.view(np.int32).copy()).to(device)
        self.state = torch.zeros(4, dtype=torch.long, device=device)
        self.log = torch.full((max(1, max_new_tokens),), -1, dtype=torch.long, device=device)
        self.params = (float(temperature), int(top_k) if do_sample else 1, float(top_p if top_p is not None else 1.0),
                       float(repetition_penalty or 1.0), bool(do_sample),
                       int(seed if seed is not None else torch.randint(0, 2 ** 31 - 1, (1,)).item()))

    @staticmethod
    def supported(top_k: int, do_sample: bool) -> bool:
        return (not do_sample) or (top_k is not None and 1 <= top_k <= 64)

    def sample(self, logits: torch.Tensor, tok_out=None, pos_out=None, len_out=None) -> None:
        t, k, p, rp, ds, seed = self.params
        ops_ext().sample_token(logits.contiguous(), self.presence, self.state, tok_out, pos_out, len_out, self.log,
                               t, k, p, rp, ds, seed)


def ops_ext():
    from ..ops import _ext
    return _ext.ops()


class GraphDecoder:
    """Static-shape decode step over a KVCache, captured once into a hipGraph (GPU)."""

    def __init__(self, model, cache: KVCache):
        self.model, self.cache = model, cache
        dev = model.model.embed_tokens.device
        self.tok = torch.zeros(1, dtype=torch.long, device=dev)
        self.pos = torch.zeros(1, dtype=torch.long, device=dev)
        self.len = torch.ones(1, dtype=torch.int32, device=dev)
        self.graph = None
        self.logits = None

    @torch.no_grad()
    def _step(self) -> torch.Tensor:
        m, cfg = self.model, self.model.config
        nq, nkv, D = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
        x = ops.embedding(self.tok, m.model.embed_tokens)
        residual = None
        cos = sin = None
        for li, layer in enumerate(m.model.layers):
            at = layer.self_attn
            h, residual = ops.add_rms_norm(x, residual, layer.input_layernorm.weight, cfg.rms_norm_eps)
            qkv = ops.linear(h, at.qkv_proj) if at.lora is None else ops.lora_linear(h, at.qkv_proj, at.lora["qkv"])
            if at.use_rope:
                if cos is None:
                    cos, sin = m.rope_tables(self.pos)
                ops.rope_(qkv, cos, sin, nq, nkv, D)
            self.cache.k[li].index_copy_(0, self.pos, qkv[:, nq * D:(nq + nkv) * D].view(1, nkv, D))
            self.cache.v[li].index_copy_(0, self.pos, qkv[:, (nq + nkv) * D:].view(1, nkv, D))
            a = ops.decode_attention(qkv[0, :nq * D].contiguous(), self.cache.k[li], self.cache.v[li], self.len,
                                     nq, nkv).view(1, nq * D)
            o = ops.linear(a, at.o_proj) if at.lora is None else ops.lora_linear(a, at.o_proj, at.lora["o"])
            h, residual = ops.add_rms_norm(o, residual, layer.post_attention_layernorm.weight, cfg.rms_norm_eps)
            x = layer.mlp(h)
        n = m.model.norm
        h, _ = ops.add_rms_norm(x, residual, n.weight, cfg.rms_norm_eps)
        return torch.nn.functional.linear(h, m.lm_head_weight).float()[0]

    def run_sampled(self, sampler: DeviceSampler, n: int, use_graph: bool = True) -> None:
        """n decode steps entirely on the device: each step runs the model on self.tok at self.pos and the
        fused sampler writes the next token / position / KV length back into the step's inputs (one
        hipGraph holds both, so consecutive replays need no host involvement)."""
        def body():
            logits = self._step()
            sampler.sample(logits, self.tok, self.pos, self.len)
        if not use_graph:
            for _ in range(n):
                body()
            return
        if self.graph is None:
            # warm up on copies of the counters so the real sequence state is untouched
            saved = [t.clone() for t in (self.tok, self.pos, self.len, sampler.state, sampler.presence, sampler.log)]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    body()
            torch.cuda.current_stream().wait_stream(s)
            for t, v in zip((self.tok, self.pos, self.len, sampler.state, sampler.presence, sampler.log), saved):
                t.copy_(v)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                body()
        for _ in range(n):
            self.graph.replay()

    def step(self, token: int, position: int, use_graph: bool = True) -> torch.Tensor:
        self.tok.fill_(token)
        self.pos.fill_(position)
        self.len.fill_(position + 1)
        if not use_graph:
            return self._step()
        if self.graph is None:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):  # warm up allocator / kernels outside capture
                    self._step()
            torch.cuda.current_stream().wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.logits = self._step()
        self.graph.replay()
        return self.logits


@torch.no_grad()
def generate(model, prompt_ids: List[int], max_new_tokens: int = 256, eos_token_id: Optional[int] = None,
             temperature: float = 0.6, top_k: int = 40, top_p: float = 0.95, repetition_penalty: float = 1.1,
             do_sample: bool = True, seed: Optional[int] = None, use_graph: Optional[bool] = None,
             device_sampling: Optional[bool] = None) -> List[int]:
    model.eval()
    dev = model.model.embed_tokens.device
    cache = KVCache(model.config, len(prompt_ids) + max_new_tokens + 1, dev, model.model.embed_tokens.dtype)
    g = torch.Generator(device=dev).manual_seed(seed) if seed is not None else None
    ids = torch.tensor(prompt_ids, device=dev)
    logits = forward_cached(model, ids, cache, prefill=True)
    gpu_path = dev.type == "cuda" and model.config.head_dim == 128 and ops.use_hip(ids)
    dec = GraphDecoder(model, cache) if gpu_path else None
    graph = gpu_path if use_graph is None else (use_graph and gpu_path)
    if device_sampling is None:
        device_sampling = DeviceSampler.supported(top_k, do_sample)
    if gpu_path and max_new_tokens > 0 and device_sampling:
        return _generate_device(model, dec, cache, prompt_ids, logits, max_new_tokens, eos_token_id, temperature, top_k,
                                top_p, repetition_penalty, do_sample, seed, graph)
    hist = ids.clone()
    out: List[int] = []
    for _ in range(max_new_tokens):
        t = sample_next(logits, hist, temperature, top_k, top_p, repetition_penalty, do_sample, g)
        out.append(t)
        if eos_token_id is not None and t == eos_token_id:
            break
        nt = torch.tensor([t], device=dev)
        hist = torch.cat([hist, nt])
        if dec is not None:
            logits = dec.step(t, cache.len, use_graph=graph).clone()
            cache.len += 1
        else:
            logits = forward_cached(model, nt, cache, prefill=False)
    return out


def _generate_device(model, dec: GraphDecoder, cache: KVCache, prompt_ids, logits, max_new_tokens, eos_token_id,
                     temperature, top_k, top_p, repetition_penalty, do_sample, seed, use_graph, check_every: int = 16):
    """Decode loop with sampling on the device (fused HIP sampler inside the decode hipGraph). The host
    only reads the token log every ``check_every`` steps to stop at EOS."""
    dev = model.model.embed_tokens.device
    sm = DeviceSampler(model.config.vocab_size, dev, prompt_ids, max_new_tokens, seed, temperature, top_k, top_p,
                       repetition_penalty, do_sample)
    sm.state[2] = cache.len - 1  # the first sampled token gets position len(prompt)
    sm.sample(logits, dec.tok, dec.pos, dec.len)  # token 1 from the prefill logits
    done = 1
    out: List[int] = []
    while True:
        if eos_token_id is not None or done >= max_new_tokens:
            toks = sm.log[:done].tolist()
            if eos_token_id is not None and eos_token_id in toks:
                out = toks[:toks.index(eos_token_id) + 1]
                break
            if done >= max_new_tokens:
                out = toks
                break
        n = min(check_every, max_new_tokens - done)
        dec.run_sampled(sm, n, use_graph=use_graph)
        done += n
    cache.len = len(prompt_ids) + len(out)
    return out
