"""HF-compatible checkpoints and resume (reference T10/T11).

* ``save_pretrained``: ``model.safetensors`` (or ``model-0000i-of-0000N.safetensors`` shards of
  at most ``max_shard_size`` + ``model.safetensors.index.json``), HF key names, the tied lm_head
  deduplicated, ``config.json`` and ``generation_config.json``. Written to a temp dir and renamed
  (atomic), rank 0 only.
* ``save_checkpoint`` adds ``optimizer.pt`` (Adam moments / fp32 master keyed by parameter name, so it
  resumes at any world size; gathered from the ZeRO-1 shards by every rank), ``scheduler.pt``,
  per-rank ``rng_state_{rank}.pth``, ``trainer_state.json`` and ``training_args.json`` under
  ``checkpoint-{step}/``; ``rotate_checkpoints`` keeps ``save_total_limit`` (never the best one).
* ``load_checkpoint`` restores everything for ``resume_from_checkpoint`` (``"auto"`` = latest).
"""
from __future__ import annotations

import json
import os
import random
import re
import shutil
from typing import Dict, Optional

import numpy as np
import torch

GEN_CONFIG = {"do_sample": True, "temperature": 0.6, "top_p": 0.95, "top_k": 40, "repetition_penalty": 1.1,
              "max_new_tokens": 3768}  # ask_tuned_model.py:55-65 decode settings


def _atomic_dir(path: str) -> str:
    tmp = path.rstrip("/") + ".tmp"
    if os.path.exists(tmp):
        shutil.rmtree(tmp)
    os.makedirs(tmp)
    return tmp


def _commit_dir(tmp: str, path: str):
    if os.path.exists(path):
        old = path.rstrip("/") + ".old"
        if os.path.exists(old):
            shutil.rmtree(old)
        os.rename(path, old)
        os.rename(tmp, path)
        shutil.rmtree(old)
    else:
        os.rename(tmp, path)


def save_state_dict_sharded(sd: Dict[str, torch.Tensor], path: str, max_shard_size: int = 5 * 1024 ** 3):
    from safetensors.torch import save_file
    tensors = {k: v.detach().contiguous().cpu() for k, v in sd.items()}
    shards, cur, cur_sz = [], {}, 0
    for k, v in tensors.items():
        sz = v.numel() * v.element_size()
        if cur and cur_sz + sz > max_shard_size:
            shards.append(cur)
            cur, cur_sz = {}, 0
        cur[k] = v
        cur_sz += sz
    if cur:
        shards.append(cur)
    meta = {"format": "pt"}
    if len(shards) == 1:
        save_file(shards[0], os.path.join(path, "model.safetensors"), metadata=meta)
        return
    wmap, total = {}, 0
    for i, sh in enumerate(shards):
        name = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
        save_file(sh, os.path.join(path, name), metadata=meta)
        for k, v in sh.items():
            wmap[k] = name
            total += v.numel() * v.element_size()
    with open(os.path.join(path, "model.safetensors.index.json"), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": wmap}, f, indent=2)


def load_state_dict(path: str, device="cpu") -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            files = sorted(set(json.load(f)["weight_map"].values()))
        sd = {}
        for fn in files:
            sd.update(load_file(os.path.join(path, fn), device=str(device)))
        return sd
    return load_file(os.path.join(path, "model.safetensors"), device=str(device))


@torch.no_grad()
def _merged_lora_state_dict(model, sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    cfg = model.config
    sd = dict(sd)
    for i, l in enumerate(model.model.layers):
        p = f"model.layers.{i}."
        a, m = l.self_attn, l.mlp
        if getattr(a, "lora", None) is not None:
            w = a.qkv_proj.detach() + a.lora["qkv"].delta_weight().to(a.qkv_proj.dtype)
            q, k, v = w.split([cfg.q_size, cfg.kv_size, cfg.kv_size], 0)
            sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"] = q, k
            sd[p + "self_attn.v_proj.weight"] = v
            sd[p + "self_attn.o_proj.weight"] = a.o_proj.detach() + a.lora["o"].delta_weight().to(a.o_proj.dtype)
        if getattr(m, "lora", None) is not None:
            w = m.gate_up_proj.detach() + m.lora["gate_up"].delta_weight().to(m.gate_up_proj.dtype)
            g, u = w.split([cfg.intermediate_size] * 2, 0)
            sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"] = g, u
            sd[p + "mlp.down_proj.weight"] = m.down_proj.detach() + m.lora["down"].delta_weight().to(m.down_proj.dtype)
    return sd


def save_pretrained(model, path: str, tokenizer=None, max_shard_size: int = 5 * 1024 ** 3, merge_lora: bool = False):
    """HF layout: safetensors + config.json + generation_config.json (+ tokenizer files). LoRA models write
    the base weights plus ``adapter_model.safetensors``; ``merge_lora=True`` writes merged weights instead."""
    from ..models.lora import lora_state_dict
    tmp = _atomic_dir(path)
    lora = any(getattr(l.self_attn, "lora", None) is not None or getattr(l.mlp, "lora", None) is not None
               for l in model.model.layers)
    sd = model.hf_state_dict()
    if lora and merge_lora:  # export: adapters folded into copies of the base weights (the model keeps them)
        sd = _merged_lora_state_dict(model, sd)
        lora = False
    save_state_dict_sharded(sd, tmp, max_shard_size)
    if lora:
        from safetensors.torch import save_file
        save_file({k: v.contiguous().cpu() for k, v in lora_state_dict(model).items()},
                  os.path.join(tmp, "adapter_model.safetensors"))
        lc = getattr(model, "_lora_config", None)
        if lc is not None:
            with open(os.path.join(tmp, "adapter_config.json"), "w") as f:
                json.dump({"peft_type": "LORA", "r": lc.r, "lora_alpha": lc.lora_alpha, "lora_dropout": lc.lora_dropout,
                           "target_modules": lc.target_modules, "task_type": "CAUSAL_LM"}, f, indent=2)
    model.config.save_pretrained(tmp)
    gc = dict(GEN_CONFIG)
    gc.update({"eos_token_id": model.config.eos_token_id, "bos_token_id": model.config.bos_token_id,
               "pad_token_id": model.config.pad_token_id})
    with open(os.path.join(tmp, "generation_config.json"), "w") as f:
        json.dump(gc, f, indent=2)
    if tokenizer is not None:
        tokenizer.save_pretrained(tmp)
    _commit_dir(tmp, path)


def from_pretrained(path: str, device="cpu", dtype=torch.bfloat16):
    from ..models import ModelConfig, build_model
    cfg = ModelConfig.from_pretrained(path)
    m = build_model(cfg, device=device, dtype=dtype)
    m.load_hf_state_dict({k: v.to(dtype) for k, v in load_state_dict(path, device).items()}, strict=False)
    return m


# ---------------------------------------------------------------------------- trainer checkpoints
def rng_state() -> Dict:
    pv, pst, pg = random.getstate()
    nk, nkeys, npos, nhg, ncg = np.random.get_state()
    st = {"python": [pv, list(pst), pg], "numpy": [nk, torch.from_numpy(np.asarray(nkeys).astype(np.int64)), int(npos),
                                                   int(nhg), float(ncg)], "cpu": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state()
    return st


def set_rng_state(st: Dict):
    pv, pst, pg = st["python"]
    random.setstate((pv, tuple(pst), pg))
    nk, nkeys, npos, nhg, ncg = st["numpy"]
    np.random.set_state((nk, nkeys.numpy().astype(np.uint32), npos, nhg, ncg))
    torch.set_rng_state(st["cpu"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state(st["cuda"])


def save_checkpoint(path: str, model, optimizer, scheduler, state, args, rank: int, tokenizer=None,
                    extra: Optional[Dict] = None, optimizer_state: Optional[Dict] = None):
    """Rank 0 writes model/optimizer/scheduler/state; every rank writes its RNG state.
    Caller must barrier before and after. ``optimizer_state`` must be gathered by EVERY rank beforehand
    (``optimizer.state_dict()`` is a collective under ZeRO-1); it is only computed here when missing,
    which is safe for replicated optimizers only."""
    if optimizer_state is None and rank == 0:
        if type(optimizer).__name__ == "ShardedAdamW" and optimizer.engine.world_size > 1:
            raise RuntimeError("ShardedAdamW.state_dict() is collective: gather it on every rank and pass "
                               "optimizer_state=")
        optimizer_state = optimizer.state_dict()
    if rank == 0:
        save_pretrained(model, path, tokenizer=tokenizer)
        torch.save(optimizer_state, os.path.join(path, "optimizer.pt"))
        torch.save({**scheduler.state_dict(), **(extra or {})}, os.path.join(path, "scheduler.pt"))
        state.to_json(os.path.join(path, "trainer_state.json"))
        args.to_json(os.path.join(path, "training_args.json"))


def save_rng(path: str, rank: int):
    os.makedirs(path, exist_ok=True)
    torch.save(rng_state(), os.path.join(path, f"rng_state_{rank}.pth"))


def list_checkpoints(output_dir: str):
    if not os.path.isdir(output_dir):
        return []
    out = []
    for d in os.listdir(output_dir):
        m = re.fullmatch(r"checkpoint-(\d+)", d)
        if m and os.path.exists(os.path.join(output_dir, d, "trainer_state.json")):
            out.append((int(m.group(1)), os.path.join(output_dir, d)))
    return [p for _, p in sorted(out)]


def latest_checkpoint(output_dir: str) -> Optional[str]:
    c = list_checkpoints(output_dir)
    return c[-1] if c else None


def rotate_checkpoints(output_dir: str, limit: Optional[int], best: Optional[str] = None):
    if not limit or limit <= 0:
        return
    ck = list_checkpoints(output_dir)
    keep = set(ck[-limit:])
    if best:
        keep.add(os.path.abspath(best) if os.path.isabs(best) else best)
    for p in ck:
        if p not in keep and os.path.abspath(p) not in {os.path.abspath(k) for k in keep}:
            shutil.rmtree(p, ignore_errors=True)


def load_checkpoint(path: str, model, optimizer, scheduler, rank: int):
    from ..train.callbacks import TrainerState
    sd = load_state_dict(path, device="cpu")
    with torch.no_grad():
        model.load_hf_state_dict({k: v.to(model.model.embed_tokens.dtype) for k, v in sd.items()}, strict=False)
        ad = os.path.join(path, "adapter_model.safetensors")
        if os.path.exists(ad):
            _load_lora(model, ad)
    osd = torch.load(os.path.join(path, "optimizer.pt"), map_location="cpu", weights_only=True)
    optimizer.load_state_dict(osd)
    ssd = torch.load(os.path.join(path, "scheduler.pt"), weights_only=True)
    scheduler.load_state_dict(ssd)
    rp = os.path.join(path, f"rng_state_{rank}.pth")
    if os.path.exists(rp):
        set_rng_state(torch.load(rp, weights_only=True))
    return TrainerState.from_json(os.path.join(path, "trainer_state.json")), ssd


def _load_lora(model, path):
    from safetensors.torch import load_file
    sd = load_file(path)
    for i, layer in enumerate(model.model.layers):
        for owner, mod_name, key in ((layer.self_attn, "self_attn", "qkv"), (layer.self_attn, "self_attn", "o"),
                                     (layer.mlp, "mlp", "gate_up"), (layer.mlp, "mlp", "down")):
            if owner.lora is None:
                continue
            fl = owner.lora[key]
            for j, (name, act) in enumerate(zip(fl.names, fl.active)):
                pre = f"base_model.model.model.layers.{i}.{mod_name}.{name}"
                if act and pre + ".lora_A.weight" in sd:
                    fl.A[j].copy_(sd[pre + ".lora_A.weight"])
                    fl.B[j].copy_(sd[pre + ".lora_B.weight"])
