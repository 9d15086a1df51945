"""``SFTConfig``: TRL/HF-compatible training configuration (reference T1, ``training.py:258-287``).

Accepts the same keyword names the reference passes (including the legacy ``max_seq_length``
alias of ``max_length`` and the ``ddp_*`` / ``dataloader_*`` knobs). Unknown HF fields are
accepted and ignored with a warning so existing scripts keep working. Defaults follow the
libraries the reference runs with (HF TrainingArguments / TRL SFTConfig), e.g. AdamW
betas (0.9, 0.999), eps 1e-8, weight_decay 0, linear LR decay without warmup.

MI355X-specific extras (all optional): ``freeze_policy``, ``lora_*``, ``master_weights``,
``ddp_first_bucket_mb``, ``pad_to_multiple_of``, ``max_steps_per_epoch``...
"""
from __future__ import annotations

import dataclasses
import json
import os
import warnings
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union


@dataclass
class SFTConfig:
    # ---- reference kwargs (training.py:258-287)
    output_dir: str = "outputs/checkpoints"
    per_device_train_batch_size: int = 8
    per_device_eval_batch_size: int = 8
    gradient_accumulation_steps: int = 1
    learning_rate: float = 2e-5
    max_grad_norm: float = 1.0
    num_train_epochs: float = 3.0
    max_steps: int = -1
    logging_steps: float = 500
    logging_first_step: bool = False
    save_steps: float = 500
    bf16: bool = True
    fp16: bool = False
    eval_strategy: str = "no"
    eval_steps: Optional[float] = None
    save_strategy: str = "steps"
    load_best_model_at_end: bool = False
    metric_for_best_model: Optional[str] = None
    greater_is_better: Optional[bool] = None
    save_total_limit: Optional[int] = None
    dataloader_pin_memory: bool = True
    dataloader_num_workers: int = 0
    remove_unused_columns: bool = True
    gradient_checkpointing: bool = False
    dataloader_drop_last: bool = False
    max_length: Optional[int] = 1024
    packing: bool = False
    # TRL's ``padding_free``: the batch's sequences flattened into one varlen sequence (``cu_seqlens`` / per-sample
    # ``position_ids``; attention never crosses samples, pads carry no loss), so the loss and every gradient are those
    # of the padded batch without the pad rows' FLOPs. None = on for GPU training without context parallelism (the
    # reference recipe's padded micro-batches carry ~11 % pad tokens, profiles/r3_recipe.md), off on CPU.
    padding_free: Optional[bool] = None
    ddp_backend: Optional[str] = None
    ddp_find_unused_parameters: Optional[bool] = None
    ddp_bucket_cap_mb: Optional[float] = None
    ddp_timeout: int = 1800
    local_rank: int = -1
    # ---- optimizer / schedule (HF defaults)
    optim: str = "adamw_torch_fused"
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    weight_decay: float = 0.0
    lr_scheduler_type: str = "linear"
    lr_scheduler_kwargs: Dict[str, Any] = field(default_factory=dict)
    warmup_steps: int = 0
    warmup_ratio: float = 0.0
    seed: int = 42
    data_seed: Optional[int] = None
    report_to: Any = "none"
    run_name: Optional[str] = None
    resume_from_checkpoint: Optional[str] = None
    # ---- TRL SFT
    dataset_text_field: str = "text"
    completion_only_loss: Optional[bool] = None
    assistant_only_loss: bool = False
    average_tokens_across_devices: bool = True
    # ---- MI355X-native extras
    freeze_policy: str = "full"             # full | last_n_layers | lora
    freeze_last_n_layers: int = 2
    lora_r: int = 16
    lora_alpha: float = 8.0
    lora_dropout: float = 0.05
    lora_target_modules: Optional[List[str]] = None
    # Reference parity: the reference updates bf16 parameters directly (no master copy, training.py:99), and torch's
    # AdamW keeps exp_avg / exp_avg_sq in the parameter dtype — bf16. The default here is the same state: bf16
    # parameters and bf16 moments, every bf16 write-back stochastically rounded (unbiased, so not less precise than the
    # reference's round-to-nearest), 14 HBM bytes per parameter and step. "auto" (default) = the parameter dtype, as
    # in torch: bf16 moments for the bf16 model the trainer builds (what bench.py runs), fp32 for an fp32 model.
    # "fp32" forces fp32 moments (22 bytes), master_weights=True adds an fp32 master copy (and makes "auto" fp32
    # moments: the master path rounds to nearest, where a bf16 exp_avg_sq would stall).
    master_weights: bool = False
    stochastic_rounding: bool = True
    optim_state_dtype: str = "auto"
    # ZeRO-1 over the DDP buckets (world_size > 1): reduce-scatter gradients, update 1/world_size of the
    # parameters per rank, all-gather them back under the next forward (train/optim.py ShardedAdamW)
    shard_optimizer_state: bool = False
    # context parallelism (ring attention, parallel/context_parallel.py): consecutive groups of this many ranks
    # share each batch with the sequence split across them; data parallelism runs across the groups
    context_parallel_size: int = 1
    context_parallel_layout: str = "zigzag"   # zigzag (causal work balanced across the group) | contiguous
    ddp_first_bucket_mb: float = 4.0
    # world > 1 with no ddp_bucket_cap_mb: time reduce-scatters of two sizes at startup, fit the per-call latency and
    # per-link bandwidth, and plan the bucket cap from them (parallel/ddp.py measure_link / fit_link); False = the
    # modelled 30 us / 100 GB/s
    ddp_link_probe: bool = True
    ddp_broadcast_params: bool = False      # weights are identical by construction (seeded / loaded)
    ddp_check_sync_every: int = 0           # cross-rank param checksum every N steps (0 = off)
    # None = auto: on the GPU, padded batches are padded to a multiple of 64 tokens (and packed batches to 256)
    # so every micro-batch GEMM has M % 256 == 0 and runs on the MFMA-tiled HIP paths; pads are label -100, so
    # the loss and gradients are unchanged. 1 = pad to the longest sample exactly (TRL's behaviour).
    pad_to_multiple_of: Optional[int] = None
    max_train_samples: Optional[int] = None
    max_eval_samples: Optional[int] = None
    eval_accumulation: bool = True
    jsonl_log: bool = True
    prefetch_batches: int = 2
    # pipeline AdamW (and ZeRO-1's parameter all-gathers) under the next forward on a side HIP stream: "auto" = on
    # when world_size > 1 (hides the gathers), off on one GPU, where the overlapped update slowed the step by 1 %
    # (profiles/r6_adamw_overlap.md); True / False force it
    optimizer_overlap: Union[bool, str] = "auto"
    gemm_tuning: bool = True                # load shipped hipBLASLt/rocBLAS selections (utils/gemm_tuning.py)
    # GA micro-batch merging (MI355X-first): gradient accumulation exists to fit a per-device batch into
    # memory; when the step's GA micro-batches together hold at most this many tokens (288 GB of HBM holds
    # far more than the reference's 48 GB L40S), they run as ONE fwd/bwd pass. Same gradient, loss
    # normalisation (global token count) and metrics; only the fp32-vs-bf16 summation order of the weight
    # gradient changes (one fp32-accumulated GEMM instead of bf16 += per micro-batch). 0 = always run GA passes.
    ga_merge_max_tokens: int = 32768
    # tokenisation cache (TRL main_process_first): rank 0 tokenises, the others load; True = output_dir/.sftamd_cache,
    # a str = that directory, False = every rank tokenises
    dataset_cache: Union[bool, str] = True
    # observability: per-step phase breakdown (data / fwd / bwd / comm_wait / optim, with
    # roctx ranges, logged as *_ms keys; adds a device sync per phase, so off by default) and GPU telemetry
    # (utilisation / power / temperature / HBM via amdsmi or rocm-smi) every N log steps into the trackers
    log_step_phases: bool = False
    log_system_metrics_every: int = 0
    # a non-finite logged loss (read at the logging cadence only: no extra host sync) is reported on stderr and in the
    # heartbeat (phase "nonfinite_loss"); True also stops training at that step
    stop_on_nonfinite_loss: bool = False

    def __post_init__(self):
        pass

    # legacy alias used by the reference (training.py:282)
    @property
    def max_seq_length(self) -> Optional[int]:
        return self.max_length

    @classmethod
    def create(cls, **kw) -> "SFTConfig":
        names = {f.name for f in dataclasses.fields(cls)}
        known, unknown = {}, {}
        for k, v in kw.items():
            if k == "max_seq_length":
                known["max_length"] = v
            elif k == "evaluation_strategy":
                known["eval_strategy"] = v
            elif k in names:
                known[k] = v
            else:
                unknown[k] = v
        if unknown:
            warnings.warn(f"SFTConfig: ignoring unsupported fields {sorted(unknown)}")
        return cls(**known)

    def resolved_eval_steps(self) -> Optional[int]:
        if self.eval_strategy in ("no", None):
            return None
        if self.eval_strategy == "epoch":
            return -1
        v = self.eval_steps if self.eval_steps is not None else self.logging_steps
        return int(v) if v else None

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def to_json(self, path: str):
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=2, default=str)

    def replace(self, **overrides) -> "SFTConfig":
        """Copy with ``overrides`` applied (same alias / unknown-field handling as the constructor)."""
        kw = self.to_dict()
        kw.update(overrides)
        return SFTConfig(**kw)


def _coerce(field_type, raw: str):
    """Parse a ``--set key=value`` string into the dataclass field's type."""
    t = str(field_type)
    low = raw.strip().lower()
    if low in ("none", "null"):
        return None
    if "bool" in t:
        if low in ("1", "true", "yes", "on"):
            return True
        if low in ("0", "false", "no", "off"):
            return False
        if "str" in t:  # Union[bool, str] (optimizer_overlap "auto", dataset_cache path)
            return raw
        raise ValueError(f"not a boolean: {raw!r}")
    if "List" in t or "Dict" in t:
        return json.loads(raw)
    if "float" in t:
        return float(raw)
    if "int" in t:
        return int(float(raw))
    return raw


def load_config_file(path: str) -> Dict[str, Any]:
    """Read SFTConfig overrides from a YAML (``yaml.safe_load``) or JSON file: a flat mapping of field
    names, optionally nested under a top-level ``sft_config:`` key."""
    with open(path) as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml
        data = yaml.safe_load(text) or {}
    else:
        data = json.loads(text)
    if not isinstance(data, dict):
        raise ValueError(f"{path}: expected a mapping of SFTConfig fields")
    return dict(data.get("sft_config", data))


def apply_overrides(cfg: SFTConfig, config_file: Optional[str] = None,
                    sets: Optional[List[str]] = None) -> SFTConfig:
    """Layering (lowest to highest): ``cfg`` (code defaults + env contract) < config file < ``--set k=v``.
    Unknown keys raise here (a typo in a config file must not be silently ignored)."""
    fields = {f.name: f.type for f in dataclasses.fields(SFTConfig)}
    aliases = {"max_seq_length": "max_length", "evaluation_strategy": "eval_strategy"}
    over: Dict[str, Any] = {}
    if config_file:
        over.update(load_config_file(config_file))
    for item in sets or []:
        if "=" not in item:
            raise ValueError(f"--set expects key=value, got {item!r}")
        k, v = item.split("=", 1)
        k = aliases.get(k.strip(), k.strip())
        if k not in fields:
            raise KeyError(f"--set: unknown SFTConfig field {k!r}")
        over[k] = _coerce(fields[k], v)
    over = {aliases.get(k, k): v for k, v in over.items()}
    bad = sorted(k for k in over if k not in fields)
    if bad:
        raise KeyError(f"unknown SFTConfig fields in overrides: {bad}")
    return cfg.replace(**over) if over else cfg


# SFTConfig(**kwargs) must accept legacy/unknown names like TRL does
_orig_init = SFTConfig.__init__


def _init(self, *args, **kw):
    names = {f.name for f in dataclasses.fields(SFTConfig)}
    if "max_seq_length" in kw:
        kw["max_length"] = kw.pop("max_seq_length")
    if "evaluation_strategy" in kw:
        kw["eval_strategy"] = kw.pop("evaluation_strategy")
    unknown = {k: kw.pop(k) for k in list(kw) if k not in names}
    if unknown:
        warnings.warn(f"SFTConfig: ignoring unsupported fields {sorted(unknown)}")
    _orig_init(self, *args, **kw)


SFTConfig.__init__ = _init


def config_from_env(base: Optional[SFTConfig] = None, world_size: int = 1) -> Dict[str, Any]:
    """The reference's env contract (training.py:56-60,240): EPOCHS, BATCH_SIZE, LEARNING_RATE,
    DATA_DIR, OUTPUT_DIR, AIM_REPO. Returns the resolved values (LR scaled by world size like
    training.py:263)."""
    epochs = int(os.getenv("EPOCHS", "4"))
    batch = int(os.getenv("BATCH_SIZE", "8"))
    lr = float(os.getenv("LEARNING_RATE", "5e-5"))
    return {
        "epochs": epochs,
        "batch_size": batch,
        "learning_rate": lr,
        "scaled_learning_rate": lr * world_size if world_size > 1 else lr,
        "data_dir": os.getenv("DATA_DIR", "/tmp/data"),
        "output_dir": os.getenv("OUTPUT_DIR", "/tmp/models"),
        "aim_repo": os.getenv("AIM_REPO", "/aim"),
    }
