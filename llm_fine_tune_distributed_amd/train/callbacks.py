"""Trainer callbacks (reference O1-O3, ``training.py:214-241``).

The protocol mirrors ``transformers.TrainerCallback`` (``on_log(args, state, control, logs=...)``
etc.) so the reference's custom callbacks work unchanged. Callbacks are called in list order with
the SAME ``logs`` dict, so a PerplexityCallback placed before an exporter is seen by it (the
reference relies on this ordering).
"""
from __future__ import annotations

import json
import math
import os
import time
import warnings
from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional


@dataclass
class TrainerState:
    epoch: float = 0.0
    global_step: int = 0
    max_steps: int = 0
    num_train_epochs: float = 0
    log_history: List[Dict[str, Any]] = field(default_factory=list)
    best_metric: Optional[float] = None
    best_model_checkpoint: Optional[str] = None
    is_world_process_zero: bool = True
    total_flos: float = 0.0
    train_batch_size: int = 0
    samples_seen: int = 0
    tokens_seen: int = 0
    nonfinite_loss_steps: List[int] = field(default_factory=list)  # logged steps whose loss was NaN / inf

    def to_json(self, path: str):
        with open(path, "w") as f:
            json.dump(asdict(self), f, indent=2)

    @classmethod
    def from_json(cls, path: str) -> "TrainerState":
        with open(path) as f:
            d = json.load(f)
        names = set(cls.__dataclass_fields__)
        return cls(**{k: v for k, v in d.items() if k in names})


@dataclass
class TrainerControl:
    should_training_stop: bool = False
    should_epoch_stop: bool = False
    should_save: bool = False
    should_evaluate: bool = False
    should_log: bool = False


class TrainerCallback:
    def on_init_end(self, args, state, control, **kw): pass
    def on_train_begin(self, args, state, control, **kw): pass
    def on_train_end(self, args, state, control, **kw): pass
    def on_epoch_begin(self, args, state, control, **kw): pass
    def on_epoch_end(self, args, state, control, **kw): pass
    def on_step_begin(self, args, state, control, **kw): pass
    def on_step_end(self, args, state, control, **kw): pass
    def on_evaluate(self, args, state, control, metrics=None, **kw): pass
    def on_save(self, args, state, control, **kw): pass
    def on_log(self, args, state, control, logs=None, **kw): pass


class CallbackHandler:
    def __init__(self, callbacks):
        self.callbacks = list(callbacks or [])

    def add(self, cb):
        self.callbacks.append(cb)

    def call(self, event: str, args, state, control, **kw):
        for cb in self.callbacks:
            fn = getattr(cb, event, None)
            if fn is not None:
                r = fn(args, state, control, **kw)
                if isinstance(r, TrainerControl):
                    control = r
        return control


class TrainingHistoryCallback(TrainerCallback):
    """Reference O1: keeps every logs dict (dumped to training_history.json by rank 0)."""

    def __init__(self):
        self.history: List[Dict[str, Any]] = []

    def on_log(self, args, state, control, logs=None, **kw):
        if logs:
            self.history.append(logs)


class PerplexityCallback(TrainerCallback):
    """Reference O2: adds perplexity = exp(loss), eval_perplexity = exp(eval_loss) in place."""

    def on_log(self, args, state, control, logs=None, **kw):
        if logs:
            if "loss" in logs:
                logs["perplexity"] = math.exp(min(logs["loss"], 80.0))
            if "eval_loss" in logs:
                logs["eval_perplexity"] = math.exp(min(logs["eval_loss"], 80.0))


class JSONLLoggerCallback(TrainerCallback):
    """Append-only metrics sink (rank 0): one JSON object per log event."""

    def __init__(self, path: str):
        self.path = path
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)

    def on_log(self, args, state, control, logs=None, **kw):
        if logs and state.is_world_process_zero:
            rec = dict(logs)
            rec.setdefault("step", state.global_step)
            rec["time"] = time.time()
            with open(self.path, "a") as f:
                f.write(json.dumps(rec) + "\n")


class PrinterCallback(TrainerCallback):
    def on_log(self, args, state, control, logs=None, **kw):
        if logs and state.is_world_process_zero:
            items = ", ".join(f"{k}={v:.4g}" if isinstance(v, float) else f"{k}={v}" for k, v in logs.items())
            print(f"[step {state.global_step}] {items}", flush=True)


class AimCallback(TrainerCallback):
    """Reference O3 (aim.hugging_face.AimCallback). Uses Aim if importable (rank 0 only), else
    degrades to a JSONL file under ``repo`` with the same (name, value, context) records."""

    def __init__(self, repo: Optional[str] = None, experiment: Optional[str] = None):
        self.repo = repo or os.getenv("AIM_REPO", "/aim")
        self.experiment = experiment
        self._run = None
        self._fallback = None

    def _setup(self, args, state):
        if self._run is not None or self._fallback is not None or not state.is_world_process_zero:
            return
        try:
            from aim import Run  # type: ignore
            self._run = Run(repo=self.repo, experiment=self.experiment)
            self._run["hparams"] = {k: v for k, v in args.to_dict().items() if isinstance(v, (int, float, str, bool))}
        except Exception as e:  # aim not installed (this image) or repo unavailable
            path = self.repo if os.access(os.path.dirname(os.path.abspath(self.repo)) or ".", os.W_OK) else "/tmp/aim"
            try:
                os.makedirs(path, exist_ok=True)
            except OSError:
                path = "/tmp/aim"
                os.makedirs(path, exist_ok=True)
            self._fallback = os.path.join(path, f"{self.experiment or 'run'}.jsonl")
            warnings.warn(f"Aim unavailable ({type(e).__name__}); tracking to {self._fallback}")

    def on_train_begin(self, args, state, control, **kw):
        self._setup(args, state)

    def on_log(self, args, state, control, logs=None, **kw):
        self._setup(args, state)
        if not logs or not state.is_world_process_zero:
            return
        for k, v in logs.items():
            if not isinstance(v, (int, float)):
                continue
            if k.startswith("sys_"):  # GPU telemetry (Aim's system metrics; amdsmi instead of NVML)
                subset, name = "system", k[4:]
            elif k.startswith("eval_"):
                subset, name = "eval", k[5:]
            else:
                subset, name = "train", k
            if self._run is not None:
                self._run.track(v, name=name, step=state.global_step, epoch=state.epoch, context={"subset": subset})
            elif self._fallback:
                with open(self._fallback, "a") as f:
                    f.write(json.dumps({"name": name, "value": v, "step": state.global_step,
                                        "context": {"subset": subset}}) + "\n")

    def on_train_end(self, args, state, control, **kw):
        if self._run is not None:
            self._run.close()
