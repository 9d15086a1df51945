"""MI355X-native distributed SFT framework (capabilities of thesteve0/llm-fine-tune-distributed).

Public API mirrors the reference's TRL surface: ``SFTConfig`` + ``SFTTrainer(...).train()``.
"""
__version__ = "0.1.0"

from .models import ModelConfig, CausalLM, build_model, get_config  # noqa: F401


def __getattr__(name):
    # lazy imports keep `import llm_fine_tune_distributed_amd` light for the launcher
    if name in ("SFTConfig",):
        from .train.config import SFTConfig
        return SFTConfig
    if name in ("SFTTrainer", "TrainOutput"):
        from .train import trainer
        return getattr(trainer, name)
    if name in ("TrainerCallback",):
        from .train.callbacks import TrainerCallback
        return TrainerCallback
    raise AttributeError(name)
