from .config import SFTConfig, apply_overrides, config_from_env, load_config_file
from .callbacks import (TrainerCallback, TrainerControl, TrainerState, TrainingHistoryCallback, PerplexityCallback,
                        AimCallback, JSONLLoggerCallback)
from .trainer import SFTTrainer, TrainOutput, set_seed

__all__ = ["SFTConfig", "config_from_env", "TrainerCallback", "TrainerControl", "TrainerState",
           "TrainingHistoryCallback", "PerplexityCallback", "AimCallback", "JSONLLoggerCallback", "SFTTrainer",
           "TrainOutput", "set_seed"]
