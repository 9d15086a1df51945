from .config import ModelConfig, get_config, llama3_8b, smollm3_3b, tiny, PRESETS
from .transformer import CausalLM, CausalLMOutput, build_model
from .lora import LoRAConfig, apply_lora, merge_lora
from .freeze import apply_freeze_policy

__all__ = ["ModelConfig", "get_config", "llama3_8b", "smollm3_3b", "tiny", "PRESETS", "CausalLM",
           "CausalLMOutput", "build_model", "LoRAConfig", "apply_lora", "merge_lora", "apply_freeze_policy"]
