"""Worker for test_fault_tolerance: tiny SFT run, checkpoint every 2 steps, resume='auto'."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_fine_tune_distributed_amd.data.dataset import TokenizedDataset  # noqa: E402
from llm_fine_tune_distributed_amd.models import build_model, tiny  # noqa: E402
from llm_fine_tune_distributed_amd.parallel.process_group import cleanup_distributed  # noqa: E402
from llm_fine_tune_distributed_amd.train import SFTConfig, SFTTrainer  # noqa: E402

out = sys.argv[1]
cfg = tiny()
m = build_model(cfg, dtype=torch.float32, seed=0)
ds = TokenizedDataset.synthetic(64, cfg.vocab_size, 5, 20, seed=1)
shard = os.environ.get("SFTAMD_TEST_SHARD", "0") == "1"
args = SFTConfig(output_dir=out, per_device_train_batch_size=2, max_steps=6, save_steps=2, logging_steps=1,
                 learning_rate=1e-3, dataloader_drop_last=True, jsonl_log=False, ddp_timeout=60,
                 shard_optimizer_state=shard, ddp_bucket_cap_mb=0.05, ddp_first_bucket_mb=0.01)
t = SFTTrainer(model=m, args=args, train_dataset=ds)
r = t.train(resume_from_checkpoint="auto")
if t.dist.is_main:
    with open(os.path.join(out, "result.json"), "w") as f:
        json.dump({"step": r.global_step, "restart": os.environ.get("SFTAMD_RESTART_COUNT"), "log": [h.get("loss") for h in t.state.log_history if "loss" in h],
                   "checksum": float(t.engine.param_flat.double().sum()), "train_loss": r.training_loss,
                   "optimizer": type(t.optimizer).__name__}, f)
    torch.save(t.engine.param_flat.clone(), os.path.join(out, "params.pt"))
cleanup_distributed()
