#!/usr/bin/env python3
"""Drop-in for the reference's ``ask_original_model.py`` (base model, ``enable_thinking=False``).

The hub checkpoint is not downloadable offline: pass ``--model <local SmolLM3-3B dir>``; without it a
random-init SmolLM3-3B is used (plumbing only)."""
import sys

from llm_fine_tune_distributed_amd.cli.ask import main

if __name__ == "__main__":
    args = sys.argv[1:]
    if "--model" not in args:
        args += ["--model", "HuggingFaceTB/SmolLM3-3B"]
    main(args)
