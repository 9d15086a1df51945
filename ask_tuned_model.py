#!/usr/bin/env python3
"""Drop-in for the reference's ``ask_tuned_model.py``: ``python ask_tuned_model.py "question"``."""
import sys

from llm_fine_tune_distributed_amd.cli.ask import main

if __name__ == "__main__":
    main(sys.argv[1:] + ["--model", "outputs/best_model"] if "--model" not in sys.argv else sys.argv[1:])
