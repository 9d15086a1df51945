#!/usr/bin/env python3
"""Drop-in for the reference's ``training.py``: same env contract and artifacts, MI355X-native engine.

    python training.py                                   # single process (GPU or CPU/gloo)
    python -m llm_fine_tune_distributed_amd.launch --nproc-per-node 8 training.py
"""
from llm_fine_tune_distributed_amd.cli.train import main

if __name__ == "__main__":
    main()
