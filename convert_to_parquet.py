#!/usr/bin/env python3
"""Drop-in for the reference's ``convert_to_parquet.py`` (JSONL -> Parquet, "For {topic}, {question}")."""
from llm_fine_tune_distributed_amd.cli.convert import main

if __name__ == "__main__":
    main()
