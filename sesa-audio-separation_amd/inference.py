#!/usr/bin/env python3
"""`python inference.py ...` drop-in (reference inference.py:148-239 CLI surface) -> sesa.inference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sesa.inference import proc_folder  # noqa: E402

if __name__ == "__main__":
    sys.exit(proc_folder())
