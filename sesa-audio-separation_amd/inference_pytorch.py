#!/usr/bin/env python3
"""`python inference_pytorch.py ...` drop-in: the script the GUI launches (reference
processing.py:250-252 prefers ``inference_pytorch.INFERENCE_PATH`` over inference.py; CLI surface
inference_pytorch.py:277-390) -> sesa.inference on the MI355X path."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sesa.inference import proc_folder  # noqa: E402

INFERENCE_PATH = os.path.abspath(__file__)   # inference_pytorch.py:19; processing.py:250 imports it

if __name__ == "__main__":
    sys.exit(proc_folder())
