#!/usr/bin/env python3
"""`python ensemble.py --files ... --type ... --output ...` drop-in: the script the GUI launches from
its base directory (reference processing.py:735; CLI ensemble.py:409-441, exit 0 / 1,
``[SESA_PROGRESS]N`` lines) -> sesa.ensemble (device blend, PCM_24 output)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sesa.ensemble import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
