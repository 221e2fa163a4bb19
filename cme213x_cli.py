#!/usr/bin/env python3
"""`python cme213x_cli.py <command> ...` == `python -m cme213x <command> ...`
from any working directory (scripts cd into data directories)."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import cme213x  # noqa: E402,F401  (installs the cme213x.* alias)

if __name__ == "__main__":
    sys.exit(importlib.import_module("2012-04_stanford_cme213_amd.__main__").main())
