#!/usr/bin/env python3
"""Run an unmodified reference entry script (e.g. the reference's test_wo_llava.py) against this package:
    python scripts/run_dropin.py /path/to/reference/test_wo_llava.py --img_dir ... --save_dir ... --json_dir ...
Our package root goes first on sys.path, so `FaithDiff`, `utils` and `CKPT_PTH` resolve here; runpy.run_path
does not put the script's own directory on sys.path."""
import os
import runpy
import sys

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "faithdiff-dev_amd")
sys.path.insert(0, PKG)
if len(sys.argv) < 2:
    sys.exit(__doc__)
script = sys.argv[1]
sys.argv = sys.argv[1:]
runpy.run_path(script, run_name="__main__")
