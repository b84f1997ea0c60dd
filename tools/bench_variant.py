#!/usr/bin/env python3
"""Run bench.py with an x3 conv kernel variant forced (esr_x3_set_kernel / esr_x3_set_tile_map), for same-box A/B of whole steps.
    python tools/bench_variant.py VARIANT [--script bench_train.py] [bench args...]"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
from esr_amd import _lib  # noqa: E402

_v = int(sys.argv[1])  # + 1000: row-major block -> tile order (esr_x3_set_tile_map 0), else XCD-grouped (1)
_lib.load().esr_x3_set_kernel(_v % 1000)
_lib.load().esr_x3_set_tile_map(0 if _v >= 1000 else 1)
args = sys.argv[2:]
script = 'bench.py'
if args[:1] == ['--script']:
    script, args = args[1], args[2:]
sys.argv = [os.path.join(REPO, script)] + args
runpy.run_path(sys.argv[0], run_name='__main__')
