#!/usr/bin/env python3
"""Run one of the benchmark scripts with ablation-library knobs set first (same-box A/B of a kernel variant on a whole
step).  Needs ESR_AMD_LIB=exp_lib/libesr_exp.so.

    python3 tools/knob_bench.py axpby_set_rows=2 [x3_set_kernel=88 ...] -- bench_zopt.py --steps 10
"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))


def main():
    argv = sys.argv[1:]
    sep = argv.index('--')
    knobs, script = argv[:sep], argv[sep + 1:]
    from esr_amd import _lib
    lib = _lib.load()
    for kv in knobs:
        name, val = kv.split('=')
        fn = getattr(lib, 'esr_' + name, None)
        if fn is None:
            raise SystemExit('no setter esr_%s (the ablation library: ESR_AMD_LIB=exp_lib/libesr_exp.so)' % name)
        if fn(int(val)) < 0:
            raise SystemExit('esr_%s(%s) rejected' % (name, val))
    sys.argv = script
    runpy.run_path(os.path.join(REPO, script[0]), run_name='__main__')


if __name__ == '__main__':
    main()
