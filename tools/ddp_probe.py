#!/usr/bin/env python3
"""Two ranks (gloo, sharing one GPU) against one process on the config-3 training loop at fixture size
(tests/test_gpu_ddp.py's worker): the largest relative L2 difference per tensor, twice.  Diagnostic of round 5: the
two-rank step is not bitwise reproducible run to run (~1e-7 relative in the weights), and the only visible differences
are the conv biases that feed a BatchNorm (analytically zero gradient, Adam-amplified rounding noise) and the BN running
means that carry them; single-process runs, alone or two at once on the GPU, are bitwise reproducible.
    usage (GPU): python tools/ddp_probe.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'tests'))
import test_gpu_ddp as T  # noqa: E402


def main():
    for cfg in ('adaptive_rel', 'past_ratio2_acc2'):
        single = T._run(1, cfg, True)[0]
        for rep in range(2):
            two = T._run(2, cfg, True)
            rows = sorted(((float(np.linalg.norm(single[5][k][2] - two[0][5][k][2]) /
                                  max(np.linalg.norm(single[5][k][2]), 1e-30)), k) for k in single[5]), reverse=True)
            print('two-rank %d %-16s equal %s; largest relative L2 differences: %s' % (
                rep, cfg, two[0][1] == single[1], ', '.join('%s %.1e' % (k, r) for r, k in rows[:12])), flush=True)


if __name__ == '__main__':
    main()
