"""Diagnostic (GPU): the C4 test's half-batch run with every torch.empty NaN-filled (reads of uninitialised memory show
as NaN or as a change), and the two-rank run's generator outputs against the single-process ones."""
import os
import sys

import numpy as np

sys.path.insert(0, 'tests')
sys.path.insert(0, 'tests/golden')
sys.path.insert(0, '.')


def main():
    import test_gpu_ddp_c4 as T
    os.environ['C4_NANFILL'] = '1'
    h = T._run(1, half=0)[0]
    print('NaN-fill half 0: first D finite', np.isfinite(h['first']['D']).all(), 'G finite',
          np.isfinite(h['first']['G']).all(), 'fake finite', [bool(np.isfinite(f).all()) for f in h['fake']],
          'logs', h['logs'], flush=True)
    os.environ['C4_NANFILL'] = '0'
    h2 = T._run(1, half=0)[0]
    print('vs normal: D equal', np.array_equal(h['first']['D'], h2['first']['D']), 'fake equal',
          [np.array_equal(a, b) for a, b in zip(h['fake'], h2['fake'])], flush=True)
    r = T._run(2)
    print('ddp rank0 vs half0 fake', [np.array_equal(a, b) for a, b in zip(r[0]['fake'], h2['fake'])],
          'D first rank0 vs half0 equal', np.array_equal(r[0]['first']['D'], h2['first']['D']), flush=True)


if __name__ == '__main__':
    main()
