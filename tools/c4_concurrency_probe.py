"""Diagnostic (GPU): is the C4 test's single-process half-batch step (tests/test_gpu_ddp_c4.py _run_half) bitwise
reproducible when another process runs the same step on the GPU at the same time?  Two concurrent world-1 runs of
half 0 against a solo run: first D / G gradients and the generator outputs, per parameter where they differ."""
import os
import sys

import numpy as np
import torch.multiprocessing as mp

sys.path.insert(0, 'tests')
sys.path.insert(0, 'tests/golden')
sys.path.insert(0, '.')


def main():
    import test_gpu_ddp_c4 as T
    solo = T._run(1, half=0)[0]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=T._worker, args=(0, 1, 0, 0, q)) for _ in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(60)
    for k, (_, r, err) in enumerate(res):
        assert err is None, err
        for tag in ('D', 'G'):
            a, b = r['first'][tag], solo['first'][tag]
            rel = float(np.linalg.norm(a - b) / np.linalg.norm(b))
            print('concurrent run %d: first %s grad vs solo: equal %s, rel %.2e' % (k, tag, np.array_equal(a, b), rel),
                  flush=True)
            if tag == 'D' and not np.array_equal(a, b):
                o, rows = 0, []
                for name, n in r['dshapes']:
                    rows.append((float(np.linalg.norm(a[o:o + n] - b[o:o + n]) / max(np.linalg.norm(b[o:o + n]), 1e-30)),
                                 name))
                    o += n
                print('  worst D params:', sorted(rows)[::-1][:6], flush=True)
        print('  fake_H equal', [np.array_equal(x, y) for x, y in zip(r['fake'], solo['fake'])], flush=True)


if __name__ == '__main__':
    main()
