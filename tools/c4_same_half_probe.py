"""Diagnostic (GPU): the C4 test's two-rank run with BOTH ranks on half 0 (tests/test_gpu_ddp_c4.py), against the
single-process half-0 run: is each rank's local gradient (captured as its buckets went out) bitwise the single
process's?  Per-parameter differences of the first D gradient."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

sys.path.insert(0, 'tests')
sys.path.insert(0, 'tests/golden')
sys.path.insert(0, '.')


def main():
    import test_gpu_ddp_c4 as T
    solo = T._run(1, half=0)[0]
    print('C4_NOFLAT=%s C4_SYNC=%s' % (os.environ.get('C4_NOFLAT'), os.environ.get('C4_SYNC')), flush=True)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=T._worker, args=(r, 2, port, 0, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(60)
    for rank, r, err in res:
        assert err is None, err
        for tag in ('D', 'G'):
            for what, v in (('local', r['local'].get(tag)), ('averaged', r['first'][tag])):
                if v is None:
                    continue
                b = solo['first'][tag]
                print('rank %d %s %s grad vs solo: bitwise %s, rel %.2e' % (
                    rank, what, tag, np.array_equal(v, b), float(np.linalg.norm(v - b) / np.linalg.norm(b))), flush=True)
                if tag == 'D' and not np.array_equal(v, b):
                    o, rows = 0, []
                    for name, n in r['dshapes']:
                        rows.append((float(np.linalg.norm(v[o:o + n] - b[o:o + n]) /
                                           max(np.linalg.norm(b[o:o + n]), 1e-30)), name, int(np.sum(v[o:o + n] != b[o:o + n])), n))
                        o += n
                    print('   worst:', sorted(rows)[::-1][:6], 'params differing:', sum(1 for x in rows if x[2]), '/',
                          len(rows), flush=True)
        print('rank %d forward inputs' % rank, r['fwd_in'], 'solo', solo['fwd_in'], flush=True)
        print('rank %d fresh generator outputs equal' % rank,
              [np.array_equal(x, y) for x, y in zip(r['fresh'], solo['fresh'])], flush=True)
        print('rank %d fake_H equal' % rank, [np.array_equal(x, y) for x, y in zip(r['fake'], solo['fake'])],
              'logs equal', r['logs'] == solo['logs'], flush=True)


if __name__ == '__main__':
    main()
