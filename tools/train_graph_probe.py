#!/usr/bin/env python3
"""The generator's training graphs (train_engine._run_graphed) of the config-3 step: their node types (hipGraphGetNodes
/ hipGraphNodeGetType through the HIP runtime) and how long replay() takes to return against how long the graph runs.
hipGraphLaunch of these graphs returned only when the graph had nearly finished (tools/prof_train_api.sh), while graphs
of the same library's kernels alone return at once (tools/graph_launch_probe2.py): which node holds the host?
    usage: python tools/train_graph_probe.py
"""
import collections
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

import bench_train as BT  # noqa: E402

_KEEP = torch.cuda.CUDAGraph


class KeptGraph(_KEEP):
    def __new__(cls, *a, **k):
        return _KEEP.__new__(cls, keep_graph=True)

    def __init__(self, *a, **k):
        super().__init__(keep_graph=True)


NODE_TYPES = {0: 'kernel', 1: 'memcpy', 2: 'memset', 3: 'host', 4: 'graph', 5: 'empty', 6: 'wait_event',
              7: 'event_record', 8: 'ext_sem_signal', 9: 'ext_sem_wait', 10: 'mem_alloc', 11: 'mem_free',
              12: 'memcpy_from_symbol', 13: 'memcpy_to_symbol'}


def node_types(g):
    hip = ctypes.CDLL('libamdhip64.so')
    raw = ctypes.c_void_p(g.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(raw, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(raw, nodes, ctypes.byref(n)) == 0
    cnt = collections.Counter()
    for k in range(n.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[k]), ctypes.byref(t))
        cnt[NODE_TYPES.get(t.value, t.value)] += 1
    return dict(cnt)


def main():
    torch.cuda.CUDAGraph = KeptGraph
    from esr_amd import train_engine as TE
    from esr_amd.SRRaGAN_model import SRRaGANModel
    args = BT.leg_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(1000)
    model = SRRaGANModel(BT.make_opt(args), device=dev)
    g = torch.Generator(device='cpu').manual_seed(7)
    hr = 4 * args.lr_size
    data = {'LR': torch.rand(args.batch, 3, args.lr_size, args.lr_size, generator=g).to(dev),
            'HR': torch.rand(args.batch, 3, hr, hr, generator=g).to(dev)}
    for _ in range(4):
        model.feed_data(data)
        model.optimize_parameters()
    torch.cuda.synchronize()
    ws = [c[1] for c in model._rrdb._esr_cache.values() if isinstance(c, tuple) and len(c) == 2 and
          hasattr(c[1], 'graphs')]
    if not ws:
        ws = [v for v in vars(TE).get('_WS_LIST', [])]
    for w in ws:
        for key, ent in w.graphs.items():
            if not isinstance(ent, tuple):
                continue
            gr = ent[0]
            print(key[0], 'nodes', node_types(gr), flush=True)
            zz = torch.ones(8 << 20, device=dev)
            for pending in (0, 0, 600, 2000):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(pending):  # ~10 us kernels queued ahead of the replay
                    zz.mul_(1.0000001)
                tq = time.perf_counter()
                gr.replay()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                print('   %4d kernels queued first (%.2f ms to enqueue): replay() takes %.2f ms, all done after %.2f ms'
                      % (pending, (tq - t0) * 1e3, (t1 - tq) * 1e3, (t2 - t0) * 1e3), flush=True)


if __name__ == '__main__':
    main()
