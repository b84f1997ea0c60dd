"""Does HIP-graph dispatch shorten the config-2 inference step?  The recorded op list (engine._OpPlan) is replayed
(a) by esr_run_ops as usual and (b) from a HIP graph captured around the same esr_run_ops call (static input / output
buffers), order-balanced A, B, A, B; ms per forward, and the outputs compared bitwise.

    python tools/graph_ab.py [--reps 10]
"""
import argparse
import ctypes
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=10)
    a = ap.parse_args()
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    from esr_amd import _lib, engine
    dev = torch.device('cuda')
    model = bench.build_model(args, dev)
    x = bench.make_input(args, dev, 0)
    with torch.no_grad():
        y0 = model(x)
        torch.cuda.synchronize()
        net = model.generated_image_model
        plan = net._esr_cache['plans'][engine.DEFAULT_PRECISION]
        lib = _lib.load()
        xs = x.clone()
        out_static = plan.run(xs)  # pointers now fixed to xs / out_static
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            _lib.check(lib.esr_run_ops(plan.ops, plan.n, None, st), 'esr_run_ops')
        torch.cuda.synchronize()

        def eager():
            st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
            _lib.check(lib.esr_run_ops(plan.ops, plan.n, None, st), 'esr_run_ops')

        res = {}
        for rnd in range(2):
            for tag, fn in (('eager', eager), ('graph', g.replay)):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault(tag, []).append(e0.elapsed_time(e1) / a.reps)
        ye = out_static.clone()
        g.replay()
        torch.cuda.synchronize()
        print({'ms_per_forward': res, 'n_ops': plan.n, 'graph_equals_eager': bool(torch.equal(ye, out_static)),
               'equals_first_forward': bool(torch.equal(y0, out_static))}, flush=True)


if __name__ == '__main__':
    main()
