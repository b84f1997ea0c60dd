#!/usr/bin/env python3
"""Does a HIP graph of THIS library's kernels return from replay() early (host runs ahead) like a graph of PyTorch
kernels (tools/graph_launch_probe.py), or block until it nearly finishes, as hipGraphLaunch of the generator's
training graphs did in the config-3 API trace (58 ms for the backward graph)?  Chains of N launches of: an x3 conv
(esr_conv3x3_fwd_x3), an elementwise kernel (esr_axpby), a PyTorch mul_ (control); then the generator's own training
forward graph (train_engine._run_graphed) timed the same way.
    usage: python tools/graph_launch_probe2.py [N]
"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
import torch  # noqa: E402
from esr_amd import _lib, engine  # noqa: E402


def timed_replay(name, fn, n):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print('%-10s N=%4d: replay() returns after %7.2f ms, graph done after %7.2f ms' % (name, n, (t1 - t0) * 1e3,
                                                                                   (t2 - t0) * 1e3), flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    lib = _lib.load()
    dev = torch.device('cuda', 0)
    B, H, W, cin, cout, cp = 4, 96, 96, 64, 32, 192
    x = torch.zeros(B, H + 2, W + 2, cp, device=dev)
    x[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, device=dev)
    xs = engine.to_split(x)
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
    b = torch.zeros(cout, device=dev)
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w, list(range(cin)), 32))
    out = torch.zeros(B, H + 2, W + 2, cp, device=dev)
    o = engine._conv_out(out, cp, cin, H, W, True)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)

    def conv():
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale, cout,
                                          ctypes.byref(o), ovf.data_ptr(), st), 'conv')
    y = torch.zeros(B, H + 2, W + 2, 64, device=dev)

    def axpby():
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(lib.esr_axpby(y.data_ptr(), 64, 0, 1.0001, y.data_ptr(), 64, 0, 0.0, None, 64, 0, 64, B, H, W, st),
                   'axpby')
    z = torch.ones(8 << 20, device=dev)

    def mul():
        z.mul_(1.0000001)
    for name, fn in (('torch_mul', mul), ('esr_axpby', axpby), ('esr_conv', conv)):
        timed_replay(name, fn, n)


if __name__ == '__main__':
    main()
