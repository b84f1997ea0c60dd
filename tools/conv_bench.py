#!/usr/bin/env python3
"""Microbenchmark of single libesr_amd conv launches at the bench shape (B=32, 148×148 LR grid) for tuning/PMC runs.

    python tools/conv_bench.py [--precision x3|f32] [--iters 20]
Prints one line per case: cin, cout, avg µs (HIP events), reference TFLOP/s.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

from esr_amd import _lib, engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', default='x3')
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--B', type=int, default=32)
    ap.add_argument('--H', type=int, default=148)
    ap.add_argument('--cases', default='128:32,192:64,64:32')
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device('cuda:0')
    B, H, W = a.B, a.H, a.H
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    for case in a.cases.split(','):
        cin, cout = map(int, case.split(':'))
        cp = 192
        x = torch.zeros(B, H + 2, W + 2, cp, device=dev)
        x[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, device=dev) * 2 - 1
        w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
        b = torch.zeros(cout, device=dev)
        pk = engine.pack_conv_weight(w, list(range(cin)), 32 if cout <= 32 else 64)
        out = torch.zeros(B, H + 2, W + 2, cp, device=dev)
        o = engine._conv_out(out, cp, 0, H, W, True)
        if a.precision == 'x3':
            xs = engine.to_split(x)
            wx, scale = engine.pack_x3(pk)

            def run():
                _lib.check(lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(),
                                                  scale, cout, ctypes.byref(o), ovf.data_ptr(), stream), 'x3')
        else:
            def run():
                _lib.check(lib.esr_conv3x3_fwd(x.data_ptr(), B, H, W, cp, cin, pk.data_ptr(), b.data_ptr(), cout,
                                               ctypes.byref(o), stream), 'f32')
        for _ in range(3):
            run()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.iters * 1e3
        fl = 2.0 * B * H * W * 9 * cin * cout
        print('%s cin=%d cout=%d: %.1f us  %.1f TFLOP/s' % (a.precision, cin, cout, us, fl / us / 1e6), flush=True)


if __name__ == '__main__':
    main()
