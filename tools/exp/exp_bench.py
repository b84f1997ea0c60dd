#!/usr/bin/env python3
"""Experimental-kernel microbench (tools/exp/libx3exp.so): same shapes as tools/conv_bench.py; compares modes."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
import torch
from esr_amd import _lib, engine

lib = _lib.load()
exp = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), os.environ.get('EXP_LIB', 'libx3exp.so')))
exp.x3exp_conv.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.c_int,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device('cuda:0')
B, H, W = 32, 148, 148
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
ovf = torch.zeros(1, dtype=torch.int32, device=dev)
modes = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else '0,1,2').split(',')]
for cin, cout in ((128, 32), (192, 64), (64, 32)):
    cp = 192
    x = torch.zeros(B, H + 2, W + 2, cp, device=dev)
    x[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, device=dev) * 2 - 1
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
    b = torch.zeros(cout, device=dev)
    pk = engine.pack_conv_weight(w, list(range(cin)), 32 if cout <= 32 else 64)
    xs = engine.to_split(x)
    wx, scale = engine.pack_x3(pk)
    outs = {}
    for mode in [-1] + modes:
        out = torch.zeros(B, H + 2, W + 2, cp, device=dev)
        o = engine._conv_out(out, cp, 0, H, W, True)
        if mode < 0:
            run = lambda: lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                                 cout, ctypes.byref(o), ovf.data_ptr(), stream)
        else:
            run = lambda: exp.x3exp_conv(mode, xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                         cout, ctypes.byref(o), ovf.data_ptr(), stream)
        for _ in range(3):
            assert run() == 0
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        fl = 2.0 * B * H * W * 9 * cin * cout
        outs[mode] = engine.from_split(out[:, 1:-1, 1:-1, :cout])
        err = '' if mode <= 0 else ''
        if mode in (0, 5):
            err = ' maxdiff vs product %.2e' % float((outs[mode] - outs[-1]).abs().max())
        print('cin=%d cout=%d mode=%d: %.1f us  %.1f TFLOP/s%s' % (cin, cout, mode, us, fl / us / 1e6, err), flush=True)
