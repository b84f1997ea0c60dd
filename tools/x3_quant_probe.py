#!/usr/bin/env python3
"""Wave-quantisation probe of the x3 conv: µs per launch of one N=32 growth conv (cin 128) over a sweep of image
widths / heights around config 2's 148² (B=32), next to its tile count in rounds of the CUs' workgroup slots — a step
in time where the rounds step says the last partial round, not the work, sets the launch time.  Also the narrow-N
HR_conv1 path (cout 3, planar) against the N=32 tiles at config 2's 592² (esr_x3_set_narrow).

    python tools/x3_quant_probe.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

from esr_amd import _lib, engine  # noqa: E402


def timed(run, iters=20):
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def conv_case(lib, dev, B, H, W, cin, cout, planar=False):
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cp = max(cin, 8)
    x = torch.zeros(B, H + 2, W + 2, cp, device=dev)
    x[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, device=dev) * 2 - 1
    xs = engine.to_split(x)
    del x
    w = torch.randn(cout, cin, 3, 3, device=dev) * 0.05
    b = torch.zeros(cout, device=dev)
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w, list(range(cin)), 32 if cout <= 32 else 64))
    if planar:
        out = torch.zeros(B, cout, H, W, device=dev)
        o = engine._conv_out(out, 0, 0, H, W, False, planar=1)
    else:
        out = torch.zeros(B, H + 2, W + 2, 64, device=dev)
        o = engine._conv_out(out, 64, 0, H, W, True)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)

    def run():
        _lib.check(lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale, cout,
                                          ctypes.byref(o), ovf.data_ptr(), stream), 'x3')
    return run, out


def main():
    lib = _lib.load()
    dev = torch.device('cuda:0')
    slots = 3 * 256
    for H, W in [(148, 132), (148, 136), (148, 140), (148, 144), (148, 148), (148, 152), (148, 156), (140, 148),
                 (144, 148), (152, 148), (156, 148), (148, 148)]:
        run, _ = conv_case(lib, dev, 32, H, W, 128, 32)
        us = timed(run)
        tiles = ((W + 11) // 12) * ((32 * (H + 2) - 2 + 31) // 32)
        print('n32 cin128 B32 %dx%d: %.1f us  %.3f us/kpx  tiles %d = %.2f rounds' % (
            H, W, us, us / (32 * H * W / 1e3), tiles, tiles / slots), flush=True)
        torch.cuda.empty_cache()
    for narrow in (1, 0, 1, 0):
        lib.esr_x3_set_narrow(narrow)
        run, out = conv_case(lib, dev, 32, 592, 592, 64, 3, planar=True)
        us = timed(run, 10)
        print('HR_conv1 cin64 cout3 B32 592^2 planar, narrow=%d: %.1f us  (%.2f TB/s of split input)' % (
            narrow, us, 32 * 594 * 594 * 64 * 4 / us / 1e6), flush=True)
        del run, out
        torch.cuda.empty_cache()
    lib.esr_x3_set_narrow(1)


if __name__ == '__main__':
    main()
