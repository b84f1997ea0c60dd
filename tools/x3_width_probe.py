#!/usr/bin/env python3
"""What a partial last column strip costs the production x3 conv: per-launch time of the N = 32 conv (12-column tiles,
three workgroups per CU) at a fixed height and batch for several widths, e.g. 144 (12 full strips), 148 (config 2's
CEM-padded width: 12 full strips + one of 4 columns) and 156 (13 full strips).  If 148 costs as much as 156, the
4-column strip costs a full strip.

    python3 tools/x3_width_probe.py [B H cin W1,W2,...]   (default 16 148 128 144,148,152,156)
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
import torch  # noqa: E402
from esr_amd import _lib, engine  # noqa: E402


def main():
    a = sys.argv[1:]
    B, H, cin = (int(v) for v in a[:3]) if len(a) >= 3 else (16, 148, 128)
    widths = [int(v) for v in a[3].split(',')] if len(a) >= 4 else [144, 148, 152, 156]
    lib = _lib.load()
    dev = torch.device('cuda:0')
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    cout, cp = 32, 192
    g = torch.Generator(device='cpu').manual_seed(cin)
    w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(dev)
    b = (torch.rand(cout, generator=g) * 0.02 - 0.01).to(dev)
    wx, scale = engine.pack_x3(engine.pack_conv_weight(w, list(range(cin)), 32))
    res = {}
    for rnd in range(3):  # interleaved rounds (clock drift)
        for W in widths:
            x = torch.zeros(B, H + 2, W + 2, cp)
            x[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, generator=g) * 2 - 1
            xs = engine.to_split(x.to(dev))
            out = torch.zeros(B, H + 2, W + 2, cp, device=dev)
            o = engine._conv_out(out, cp, cin if cin + cout <= cp else 0, H, W, True)

            def run():
                _lib.check(lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                                  cout, ctypes.byref(o), ovf.data_ptr(), stream), 'conv_x3')
            for _ in range(5):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(40):
                run()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(W, []).append(e0.elapsed_time(e1) / 40 * 1e3)
            del x, xs, out
    base = min(res[widths[0]])
    print('B=%d H=%d cin=%d N=32: per-launch us (min of 3 rounds of 40)' % (B, H, cin))
    for W in widths:
        t = min(res[W])
        print('  W=%4d  strips %5.2f  %7.1f us   per column %.3f us   vs W=%d x W/%d: %.3f' % (
            W, W / 12, t, t / W, widths[0], widths[0], t / (base * W / widths[0])), flush=True)


if __name__ == '__main__':
    main()
