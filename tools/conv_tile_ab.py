"""A/B timing of the exact-fp32 conv tile height (esr_conv_set_tile 8 / 4 / automatic) on config-3 shapes (B=16,
96² LR): µs per esr_conv3x3_fwd launch, TFLOP/s, and a bitwise comparison of the outputs.

    python tools/conv_tile_ab.py
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'explorable-super-resolution_old_amd'))
from esr_amd import _lib, engine as E  # noqa: E402

SHAPES = [  # name, cin, in_cp, cout, H, W, B
    ('fwd_c0', 72, 264, 32, 96, 96, 16),
    ('fwd_c2', 136, 264, 32, 96, 96, 16),
    ('fwd_c4', 200, 264, 64, 96, 96, 16),
    ('dg_m4', 64, 64, 32, 96, 96, 16),
    ('dg_m1', 160, 160, 32, 96, 96, 16),
    ('dg_x', 192, 192, 64, 96, 96, 16),
    ('up_dg', 64, 64, 64, 192, 192, 16),
    ('c2_f32', 136, 200, 32, 148, 148, 32),
]


def main():
    lib = _lib.load()
    dev = torch.device('cuda')
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, cin, in_cp, cout, H, W, B in SHAPES:
        x = torch.randn(B, H + 2, W + 2, in_cp, device=dev)
        w = torch.randn(cout, cin, 3, 3) / (3 * cin ** 0.5)
        wp = E.pack_conv_weight(w, list(range(cin)), 32 if cout <= 32 else 64).to(dev)
        bias = torch.zeros(cout, device=dev)
        flops = 2 * 9 * cin * cout * B * H * W
        row, outs = {}, {}
        for rows in (8, 4, 0):
            out = torch.zeros(B, H + 2, W + 2, cout, device=dev)
            o = E._conv_out(out, cout, 0, H, W, 1)
            lib.esr_conv_set_tile(rows)
            for _ in range(3):
                _lib.check(lib.esr_conv3x3_fwd(x.data_ptr(), B, H, W, in_cp, cin, wp.data_ptr(), bias.data_ptr(), cout,
                                               ctypes.byref(o), st), 'conv')
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                lib.esr_conv3x3_fwd(x.data_ptr(), B, H, W, in_cp, cin, wp.data_ptr(), bias.data_ptr(), cout,
                                    ctypes.byref(o), st)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000 / reps
            outs[rows] = out
            row['t%d_us' % rows] = round(us, 2)
            row['t%d_tflops' % rows] = round(flops / us / 1e6, 1)
        row['bitwise_equal'] = bool(torch.equal(outs[8], outs[4]))
        print(name, json.dumps(row), flush=True)
    lib.esr_conv_set_tile(0)


if __name__ == '__main__':
    main()
