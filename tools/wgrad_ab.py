"""A/B timing of the generator weight-gradient kernels (esr_wgrad_set_kernel 0 / 1) on the config-3 conv shapes
(B=16, 96² LR): average µs per esr_conv3x3_wgrad launch and TFLOP/s (2·9·Cin·Cout per output pixel).

    python tools/wgrad_ab.py
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'explorable-super-resolution_old_amd'))
from esr_amd import _lib  # noqa: E402

SHAPES = [  # name, cin, in_cp, cout, dout_cp, up2, H, W
    ('rdb_c0', 72, 264, 32, 264, 0, 96, 96),
    ('rdb_c2', 136, 264, 32, 264, 0, 96, 96),
    ('rdb_c4', 200, 264, 64, 64, 0, 96, 96),
    ('up1', 64, 72, 64, 72, 1, 192, 192),
    ('up2', 64, 72, 64, 72, 1, 384, 384),
    ('hr0', 72, 72, 64, 72, 0, 384, 384),
    ('hr1', 72, 72, 3, 8, 0, 384, 384),
]


def main():
    lib = _lib.load()
    dev = torch.device('cuda')
    B = 16
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for name, cin, in_cp, cout, d_cp, up2, H, W in SHAPES:
        Hi, Wi = (H // 2, W // 2) if up2 else (H, W)
        x = torch.randn(B, Hi + 2, Wi + 2, in_cp, device=dev)
        d = torch.randn(B, H + 2, W + 2, d_cp, device=dev)
        chunks = (cin + 31) // 32
        ntiles = B * ((H + 7) // 8) * ((W + 31) // 32)
        splits = max(1, min(128, -(-1024 // chunks), ntiles))
        cin_pad, cout_pad = 32 * chunks, 64 if cout > 32 else 32
        n = 9 * cin_pad * cout_pad + cout_pad
        part = torch.empty(splits * n, device=dev)
        flops = 2 * 9 * cin * cout * B * H * W
        row = {}
        outs = {}
        for v in (0, 1):
            lib.esr_wgrad_set_kernel(v)
            for _ in range(3):
                lib.esr_conv3x3_wgrad(x.data_ptr(), in_cp, cin, up2, d.data_ptr(), d_cp, 0, cout, B, H, W, splits,
                                      part.data_ptr(), st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                lib.esr_conv3x3_wgrad(x.data_ptr(), in_cp, cin, up2, d.data_ptr(), d_cp, 0, cout, B, H, W, splits,
                                      part.data_ptr(), st)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000 / reps
            out = torch.empty(n, device=dev)
            lib.esr_wgrad_reduce(part.data_ptr(), splits, n, 1.0, out.data_ptr(), st)
            outs[v] = out
            row['v%d_us' % v] = round(us, 2)
            row['v%d_tflops' % v] = round(flops / us / 1e6, 1)
        torch.cuda.synchronize()
        row['rel_diff'] = float((outs[0] - outs[1]).abs().max() / outs[0].abs().max())
        row['splits'] = splits
        res[name] = row
        print(name, json.dumps(row), flush=True)
    lib.esr_wgrad_set_kernel(1)


if __name__ == '__main__':
    main()
