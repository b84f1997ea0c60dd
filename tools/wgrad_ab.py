"""A/B timing of the generator weight-gradient kernels on the config-3 conv shapes (B=16, 96² LR): the exact-fp32
12-wave kernel reading split-f16 activations (flags 2, the round-1 training path) against the x3 kernel (flags 6),
the latter also at other split-K counts, and the x3 kernels on a split-f16 output gradient (flags 14, the x3
backward's residual blocks): LDS-DMA (wgrad3d, default) vs register-staged (esr_wgrad3_set_dma(0)).  Average µs per esr_conv3x3_wgrad launch (+ its esr_wgrad_reduce) and
TFLOP/s (2·9·Cin·Cout per output pixel), order-balanced (A, B, A, B; the last pair is reported).

    python tools/wgrad_ab.py [--splits-scale 1,0.5,0.25]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'explorable-super-resolution_old_amd'))
from esr_amd import _lib  # noqa: E402
from esr_amd import engine as E  # noqa: E402

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
    ap = argparse.ArgumentParser()
    ap.add_argument('--splits-scale', default='1,0.5,0.25')
    ap.add_argument('--reps', type=int, default=20)
    a = ap.parse_args()
    scales = [float(s) for s in a.splits_scale.split(',')]
    lib = _lib.load()
    dev = torch.device('cuda')
    B = 16
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for name, cin, in_cp, cout, d_cp, up2, H, W in SHAPES:
        Hi, Wi = (H // 2, W // 2) if up2 else (H, W)
        x = E.to_split(torch.randn(B, Hi + 2, Wi + 2, in_cp, device=dev))
        d = torch.randn(B, H + 2, W + 2, d_cp, device=dev) * 1e-7
        ds = E.to_split(d * 2.0 ** 30) if cout % 8 == 0 and d_cp % 8 == 0 else None  # S·d, split-f16
        chunks = (cin + 31) // 32
        ntiles = B * ((H + 7) // 8) * ((W + 31) // 32)
        splits0 = max(1, min(128, -(-1024 // chunks), ntiles))
        splits_x3 = max(1, min(128, 256 // chunks, ntiles))
        cin_pad, cout_pad = 32 * chunks, 64 if cout > 32 else 32
        n = 9 * cin_pad * cout_pad + cout_pad
        part = torch.empty(splits0 * n, device=dev)
        flops = 2 * 9 * cin * cout * B * H * W
        variants = [('f32', 2, splits0)] + [('x3_s%d' % max(1, int(splits0 * s)), 6, max(1, int(splits0 * s)))
                                            for s in scales] + [("x3_auto", 6, splits_x3)]
        if ds is not None:
            variants += [('x3_dsplit_dma', 14, splits_x3), ('x3_dsplit_reg', 30, splits_x3)]  # 16: tool-local tag

        def run(flags, splits, reps, out=None):
            lib.esr_wgrad3_set_dma(0 if flags & 16 else 1)
            dd, sc = (ds, 2.0 ** -30) if flags & 8 else (d, 1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                _lib.check(lib.esr_conv3x3_wgrad(x.data_ptr(), in_cp, cin, up2 | (flags & 15), dd.data_ptr(), d_cp, 0,
                                                 cout, B, H, W, splits, part.data_ptr(), st), 'wgrad')
                if out is not None:
                    _lib.check(lib.esr_wgrad_reduce(part.data_ptr(), splits, n, sc, out.data_ptr(), st), 'reduce')
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1000 / reps

        row, outs = {'splits0': splits0}, {}
        for rnd in range(2):
            for tag, flags, splits in variants:
                run(flags, splits, 2)
                us = run(flags, splits, a.reps)
                out = torch.empty(n, device=dev)
                us_red = run(flags, splits, a.reps, out)
                outs[tag] = out
                if rnd == 1:
                    row[tag + '_us'] = round(us, 2)
                    row[tag + '_with_reduce_us'] = round(us_red, 2)
                    row[tag + '_tflops'] = round(flops / us / 1e6, 1)
        ref = outs['f32']
        for tag in outs:
            if tag != 'f32':
                row[tag + '_rel_diff'] = float((outs[tag] - ref).norm() / ref.norm())
        print(name, json.dumps(row), flush=True)
    lib.esr_wgrad3_set_dma(1)


if __name__ == '__main__':
    main()
