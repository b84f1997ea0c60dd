"""A/B timing of the discriminator gather-GEMM forward (esr_dconv_fwd) on the config-3 layer shapes (B=16, D input
304², Discriminator_VGG_128_ nb=6): exact fp32, x3 with 64-channel N tiles, x3 with 128 (default).  Order-balanced
(two rounds, the second reported); µs per launch, TFLOP/s, and the results' normwise difference from the fp32 gather
kernel.  Variants: f32_gather (the per-tap gather kernel), f32_halo (halo-tile kernel, the fp32 default), x3 with 64-
and 128-channel N tiles.  Also the data gradient (all phase classes) per variant.  *_direct: the 4×4 stride-2 layers
as the direct stride-2 gather and one data-gradient launch per phase class instead of their space-to-depth form
(dconv.S2D).  AB_LAYERS (comma list of layer names) and AB_TAGS (comma list of variant tags) select a subset.

    python tools/dconv_ab.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'explorable-super-resolution_old_amd'))
from esr_amd import _lib, dconv  # noqa: E402

LAYERS = [  # name, ci, co, k, s, p, H
    ('conv0_im2col', 32, 64, 1, 1, 0, 304),
    ('conv0_1', 64, 64, 4, 2, 1, 304),
    ('conv1_0', 64, 128, 3, 1, 1, 152),
    ('conv1_1', 128, 128, 4, 2, 1, 152),
    ('conv2_0', 128, 256, 3, 1, 1, 76),
    ('conv2_1', 256, 256, 4, 2, 1, 76),
    ('fc8', 256, 100, 8, 1, 0, 38),
]


def main():
    lib = _lib.load()
    dev = torch.device('cuda')
    B = 16
    variants = [('f32', 0, 0, 1), ('f32_halo', 0, 1, 1), ('x3_n128', 1, 0, 1), ('x3_halo', 1, 1, 1), ('x6', 3, 0, 1),
                ('x6_halo', 3, 1, 1), ('f32_halo_direct', 0, 1, 0), ('x3_halo_direct', 1, 1, 0),
                ('x3_halo_sdall', 1, 2, 1), ('x3_halo_n64', 2, 1, 1), ('x3_halo_occ2', 1, 1, 1), ('x3_halo_cw32', 1, 1, 1)]
    if 'AB_TAGS' in os.environ:
        keep = set(os.environ['AB_TAGS'].split(',')) | {'f32'}
        variants = [v for v in variants if v[0] in keep]
    layers = LAYERS
    if 'AB_LAYERS' in os.environ:
        layers = [l for l in LAYERS if l[0] in os.environ['AB_LAYERS'].split(',')]
    for name, ci, co, k, s, p, H in layers:
        x = torch.randn(B, H, H, ci, device=dev)
        w = torch.randn(co, ci, k, k, device=dev) / (ci * k * k) ** 0.5
        b = torch.randn(co, device=dev) * 0.1
        Ho = dconv.out_size(H, k, s, p)
        flops = 2 * B * Ho * Ho * co * ci * k * k
        row, outs = {}, {}
        gy = torch.randn(B, Ho, Ho, co, device=dev) * 1e-8
        for rnd in range(2):
            for tag, mode, halo, s2d in variants:
                dconv.S2D = bool(s2d)
                dconv.set_precision({0: 'f32', 3: 'x6'}.get(mode, 'x3'))
                dconv._LIB_MODE['x3'] = 2 if mode == 2 else 1  # per-call prec code (x3 with 64-wide tiles: 2)
                lib.esr_dconv_set_halo(halo)
                lib.esr_dconv_set_rows(min(halo, 1))  # *_halo: the halo forward and the tap-row weight gradient
                lib.esr_dconv_set_occ3(0 if tag.endswith('_occ2') else 1)
                lib.esr_dconv_set_cw16(0 if tag.endswith('_cw32') else 1)
                for _ in range(2):
                    dconv.conv_forward(x, w, b, k, s, p)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    y = dconv.conv_forward(x, w, b, k, s, p)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 100
                dconv.conv_dgrad(gy, w, k, s, p, H, H)
                e0.record()
                for _ in range(10):
                    gx = dconv.conv_dgrad(gy, w, k, s, p, H, H)
                e1.record()
                torch.cuda.synchronize()
                us_d = e0.elapsed_time(e1) * 100
                dconv.conv_wgrad(x, gy, k, s, p)
                e0.record()
                for _ in range(10):
                    gw = dconv.conv_wgrad(x, gy, k, s, p)
                e1.record()
                torch.cuda.synchronize()
                us_w = e0.elapsed_time(e1) * 100
                outs[tag] = y
                outs[tag + 'w'] = gw
                outs[tag + 'd'] = gx
                if rnd:
                    row[tag + '_us'] = round(us, 1)
                    row[tag + '_tflops'] = round(flops / us / 1e6, 1)
                    row[tag + '_wgrad_us'] = round(us_w, 1)
                    row[tag + '_dgrad_us'] = round(us_d, 1)
        for tag in [v[0] for v in variants[1:]]:
            row[tag + '_diff'] = float((outs[tag] - outs['f32']).norm() / outs['f32'].norm())
            row[tag + '_dgrad_diff'] = float((outs[tag + 'd'] - outs['f32d']).norm() / outs['f32d'].norm())
            row[tag + '_wgrad_diff'] = float((outs[tag + 'w'] - outs['f32w']).norm() / outs['f32w'].norm())
        print(name, json.dumps(row), flush=True)
    dconv._LIB_MODE['x3'] = 1
    lib.esr_dconv_set_halo(1)
    lib.esr_dconv_set_rows(0)
    dconv.S2D = True


if __name__ == '__main__':
    main()
