"""Time split of the LDS-DMA x3 weight-gradient kernel (wgrad3d, the x3 backward's residual-block weight gradients)
at the config-3 shapes (B=16, 96² LR, latent: concat buffers of 200 channels, concat-gradient buffers of 264), on the
ablation library's diagnostic modes (esr_wgrad3d_set_dbg; garbage results): 0 = the kernel as built, 1 = LDS-DMA of
each workgroup's first pixel tile only ("compute alone"), 2 = no fragment reads / MFMAs ("DMA alone"), 3 = both (loop
skeleton).  Average µs per launch, order-balanced (two rounds, the second reported), TFLOP/s fp32-equivalent
(2·9·Cin·Cout per output pixel).  Then the K-block loop unroll (esr_wgrad3d_set_unroll 1 / 2 / 4 = product since round 6): µs per
launch and whether the partials are bitwise the product's.

    python tools/wgrad3d_split.py
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'explorable-super-resolution_old_amd'))
from esr_amd import _lib  # noqa: E402
from esr_amd import engine as E  # noqa: E402

SHAPES = [  # name, cin, in_cp, cout, d_cp, d_coff  (RDB convs 1, 3 and 5 of the latent C3 step)
    ('rdb_conv1', 72, 200, 32, 264, 72),
    ('rdb_conv3', 136, 200, 32, 264, 136),
    ('rdb_conv5', 200, 200, 64, 264, 200),
]


def main():
    lib = _lib.load_ablation()
    dev = torch.device('cuda')
    B, H, W = 16, 96, 96
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    x = E.to_split(torch.randn(B, H + 2, W + 2, 200, device=dev))
    ds = E.to_split(torch.randn(B, H + 2, W + 2, 264, device=dev))
    for name, cin, in_cp, cout, d_cp, d_coff in SHAPES:
        chunks = (cin + 31) // 32
        ntiles = B * ((H + 7) // 8) * ((W + 31) // 32)
        splits = max(1, min(128, 256 // chunks, ntiles))
        cout_pad = 64 if cout > 32 else 32
        n = 9 * 32 * chunks * cout_pad + cout_pad
        part = torch.empty(splits * n, device=dev)
        flops = 2 * 9 * cin * cout * B * H * W

        def run(mode, reps):
            lib.esr_wgrad3d_set_dbg(mode)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                _lib.check(lib.esr_conv3x3_wgrad(x.data_ptr(), in_cp, cin, 14, ds.data_ptr(), d_cp, d_coff, cout, B, H,
                                                 W, splits, part.data_ptr(), st), 'wgrad')
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1000 / reps

        row = {'splits': splits, 'workgroups': chunks * splits}
        for rnd in range(2):
            for mode in (0, 1, 2, 3):
                run(mode, 3)
                us = run(mode, 30)
                if rnd == 1:
                    row['mode%d_us' % mode] = round(us, 2)
                    row['mode%d_tflops' % mode] = round(flops / us / 1e6, 1)
        lib.esr_wgrad3d_set_dbg(0)
        parts, times = {}, {1: [], 2: [], 4: []}
        for order in ((2, 4, 1), (4, 1, 2), (1, 2, 4), (2, 4, 1)):  # rotated: each position once, the first twice
            for u in order:
                lib.esr_wgrad3d_set_unroll(u)
                part.fill_(float('nan'))
                run(0, 3)
                times[u].append(round(run(0, 30), 2))
                parts[u] = part.clone()
        for u in (1, 2, 4):
            row['unroll%d_us' % u] = times[u]
        row['unroll1_bitwise'] = bool(torch.equal(parts[1], parts[2]))
        row['unroll4_bitwise'] = bool(torch.equal(parts[4], parts[2]))
        lib.esr_wgrad3d_set_unroll(4)
        print(name, json.dumps(row), flush=True)


if __name__ == '__main__':
    main()
