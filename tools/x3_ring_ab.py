#!/usr/bin/env python3
"""A/B of the two x3 3×3-conv kernels for N <= 32 (classic two-stage vs ring, esr_x3_set_kernel) on the config-2/3
shapes: same inputs, outputs compared bitwise (same MFMA order per accumulator), time per launch with HIP events."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
import torch  # noqa: E402
from esr_amd import _lib, engine  # noqa: E402

lib = _lib.load()
dev = torch.device('cuda:0')
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
ovf = torch.zeros(1, dtype=torch.int32, device=dev)
B = int(os.environ.get('AB_B', '32'))
VARIANTS = [int(v) for v in os.environ.get('AB_VARIANTS', '0,1,2').split(',')]
NAMES = {0: 'classic 1-stage x2 WG', 1: 'auto', 2: 'ring', 15: 'ring+stagger', 3: 'dbg:no-dma', 4: 'dbg:no-compute', 5: 'dbg:no-mfma',
         6: 'nodma+nobar', 7: 'nodma+slot0', 8: 'nodma+nopred', 9: 'nodma+all3', 10: 'nodma+nomfma',
         11: 'reads+restage', 12: 'reads only', 13: 'no-ep-stores', 14: 'dma only,no ep', 16: 'pring pf1',
         17: 'pring pf2', 18: 'ring (compiler reads)', 19: 'probe:const-A', 20: 'classic (compiler reads)', 21: 'classic pf1', 22: 'classic 2-stage', 23: 'n64 8-row 1-stage x2 WG', 25: 'n32 8-row 1-stage x3 WG', 26: 'n32 16-row 1-stage x2 WG', 27: 'n32 16-row direct-ep', 28: 'n32 8-row direct-ep', 29: 'dbg:16-row no-dma', 30: 'dbg:16-row no-compute'}
COUT = int(os.environ.get('AB_COUT', '32'))
REPS = int(os.environ.get('AB_REPS', '50'))
HWS = [int(v) for v in os.environ.get('AB_HW', '148,96').split(',')]
CINS = [int(v) for v in os.environ['AB_CIN'].split(',')] if 'AB_CIN' in os.environ else None
for H, W in ((h, h) for h in HWS):
    for cin in CINS or ((64, 128, 160) if COUT <= 32 else (192,)):
        cout, cp = COUT, 192
        g = torch.Generator(device='cpu').manual_seed(cin)
        x = torch.zeros(B, H + 2, W + 2, cp)
        x[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, generator=g) * 2 - 1
        x = x.to(dev)
        w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(dev)
        b = (torch.rand(cout, generator=g) * 0.02 - 0.01).to(dev)
        wx, scale = engine.pack_x3(engine.pack_conv_weight(w, list(range(cin)), 32 if cout <= 32 else 64))
        xs = engine.to_split(x)
        res = {}
        for variant in VARIANTS:
            lib.esr_x3_set_kernel(variant % 1000)
            lib.esr_x3_set_tile_map(0 if variant >= 1000 else 1)  # variant + 1000: row-major block order
            out = torch.zeros(B, H + 2, W + 2, cp, device=dev)
            o = engine._conv_out(out, cp, cin if cin + cout <= cp else 0, H, W, True)

            def run():
                return lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                              cout, ctypes.byref(o), ovf.data_ptr(), stream)
            for _ in range(3):
                _lib.check(run(), 'conv_x3')
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(REPS):
                run()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / REPS * 1e3
            fl = 2.0 * B * H * W * 9 * cin * cout
            res[variant] = (us, out)
            print('B=%d %dx%d cin=%d cout=%d %-14s: %8.1f us  %6.1f TFLOP/s' % (
                B, H, W, cin, cout, NAMES.get(variant % 1000, str(variant)) + ('+rowmajor' if variant >= 1000 else ''), us, fl / us / 1e6), flush=True)
        v0 = VARIANTS[0]
        for v in VARIANTS[1:]:
            same = torch.equal(res[v0][1], res[v][1]) if v % 1000 < 3 or (v % 1000 >= 15 and v % 1000 not in (19, 29, 30)) else True
            print('   %s/%s speedup %.3f, outputs bitwise equal: %s' % (NAMES.get(v % 1000, str(v)) + ('+rowmajor' if v >= 1000 else ''), NAMES.get(v0 % 1000, str(v0)), res[v0][0] / res[v][0],
                                                                      same), flush=True)
            assert same
lib.esr_x3_set_kernel(1)
lib.esr_x3_set_tile_map(1)
