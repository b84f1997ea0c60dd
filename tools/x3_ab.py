#!/usr/bin/env python3
"""Interleaved A/B of x3 3x3-conv kernel variants (esr_x3_set_kernel) at the bench shapes.

Env: AB_VARIANTS (comma list; variant + 1000 = row-major block order), AB_DIAG (variants whose outputs are garbage by
design: not compared), AB_COUT, AB_CIN, AB_HW, AB_B, AB_REPS, AB_ROUNDS.  Every variant runs once per round, rounds
interleaved (MI355X clocks drift between blocks of one variant); the min and median over rounds are printed.  Outputs
of the non-diagnostic variants are compared bitwise with the first variant."""
import ctypes
import os
import statistics
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
VARIANTS = [int(v) for v in os.environ.get('AB_VARIANTS', '1').split(',')]
DIAG = {int(v) for v in os.environ.get('AB_DIAG', '').split(',') if v}
COUT = int(os.environ.get('AB_COUT', '32'))
REPS = int(os.environ.get('AB_REPS', '20'))
ROUNDS = int(os.environ.get('AB_ROUNDS', '4'))
HWS = [int(v) for v in os.environ.get('AB_HW', '148').split(',')]
CINS = [int(v) for v in os.environ['AB_CIN'].split(',')] if 'AB_CIN' in os.environ else \
    ((64, 128, 160) if COUT <= 32 else (192,))
for H in HWS:
    W = H
    for cin in CINS:
        cout, cp = COUT, 192 if cin <= 192 else 200
        g = torch.Generator(device='cpu').manual_seed(cin)
        x = torch.zeros(B, H + 2, W + 2, cp)
        x[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, generator=g) * 2 - 1
        x = x.to(dev)
        w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(dev)
        b = (torch.rand(cout, generator=g) * 0.02 - 0.01).to(dev)
        wx, scale = engine.pack_x3(engine.pack_conv_weight(w, list(range(cin)), 32 if cout <= 32 else 64))
        xs = engine.to_split(x)
        outs, times = {}, {v: [] for v in VARIANTS}
        fl = 2.0 * B * H * W * 9 * cin * cout
        for rnd in range(ROUNDS):
            for variant in (VARIANTS if rnd % 2 == 0 else VARIANTS[::-1]):
                lib.esr_x3_set_kernel(variant % 1000)
                lib.esr_x3_set_tile_map(0 if variant >= 1000 else 1)
                out = outs.get(variant)
                if out is None:
                    out = outs[variant] = torch.zeros(B, H + 2, W + 2, cp, device=dev)
                coff = cin if cin + cout <= cp else 0
                o = engine._conv_out(out, cp, coff, H, W, True)

                def run():
                    return lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                                  cout, ctypes.byref(o), ovf.data_ptr(), stream)
                for _ in range(2):
                    _lib.check(run(), 'conv_x3')
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(REPS):
                    run()
                e.record()
                torch.cuda.synchronize()
                times[variant].append(s.elapsed_time(e) / REPS * 1e3)
        v0 = VARIANTS[0]
        for v in VARIANTS:
            t = times[v]
            same = ''
            if v not in DIAG and v != v0:
                a = engine.from_split(outs[v][..., coff:coff + cout].contiguous()).double()
                r = engine.from_split(outs[v0][..., coff:coff + cout].contiguous()).double()
                err = float((a - r).abs().max() / r.abs().max())
                same = ' bitwise==v%d: %s normwise %.1e' % (v0, torch.equal(outs[v], outs[v0]), err)
            print('B=%d %dx%d cin=%d cout=%d v%-5d min %7.1f us  med %7.1f us  %6.1f TFLOP/s  x%.3f vs v%d%s' % (
                B, H, W, cin, cout, v, min(t), statistics.median(t), fl / min(t) / 1e6, min(times[v0]) / min(t), v0,
                same), flush=True)
lib.esr_x3_set_kernel(1)
lib.esr_x3_set_tile_map(1)
