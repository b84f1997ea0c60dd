#!/usr/bin/env python3
"""Where a workgroup of the production N = 32 x3 conv (12-column tiles, three per CU) spends its time: the stamped
diagnostic build (ablation library, esr_x3_set_kernel(87), esr_x3c_set_stamps) records s_memrealtime (100 MHz) on wave 0 at the
kernel start, per K chunk before its LDS-DMA issue (A), after its wait + barrier (B) and after its compute (C), and
after the epilogue.  Per shape it prints the launch's span, the shares of workgroup time in: chunk-0 load (prologue),
later chunks' load waits (B - A), compute (C - B), the barrier before the next chunk's DMA (A' - C), and the
epilogue; and how the workgroups' start times spread over the launch (rounds).  Only shares mean anything: the
stamps' waits forbid overlaps the real kernel has (MI355X guide §7, in-kernel stamps).

    ESR_AMD_LIB=exp_lib/libesr_exp.so python3 tools/x3c_stamps.py [B:H:cin[:W] ...]   (default 32:148:128 16:96:128 8:172:128)

The last lines compare the workgroups of the last column strip (partial when W is no multiple of 12) with the rest.
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from esr_amd import _lib, engine  # noqa: E402

NS, NCH = 38, 12


def main():
    lib = _lib.load()
    if not hasattr(lib, 'esr_x3c_set_stamps'):
        raise SystemExit('needs the ablation library (ESR_AMD_LIB=exp_lib/libesr_exp.so)')
    lib.esr_x3c_set_stamps.argtypes = [ctypes.c_void_p]
    dev = torch.device('cuda:0')
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ovf = torch.zeros(1, dtype=torch.int32, device=dev)
    shapes = sys.argv[1:] or ['32:148:128', '16:96:128', '8:172:128']
    for spec in shapes:
        f = [int(v) for v in spec.split(':')]
        B, H, cin = f[:3]
        W = f[3] if len(f) > 3 else H
        cout, cp = 32, 192
        g = torch.Generator(device='cpu').manual_seed(cin)
        x = torch.zeros(B, H + 2, W + 2, cp)
        x[:, 1:-1, 1:-1, :cin] = torch.rand(B, H, W, cin, generator=g) * 2 - 1
        xs = engine.to_split(x.to(dev))
        w = (torch.randn(cout, cin, 3, 3, generator=g) * 0.05).to(dev)
        b = (torch.rand(cout, generator=g) * 0.02 - 0.01).to(dev)
        wx, scale = engine.pack_x3(engine.pack_conv_weight(w, list(range(cin)), 32))
        out = torch.zeros(B, H + 2, W + 2, cp, device=dev)
        o = engine._conv_out(out, cp, cin if cin + cout <= cp else 0, H, W, True)
        ntiles = ((W + 11) // 12) * ((B * (H + 2) - 2 + 31) // 32)
        st = torch.zeros(ntiles * NS, dtype=torch.int64, device=dev)

        def run():
            _lib.check(lib.esr_conv3x3_fwd_x3(xs.data_ptr(), B, H, W, cp, cin, wx.data_ptr(), b.data_ptr(), scale,
                                              cout, ctypes.byref(o), ovf.data_ptr(), stream), 'conv_x3')
        lib.esr_x3_set_kernel(1)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        t_prod = e0.elapsed_time(e1) / 10 * 1e3
        lib.esr_x3_set_kernel(87)
        if lib.esr_x3c_set_stamps(ctypes.c_void_p(st.data_ptr())) != 0:
            raise SystemExit('esr_x3c_set_stamps failed')
        for _ in range(3):
            run()
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        t_diag = e0.elapsed_time(e1) * 1e3
        lib.esr_x3c_set_stamps(None)
        lib.esr_x3_set_kernel(1)
        s = st.view(ntiles, NS).cpu().numpy().astype(np.float64)
        nch = (cin + 15) // 16
        t0, tend = s[:, 0], s[:, NS - 1]
        A = s[:, 1:1 + 3 * nch:3]
        Bq = s[:, 2:2 + 3 * nch:3]
        C = s[:, 3:3 + 3 * nch:3]
        span = tend.max() - t0.min()
        clk = 0.1  # s_memrealtime: 100 MHz ticks (GHz units below: ticks / clk / 1e3 = us)
        print('   stamped span %.1f us (launch %.1f us)' % (span / clk / 1e3, t_diag))
        wg = tend - t0
        parts = {
            'prologue (start -> chunk 0 issued)': (A[:, 0] - t0).sum(),
            'chunk 0 load wait': (Bq[:, 0] - A[:, 0]).sum(),
            'later chunks: load wait (B - A)': (Bq[:, 1:] - A[:, 1:]).sum(),
            'compute (C - B)': (C - Bq).sum(),
            'barrier before next DMA (A\' - C)': (A[:, 1:] - C[:, :-1]).sum(),
            'epilogue (last C -> end)': (tend - C[:, -1]).sum(),
        }
        tot = wg.sum()
        print('B=%d %dx%d cin=%d: %d workgroups; production %.1f us, stamped build %.1f us ' % (B, H, W, cin, ntiles, t_prod, t_diag), flush=True)
        tiles_x = (W + 11) // 12
        b = np.arange(ntiles)  # stamps are per blockIdx; its tile under the XCD map (esr_conv_x3c.hip xcd_tile)
        x, l, q, r = b % 8, b // 8, ntiles // 8, ntiles % 8
        tile = np.where(x < r, x * (q + 1) + l, r * (q + 1) + (x - r) * q + l)
        tx = tile % tiles_x
        last = tx == tiles_x - 1
        for k, v in parts.items():
            print('   %-38s %5.1f %%   (%.2f us per workgroup)' % (k, 100 * v / tot, v / ntiles / clk / 1e3))
        rel = (t0 - t0.min()) / span
        hist = np.histogram(rel, bins=10, range=(0, 1))[0]
        print('   workgroup start times over the launch (deciles): %s' % ' '.join(str(int(v)) for v in hist))
        print('   mean workgroup duration %.1f us; per chunk: load wait %.2f us, compute %.2f us (chunks 1..%d)'
              % (wg.mean() / clk / 1e3, (Bq[:, 1:] - A[:, 1:]).mean() / clk / 1e3,
                 (C[:, 1:] - Bq[:, 1:]).mean() / clk / 1e3, nch - 1), flush=True)
        for name, m in (('last strip', last), ('other strips', ~last)):
            print('   %-12s workgroups %4d: duration %.2f us, load wait %.2f, compute %.2f, epilogue %.2f us' % (
                name, m.sum(), wg[m].mean() / clk / 1e3, (Bq[m][:, 1:] - A[m][:, 1:]).mean() / clk / 1e3,
                (C[m][:, 1:] - Bq[m][:, 1:]).mean() / clk / 1e3, (tend[m] - C[m][:, -1]).mean() / clk / 1e3), flush=True)


if __name__ == '__main__':
    main()
