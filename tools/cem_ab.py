#!/usr/bin/env python3
"""Timing of the CEM stencil kernels at the config-2 shape, tiled (default) vs direct (esr_cem_set_direct(1)),
interleaved rounds; algorithmic bytes and FLOPs per launch as DESIGN.md §4 counts them."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from esr_amd import _lib  # noqa: E402
from oracle import esr_oracle as O  # noqa: E402

lib = _lib.load()
dev = torch.device('cuda:0')
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
design = O.cem_design(4)
print({k: (getattr(v, 'shape', v)) for k, v in design.items()} if isinstance(design, dict) else type(design))
B, H, W = 32, 148, 148
ki, kd, M, ph = 27, 17, 40, 1
for k in ('inv', 'ki', 'kd', 'ph', 'M'):
    pass
g = torch.Generator().manual_seed(0)
r = torch.randn(B, 3, H, W, generator=g).to(dev)
wi = torch.randn(ki, ki, generator=g).to(dev) * 0.05
wd = torch.randn(kd, kd, generator=g).to(dev) * 0.05
gen = torch.randn(B, 3, 4 * H, 4 * W, generator=g).to(dev)
lr = torch.randn(B, 3, H, W, generator=g).to(dev)
q = torch.empty_like(r)
out = torch.empty(B, 3, 4 * H - 2 * M, 4 * W - 2 * M, device=dev)
ops = {
    'cem_down': (lambda: lib.esr_cem_down(gen.data_ptr(), lr.data_ptr(), r.data_ptr(), B, H, W, 4, ph, wd.data_ptr(), kd, 0, st),
                 (gen.numel() + 2 * r.numel()) * 4),
    'cem_inv': (lambda: lib.esr_cem_inv(r.data_ptr(), q.data_ptr(), B, H, W, wi.data_ptr(), ki, st), 2 * r.numel() * 4),
    'cem_up_add': (lambda: lib.esr_cem_up_add(q.data_ptr(), gen.data_ptr(), out.data_ptr(), B, H, W, 4, ph, wd.data_ptr(),
                                              kd, M, st), (q.numel() + 2 * out.numel()) * 4),
}
res = {}
for rnd in range(4):
    for direct in ((0, 1) if rnd % 2 == 0 else (1, 0)):
        lib.esr_cem_set_direct(direct)
        for name, (fn, nbytes) in ops.items():
            fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                fn()
            e.record()
            torch.cuda.synchronize()
            res.setdefault((name, direct), []).append(s.elapsed_time(e) / 20 * 1e3)
lib.esr_cem_set_direct(0)
for (name, direct), t in sorted(res.items()):
    nb = ops[name][1]
    print('%-11s %-6s min %7.1f us  %6.2f TB/s algorithmic (%.1f MB)' % (name, 'direct' if direct else 'tiled', min(t),
                                                                      nb / min(t) / 1e6, nb / 1e6))
