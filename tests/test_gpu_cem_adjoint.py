"""GPU parity of esr_cem_adjoint (csrc/esr_train.hip), the exact adjoint of the CEM stencils with replicate padding
(CEMnet.py:149-162), against float64 autograd (vjp) of the same stencil on the CPU, for the three calls the generator
backward makes (train_engine.generator_backward: Upscale_OP, the inverse filter, DownscaleOP with alpha -1 accumulated)
and for odd sizes where the clamped border rows and columns are a large share.  Bar: 1e-6 normwise (fp32)."""
import ctypes

import pytest
import torch

from conftest import normwise_rel

from esr_amd import _lib

pytestmark = pytest.mark.gpu


def _stencil(x, w, s, c, Oy, Ox):
    """out[o] = sum_u w[u] x[clamp(s*o + c + u - K//2)] per plane (2-D, replicate clamp), x [P][Ly][Lx]."""
    K = w.shape[0]
    Ly, Lx = x.shape[1:]
    iy = (s * torch.arange(Oy)[:, None] + c + torch.arange(K)[None, :] - K // 2).clamp(0, Ly - 1)  # [Oy][K]
    ix = (s * torch.arange(Ox)[:, None] + c + torch.arange(K)[None, :] - K // 2).clamp(0, Lx - 1)  # [Ox][K]
    g = x[:, iy[:, None, :, None], ix[None, :, None, :]]  # [P][Oy][Ox][K][K]
    return (g * w).sum((-2, -1))


@pytest.mark.parametrize('P,Ly,Lx,K,s,c,os_,oc,alpha,acc', [
    (6, 64, 72, 17, 1, 0, 4, 1, 1.0, 0),     # Upscale_OP adjoint (HR -> LR phase samples), sf 4
    (6, 16, 18, 13, 1, 0, 1, 0, 1.0, 0),     # inverse filter adjoint (LR -> LR)
    (6, 64, 72, 17, 4, 1, 1, 0, -1.0, 1),    # DownscaleOP adjoint (LR -> HR), accumulated with alpha -1
    (3, 13, 11, 17, 4, 1, 1, 0, 1.0, 0),     # tiny HR grid: most outputs on or near the clamped border
    (3, 22, 26, 9, 2, 0, 2, 0, 1.0, 0),      # sf 2 (phase 0)
    (4, 70, 90, 41, 1, 0, 1, 0, 1.0, 0),     # inverse filter adjoint at the KernelGAN-recipe size (41², tiled path)
    (2, 37, 130, 41, 1, 0, 1, 0, -0.5, 1),   # ... accumulated, several 64 × 16 output tiles, ragged edges
    (2, 3, 5, 41, 1, 0, 1, 0, 1.0, 0),       # ... grid far smaller than the taps (one interior output)
    (2, 2, 9, 13, 1, 0, 1, 0, 1.0, 0),       # ... no interior rows (generic path only)
])
def test_cem_adjoint_vs_float64_vjp(gpu_device, P, Ly, Lx, K, s, c, os_, oc, alpha, acc):
    gen = torch.Generator().manual_seed(K * 100 + Ly)
    w = torch.randn(K, K, generator=gen, dtype=torch.float64) / K
    Oy, Ox = -(-Ly // s), -(-Lx // s)  # forward output size: the strided grid over the input
    if s == 1:
        Oy, Ox = Ly, Lx
    g = torch.randn(P, Oy, Ox, generator=gen, dtype=torch.float64)
    x = torch.zeros(P, Ly, Lx, dtype=torch.float64, requires_grad=True)
    ref, = torch.autograd.grad(_stencil(x, w, s, c, Oy, Ox), x, g)  # F^T g on the full input grid
    ref = alpha * ref[:, oc::os_, oc::os_]
    base = torch.randn(ref.shape, generator=gen, dtype=torch.float64)
    if acc:
        ref = ref + base
    lib = _lib.load()
    gd, wd = g.float().to(gpu_device), w.float().to(gpu_device)
    out = base.float().to(gpu_device) if acc else torch.empty(ref.shape, device=gpu_device)
    st = ctypes.c_void_p(torch.cuda.current_stream(gpu_device).cuda_stream)
    _lib.check(lib.esr_cem_adjoint(gd.data_ptr(), P, Oy, Ox, wd.data_ptr(), K, s, c, Ly, Lx, os_, oc, alpha, acc,
                                   out.data_ptr(), st), 'esr_cem_adjoint')
    torch.cuda.synchronize()
    assert normwise_rel(out.double().cpu(), ref) < 1e-6
    # the interior fast paths (default: per-output, or the tiled stride-1 kernel) are bitwise the generic per-tap range
    # search
    out2 = base.float().to(gpu_device) if acc else torch.empty(ref.shape, device=gpu_device)
    _lib.check(lib.esr_cem_adjoint(gd.data_ptr(), P, Oy, Ox, wd.data_ptr(), K, s, c, Ly, Lx, os_, oc, alpha, acc | 2,
                                   out2.data_ptr(), st), 'esr_cem_adjoint generic')
    torch.cuda.synchronize()
    if s == 1 and os_ == 1 and oc == 0 and Ly >= 3 and Lx >= 3:
        # the stride-1 (inverse filter) adjoint: interior outputs tiled, bitwise; the clamped border rows / columns
        # are summed by a block per output in a tree order
        assert torch.equal(out[:, 1:-1, 1:-1], out2[:, 1:-1, 1:-1])
        assert normwise_rel(out.double().cpu(), out2.double().cpu()) < 1e-6
    else:
        assert torch.equal(out, out2)
