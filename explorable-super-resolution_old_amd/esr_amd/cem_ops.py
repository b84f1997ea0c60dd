"""CEM image resampling on the device: the reference's NumPy `imresize` / `DT_Satisfying_Upscale` family
(imresize_CEM.py:7-71; CEMnet.py:53-57, 88-100) as batched launches of the CEM stencils (csrc/esr_cem.hip).

Every function takes float32 ROCm tensors whose last two dims are (H, W); leading dims are any number of image planes
(the filters are depthwise and identical per plane).  The stencils work on stacks of 3 planes, so the plane count is
rounded up to a multiple of 3 with zero planes.  Filters are 2-D float32 device tensors; the callers
(imresize_CEM.imresize, CEMnet) derive them from the float64 design exactly as the reference's conv2 calls use them:

    scipy conv2(x, K)  ==  cross-correlation with rot180(K)

    downscale 1/sf   conv2(edge_pad(x), rot180(k_up / sf²), 'valid')[pre::sf]   ->  esr_cem_down,   w = k_up / sf²
    upscale ×sf      conv2(edge_pad(zero_stuff(x)), k_up, 'valid')             ->  esr_cem_up_add, w = rot180(k_up)
    conv2(x, inv, 'same')  (zero padding)                                     ->  esr_cem_inv,    w = rot180(inv)

Edge padding is the stencils' index clamping; the zero-padded variants pad with zeros first (a clamped read of a zero
border is zero).  There is no CPU path.
"""
import ctypes

import torch
import torch.nn.functional as F

from . import _lib


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check(x, *ws):
    for t in (x,) + ws:
        if not t.is_cuda or t.dtype != torch.float32:
            raise RuntimeError('esr_amd.cem_ops: tensors must be float32 on a ROCm device (this build has no CPU path)')
    for w in ws:
        if w.dim() != 2 or w.shape[0] != w.shape[1] or not w.shape[0] & 1:
            raise RuntimeError('esr_amd.cem_ops: filters must be square with an odd side, got %s' % (tuple(w.shape),))


def _planes(x):
    """[..., H, W] -> ([P, 3, H, W] contiguous, number of real planes)."""
    H, W = x.shape[-2:]
    flat = x.reshape(-1, H, W)
    n = flat.shape[0]
    P = -(-n // 3)
    if 3 * P != n:
        flat = torch.cat([flat, flat.new_zeros(3 * P - n, H, W)])
    return flat.contiguous().view(P, 3, H, W), n


def _unplanes(y, n, lead):
    H, W = y.shape[-2:]
    return y.reshape(-1, H, W)[:n].reshape(*lead, H, W)


def phase(sf):
    """calc_strides(None, sf) pre_stride (imresize_CEM.py:83-85): the sample kept / stuffed within each sf-block."""
    return sf - sf // 2 - 1


def downscale(x, w, sf, zero_pad=False):
    """y[i, j] = sum_uv w[u, v] x[sf*i+ph+u-k//2, sf*j+ph+v-k//2], x edge-padded (or zero-padded); H, W % sf == 0."""
    _check(x, w)
    lead, (H, W) = x.shape[:-2], x.shape[-2:]
    if H % sf or W % sf:
        raise RuntimeError('esr_amd.cem_ops.downscale: image size %dx%d is not a multiple of %d' % (H, W, sf))
    k = w.shape[0]
    c = -(-(k // 2) // sf) if zero_pad else 0       # LR pixels of zero border (enough for the kernel's reach)
    if c:
        x = F.pad(x.reshape(-1, H, W), (sf * c,) * 4)
    xp, n = _planes(x)
    P, _, Hp, Wp = xp.shape
    y = torch.empty(P, 3, Hp // sf, Wp // sf, device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().esr_cem_down(xp.data_ptr(), None, y.data_ptr(), P, Hp // sf, Wp // sf, sf, phase(sf),
                                        w.contiguous().data_ptr(), k, 1, _stream(x)), 'esr_cem_down')
    if c:
        y = y[:, :, c:c + H // sf, c:c + W // sf]
    return _unplanes(y, n, lead)


def upscale(x, w, sf, zero_pad=False, crop=0):
    """y = xcorr(pad(S), w) with S = x zero-stuffed at the stride phase on the ×sf grid, pad = edge (clamp) or zero,
    then `crop` HR pixels removed from every side (fused: the cropped border is never computed)."""
    _check(x, w)
    lead, (h, wd) = x.shape[:-2], x.shape[-2:]
    k = w.shape[0]
    c = -(-(k // 2) // sf) if zero_pad else 0
    if c:
        x = F.pad(x.reshape(-1, h, wd), (c,) * 4)
    xp, n = _planes(x)
    P, _, hp, wp = xp.shape
    M = sf * c + crop
    if 2 * M >= sf * hp or 2 * M >= sf * wp:
        raise RuntimeError('esr_amd.cem_ops.upscale: crop %d leaves an empty image' % crop)
    zero = torch.zeros(P, 3, sf * hp, sf * wp, device=x.device, dtype=torch.float32)
    y = torch.empty(P, 3, sf * hp - 2 * M, sf * wp - 2 * M, device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().esr_cem_up_add(xp.data_ptr(), zero.data_ptr(), y.data_ptr(), P, hp, wp, sf, phase(sf),
                                          w.contiguous().data_ptr(), k, M, _stream(x)), 'esr_cem_up_add')
    return _unplanes(y, n, lead)


def filter_same(x, w, zero_pad=True):
    """xcorr(pad(x), w) at the input resolution ('same' size); zero or edge (replicate) padding."""
    _check(x, w)
    lead, (H, W) = x.shape[:-2], x.shape[-2:]
    k = w.shape[0]
    p = k // 2 if zero_pad else 0
    if p:
        x = F.pad(x.reshape(-1, H, W), (p,) * 4)
    xp, n = _planes(x)
    P, _, Hp, Wp = xp.shape
    y = torch.empty_like(xp)
    _lib.check(_lib.load().esr_cem_inv(xp.data_ptr(), y.data_ptr(), P, Hp, Wp, w.contiguous().data_ptr(), k,
                                       _stream(x)), 'esr_cem_inv')
    if p:
        y = y[:, :, p:p + H, p:p + W]
    return _unplanes(y, n, lead)
