"""Discriminator convolutions on the HIP gather-GEMM kernels (csrc/esr_dconv.hip), differentiable to any order.

Discriminator_VGG_128_ (architecture.py:222-284) is built from conv_block(CNA) layers (block.py:129-156): Conv2d with
k = 3 / 4 / 8 / 1, stride 1 / 2, then BatchNorm + LeakyReLU.  The D step (SRRaGAN_model.py:360-433) needs their forward,
data gradient and weight gradient, and the WGAN-GP penalty (loss.py:244-263: autograd.grad(create_graph=True) followed
by .backward()) differentiates the data gradient once more.  The three maps

    conv  (x, w)  -> y        DConvFn
    dgrad (gy, w) -> gx       DgradFn     (adjoint of conv in x)
    wgrad (x, gy) -> gw       WgradFn     (adjoint of conv in w)

are bilinear and each one's backward is made of the other two, so autograd can differentiate through them any number
of times with every convolution running on the MFMA kernels.  Tensors are channels-last: the module-level wrapper
HipConv2d takes/returns NCHW tensors with NHWC storage (torch.channels_last), which BatchNorm / LeakyReLU accept as is.
There is no CPU path: a CPU tensor raises.
"""
import ctypes
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

MAX_TAPS = 64
# Precision of the discriminator convolutions (forward, data and weight gradients): 'x3' = split-f16 operands (hi, lo)
# with per-K-step power-of-two scaling on f16 MFMA (3 products, ~2^-22 per product), 'x6' = three f16 pieces and six
# products (each operand to ~33 bits: an fp32 FMA chain's accuracy, esr_dconv.hip), 'f32' = exact fp32 MFMA.
PRECISION = os.environ.get('ESR_DCONV_PRECISION', 'x3')
# esr_dconv_* `prec` argument (include/esr_amd.h): per call, the library keeps no precision state
_LIB_MODE = {'f32': 0, 'x3': 1, 'x6': 3}
# x3: 128-wide N tiles where the grid allows (prec 1); '0' = 64-wide only (prec 2, identical results; A/B)
if os.environ.get('ESR_DCONV_NB128', '1') == '0':
    _LIB_MODE['x3'] = 2
# 4×4 stride-2 convs (and any even k at stride 2) and their data gradients as (k/2)×(k/2)-tap stride-1 convs over the
# space-to-depth source / into the depth-to-space gradient (esr_dconv_fwd_sd, one launch each); '0' = the direct
# stride-2 gather and one launch per phase class (A/B)
S2D = os.environ.get('ESR_DCONV_S2D', '1') != '0'
# x3 halo-tile launches take their weights pre-split (one scale per tensor, LDS-DMA'd: no per-step max / split in the
# kernel); '0' = the kernel splits the fp32 weight slab per K step (A/B)
PRESPLIT = os.environ.get('ESR_DCONV_PRESPLIT', '1') != '0'
# conv bias gradients (Σ over pixels of the output gradient) accumulated in float64 ('0': float32 sums)
BIAS_F64 = os.environ.get('ESR_DCONV_BIAS_F64', '0') != '0'
# first-order bias gradients by esr_colsum (float64 partials, one pass); '0' = PyTorch's sum (A/B)
COLSUM = os.environ.get('ESR_DCONV_COLSUM', '1') != '0'


def set_precision(p):
    """Select 'x3', 'x6' or 'f32' for the discriminator convolutions (the default of every launch that does not name
    its own); returns the previous setting."""
    global PRECISION
    if p not in _LIB_MODE:
        raise ValueError(p)
    prev, PRECISION = PRECISION, p
    return prev


def _mode(prec):
    """The library's `prec` code for a launch: `prec` ('x3' / 'x6' / 'f32') or, if None, the module default."""
    return _LIB_MODE[PRECISION if prec is None else prec]


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _i32(vals):
    return (ctypes.c_int32 * max(1, len(vals)))(*vals)


def _check_dev(*ts):
    for t in ts:
        if t is not None and (not t.is_cuda or t.dtype != torch.float32):
            raise RuntimeError('esr_amd.dconv: discriminator tensors must be float32 on a ROCm device '
                               '(this build has no CPU path)')


def out_size(n, k, s, p):
    return (n + 2 * p - k) // s + 1


class _Packed:
    """Packed weights of one launch: wp [T][nck][n_pad][32] fp32 (esr_dconv_fwd's layout) and, built on first use by an
    x3 launch, their pre-split form for the halo-tile kernel (include/esr_amd.h esr_dconv_fwd_sd w_split / w_exp)."""
    __slots__ = ('wp', 'nck', 'n_pad', '_split')

    def __init__(self, wp, nck, n_pad):
        self.wp, self.nck, self.n_pad, self._split = wp, nck, n_pad, None

    def __iter__(self):
        return iter((self.wp, self.nck, self.n_pad))

    def split(self):
        """(f16 rows [T][nck][n_pad][8 slots][8], int32 [1] exponent E): v = wp·2^E with one power of two per tensor
        (max |v| in [2^14, 2^15)), hi = f16(v), lo = f16(v - hi); logical slot l = piece·4 + k (8 channels each) stored
        at position l ^ ((n >> 1) & 7).  Device ops only (no host sync)."""
        if self._split is None:
            wp = self.wp
            T, nck, n_pad, _ = wp.shape
            rows = torch.empty(T, nck, n_pad, 8, 8, device=wp.device, dtype=torch.float16)
            e = torch.empty(1, device=wp.device, dtype=torch.int32)
            _check_dev(wp)
            scratch = torch.empty(512, device=wp.device)  # esr_dconv_presplit: two launches, no host sync
            _lib.check(_lib.load().esr_dconv_presplit(wp.data_ptr(), T * nck * n_pad, n_pad, scratch.data_ptr(),
                                                      rows.data_ptr(), e.data_ptr(), _stream(wp)),
                       'esr_dconv_presplit')
            self._split = (rows, e)
        return self._split


def _pack(wt, n_out):
    """wt [T][K][N] -> packed [T][nck][n_pad][32] (esr_dconv_fwd's weight layout)."""
    T, K, N = wt.shape
    nck = (K + 31) // 32
    n_pad = 64 * ((n_out + 63) // 64)
    buf = wt.new_zeros(T, nck * 32, n_pad)
    buf[:, :K, :N] = wt
    return _Packed(buf.view(T, nck, 32, n_pad).permute(0, 1, 3, 2).contiguous(), nck, n_pad)


def _packed(w, key, make):
    """make() -> packed weights of `w` (_pack's result), memoised on w while w is a discriminator parameter
    (HipConv2d marks its weight) that is unchanged: same storage and version counter (and FlatAdam buffer version),
    i.e. until the optimiser step, load_state_dict or a .data swap (the generator's packing is keyed the same way,
    engine._param_key).  The
    discriminator runs ~4 forwards and their (double) backwards per training step on the same weights; without the
    memo every launch repacks them (3 PyTorch ops each)."""
    if not getattr(w, '_esr_dconv_param', False):
        return make()
    memo = getattr(w, '_esr_packs', None)
    if memo is None:
        memo = w._esr_packs = {}
    fl = getattr(w, '_esr_flat', None)  # a FlatAdam view: its in-place update bumps the buffer's version, not w's
    ver = (w.data_ptr(), w._version, None if fl is None else fl._version)
    hit = memo.get(key)
    if hit is not None and hit[0] == ver:
        return hit[1]
    val = make()
    memo[key] = (ver, val)
    return val


def _gather(src, packed, bias, out, MH, MW, omy, oay, omx, oax, smy, smx, offy, offx, s2d_pad=None, d2s_pad=None,
            prec=None):
    """One esr_dconv_fwd launch: src [B][Hs][Ws][C] and out [B][Ho][Wo][N] contiguous NHWC, `packed` = _pack(wt [T][K][N'],
    N').  s2d_pad: src is read through its space-to-depth view (K = 4C virtual channels); d2s_pad: out is written
    through its depth-to-space view (N' = 4N virtual channels); include/esr_amd.h esr_dconv_fwd_sd."""
    B, Hs, Ws, C = src.shape
    _, Ho, Wo, N = out.shape
    wp, nck, n_pad = packed
    kc = 4 * C if s2d_pad is not None else C
    n = 4 * N if d2s_pad is not None else N
    lib = _lib.load()
    mode = _mode(prec)
    sd = s2d_pad is not None or d2s_pad is not None
    # the pre-split weights feed only the x3 halo kernel: not built for launches the gather kernel takes
    wsx, wexp = packed.split() if (mode in (1, 2) and PRESPLIT and
                                   lib.esr_dconv_uses_halo(smy, smx, len(offy), MW, int(sd), mode) == 1) \
        else (None, None)
    oy, ox = _i32(offy), _i32(offx)
    # split-K where the grid would fill few CUs and K is long (the 8x8 pseudo-FC layer); the library says how many
    ks = lib.esr_dconv_fwd_splits_sd(B, MH, MW, n, kc, smy, smx, len(offy), oy, ox, int(sd), mode)
    if ks < 1:
        raise RuntimeError('esr_dconv_fwd_splits failed with esr_status %d' % ks)
    part = torch.empty(ks * B * MH * MW * n_pad, device=src.device) if ks > 1 else None
    _lib.check(lib.esr_dconv_fwd_sd(src.data_ptr(), B, Hs, Ws, C, kc, wp.data_ptr(), nck, n_pad,
                                    None if bias is None else bias.data_ptr(), out.data_ptr(), Ho, Wo, N, n, MH, MW,
                                    omy, oay, omx, oax, smy, smx, len(offy), oy, ox, ks,
                                    None if part is None else part.data_ptr(),
                                    C if s2d_pad is not None else 0, s2d_pad or 0,
                                    N if d2s_pad is not None else 0, d2s_pad or 0, mode,
                                    None if wsx is None else wsx.data_ptr(), None if wexp is None else wexp.data_ptr(),
                                    _stream(src)),
               'esr_dconv_fwd')


def _s2d_form(k, s, C):
    """Whether a k×k stride-s conv runs in its space-to-depth form ((k/2)² taps, 4C channels)."""
    return S2D and s == 2 and k % 2 == 0 and C % 4 == 0


def _s2d_weights(w):
    """w [Co][Ci][k][k] -> [(k/2)²][4Ci][Co]: tap (a, b) of the space-to-depth form holds w[:, :, 2a + py, 2b + px] at
    virtual channel (ci / G)·4G + (2py + px)·G + ci % G, G = 32 if 32 | Ci else Ci (include/esr_amd.h
    esr_dconv_fwd_sd: a 32-channel K chunk is then 32 channels of one real pixel)."""
    Co, Ci, k, _ = w.shape
    h = k // 2
    G = 32 if Ci % 32 == 0 else Ci
    wt = w.permute(2, 3, 1, 0).reshape(h, 2, h, 2, Ci // G, G, Co)  # [a][py][b][px][cb][cg][co]
    return wt.permute(0, 2, 4, 1, 3, 5, 6).reshape(h * h, 4 * Ci, Co)


def conv_forward(x, w, b, k, s, p, prec=None):
    """y = conv2d(x, w, b, stride s, zero padding p) on NHWC x [B][H][W][Ci]; w [Co][Ci][k][k]."""
    _check_dev(x, w, b)
    B, H, W, Ci = x.shape
    Co = w.shape[0]
    Ho, Wo = out_size(H, k, s, p), out_size(W, k, s, p)
    y = torch.empty(B, Ho, Wo, Co, device=x.device, dtype=torch.float32)
    # y[yo] = sum over taps (a, b) of W'[a, b] . Z[yo + a, xo + b], Z = s2d(pad(x, p)); only where it is halo-tiled
    if _s2d_form(k, s, Ci) and _lib.load().esr_dconv_uses_halo(1, 1, (k // 2) ** 2, Wo, 1, _mode(prec)) == 1:
        wp = _packed(w, ('fwd_s2d',), lambda: _pack(_s2d_weights(w.detach()), Co))
        h = k // 2
        _gather(x, wp, None if b is None else b.detach().contiguous(), y, Ho, Wo, 1, 0, 1, 0, 1, 1,
                [a for a in range(h) for _ in range(h)], [c for _ in range(h) for c in range(h)], s2d_pad=p, prec=prec)
        return y
    wp = _packed(w, ('fwd',), lambda: _pack(w.detach().permute(2, 3, 1, 0).reshape(k * k, Ci, Co), Co))
    taps = [(ky, kx) for ky in range(k) for kx in range(k)]
    _gather(x, wp, None if b is None else b.detach().contiguous(), y, Ho, Wo, 1, 0, 1, 0, s, s,
            [ky - p for ky, _ in taps], [kx - p for _, kx in taps], prec=prec)
    return y


def conv_dgrad(gy, w, k, s, p, H, W, prec=None):
    """gx = conv_transpose of gy (NHWC [B][Ho][Wo][Co]) back to the [B][H][W][Ci] input grid: one launch per phase
    class (cy, cx) of the stride, each gathering over the taps that land on that class."""
    _check_dev(gy, w)
    B, Ho, Wo, Co = gy.shape
    Ci = w.shape[1]
    wd = w.detach()
    if _s2d_form(k, s, Ci):  # dZ[Y, X] = sum over taps (a, b) of W'[a, b]^T . gy[Y - a, X - b]; gx = d2s(dZ) unpadded
        h = k // 2
        gx = torch.empty(B, H, W, Ci, device=gy.device, dtype=torch.float32)
        wp = _packed(w, ('dgrad_s2d',), lambda: _pack(_s2d_weights(wd).transpose(1, 2).contiguous(), 4 * Ci))
        _gather(gy, wp, None, gx, (H - 1 + p) // 2 + 1, (W - 1 + p) // 2 + 1, 1, 0, 1, 0, 1, 1,
                [-a for a in range(h) for _ in range(h)], [-c for _ in range(h) for c in range(h)], d2s_pad=p,
                prec=prec)
        return gx
    classes = []
    full = True
    for cy in range(s):
        for cx in range(s):
            MH, MW = (H - cy + s - 1) // s, (W - cx + s - 1) // s
            tys = [ky for ky in range(k) if (cy + p - ky) % s == 0]
            txs = [kx for kx in range(k) if (cx + p - kx) % s == 0]
            if MH <= 0 or MW <= 0:
                continue
            if not tys or not txs:
                full = False
                continue
            classes.append((cy, cx, MH, MW, [(ky, kx) for ky in tys for kx in txs]))
    gx = (torch.empty if full else torch.zeros)(B, H, W, Ci, device=gy.device, dtype=torch.float32)
    for cy, cx, MH, MW, taps in classes:
        wp = _packed(w, ('dgrad', s, p, cy, cx),
                     lambda taps=taps: _pack(torch.stack([wd[:, :, ky, kx] for ky, kx in taps]), Ci))  # [T][Co][Ci]
        _gather(gy, wp, None, gx, MH, MW, s, cy, s, cx, 1, 1,
                [(cy + p - ky) // s for ky, _ in taps], [(cx + p - kx) // s for _, kx in taps], prec=prec)
    return gx


def conv_wgrad(x, gy, k, s, p, prec=None):
    """gw [Co][Ci][k][k] = sum over pixels of x (gathered per tap) * gy; split-K over pixels + deterministic reduce."""
    _check_dev(x, gy)
    B, H, W, Ci = x.shape
    _, Ho, Wo, Co = gy.shape
    T = k * k
    cin_pad, cout_pad = 64 * ((Ci + 63) // 64), 64 * ((Co + 63) // 64)
    n = T * cin_pad * cout_pad
    taps = [(ky, kx) for ky in range(k) for kx in range(k)]
    oy, ox = _i32([ky - p for ky, _ in taps]), _i32([kx - p for _, kx in taps])
    lib = _lib.load()
    mode = _mode(prec)
    st = _stream(x)
    splits = lib.esr_dconv_wgrad_splits(B, Ho, Wo, Ci, Co, s, s, T, oy, ox, mode)  # split-K over pixels
    if splits < 1:
        raise RuntimeError('esr_dconv_wgrad_splits failed with esr_status %d' % splits)
    partial = torch.empty(splits * n, device=x.device, dtype=torch.float32)
    red = torch.empty(n, device=x.device, dtype=torch.float32)
    _lib.check(lib.esr_dconv_wgrad(x.data_ptr(), B, H, W, Ci, Ci, gy.data_ptr(), Ho, Wo, Co, Co, s, s, T, oy, ox,
                                   splits, partial.data_ptr(), mode, st), 'esr_dconv_wgrad')
    _lib.check(lib.esr_wgrad_reduce(partial.data_ptr(), splits, n, 1.0, red.data_ptr(), st), 'esr_wgrad_reduce')
    return red.view(k, k, cin_pad, cout_pad)[:, :, :Ci, :Co].permute(3, 2, 0, 1).contiguous()


def colsum(t):
    """Σ over every dimension but the last of a contiguous float tensor (esr_colsum: float64 partial sums in fixed
    order, one pass; PyTorch's sum over (0, 1, 2) of an NHWC tensor ran at ~0.2 TB/s)."""
    _check_dev(t)
    t = t.contiguous()
    C = t.shape[-1]
    P = t.numel() // C
    lib = _lib.load()
    out = torch.empty(C, device=t.device, dtype=torch.float32)
    ws = torch.empty(int(lib.esr_bn_workspace_floats(P, C)), device=t.device, dtype=torch.float32)
    _lib.check(lib.esr_colsum(t.data_ptr(), P, C, out.data_ptr(), ws.data_ptr(), _stream(t)), 'esr_colsum')
    return out


# The precision of a conv is fixed when its forward runs (the module default, or the layer's own
# HipConv2d.esr_precision) and travels to every launch of its backward and double backward.
class DConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, k, s, p, prec=None):
        prec = prec or PRECISION
        ctx.save_for_backward(x, w)
        ctx.geom = (k, s, p, prec)
        ctx.has_bias = b is not None
        return conv_forward(x, w, b, k, s, p, prec)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        k, s, p, prec = ctx.geom
        gy = gy.contiguous()
        gx = DgradFn.apply(gy, w, k, s, p, x.shape[1], x.shape[2], prec) if ctx.needs_input_grad[0] else None
        gw = WgradFn.apply(x, gy, k, s, p, prec) if ctx.needs_input_grad[1] else None
        gb = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            if torch.is_grad_enabled() or not COLSUM:  # create_graph: a differentiable sum
                gb = gy.sum((0, 1, 2), dtype=torch.float64).float() if BIAS_F64 else gy.sum((0, 1, 2))
            else:
                gb = colsum(gy)
        return gx, gw, gb, None, None, None, None


class DgradFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gy, w, k, s, p, H, W, prec=None):
        ctx.save_for_backward(gy, w)
        ctx.geom = (k, s, p, prec)
        return conv_dgrad(gy, w, k, s, p, H, W, prec)

    @staticmethod
    def backward(ctx, ggx):
        gy, w = ctx.saved_tensors
        k, s, p, prec = ctx.geom
        ggx = ggx.contiguous()
        g_gy = DConvFn.apply(ggx, w, None, k, s, p, prec) if ctx.needs_input_grad[0] else None
        g_w = WgradFn.apply(ggx, gy, k, s, p, prec) if ctx.needs_input_grad[1] else None
        return g_gy, g_w, None, None, None, None, None, None


class WgradFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gy, k, s, p, prec=None):
        ctx.save_for_backward(x, gy)
        ctx.geom = (k, s, p, prec)
        return conv_wgrad(x, gy, k, s, p, prec)

    @staticmethod
    def backward(ctx, ggw):
        x, gy = ctx.saved_tensors
        k, s, p, prec = ctx.geom
        ggw = ggw.contiguous()
        g_x = DgradFn.apply(gy, ggw, k, s, p, x.shape[1], x.shape[2], prec) if ctx.needs_input_grad[0] else None
        g_gy = DConvFn.apply(x, ggw, None, k, s, p, prec) if ctx.needs_input_grad[1] else None
        return g_x, g_gy, None, None, None, None


class _ToNHWC(torch.autograd.Function):
    """NCHW-contiguous -> NHWC copy whose gradient comes back NCHW-contiguous (the discriminator's input gradient is
    used with .view() by GradientPenaltyLoss, loss.py:255-263, as in the reference)."""

    @staticmethod
    def forward(ctx, x):
        return x.permute(0, 2, 3, 1).contiguous()

    @staticmethod
    def backward(ctx, g):
        return g.permute(0, 3, 1, 2).contiguous()


def _im2col(xh, k, p):
    """[B][H][W][C] -> [B][Ho][Wo][32] (stride 1): channel (ky*k + kx)*C + c = x[y + ky - p][x + kx - p][c] (zero
    outside), zero-filled to 32 channels (esr_dconv_im2col: one pass; the pad + cat of slices took two)."""
    _check_dev(xh)
    xh = xh.contiguous()
    B, H, W, C = xh.shape
    out = torch.empty(B, out_size(H, k, 1, p), out_size(W, k, 1, p), 32, device=xh.device, dtype=torch.float32)
    _lib.check(_lib.load().esr_dconv_im2col(xh.data_ptr(), B, H, W, C, k, p, out.data_ptr(), _stream(xh)),
               'esr_dconv_im2col')
    return out


def _col2im(gc, k, p, H, W, C):
    """The adjoint of _im2col: every tap's channel group added back at its shift, in tap order from zero
    (esr_dconv_col2im: one pass; the zeros + k² shifted in-place adds + copy took 11 launches over the image)."""
    _check_dev(gc)
    gc = gc.contiguous()
    B = gc.shape[0]
    gx = torch.empty(B, H, W, C, device=gc.device, dtype=torch.float32)
    _lib.check(_lib.load().esr_dconv_col2im(gc.data_ptr(), B, H, W, C, k, p, gx.data_ptr(), _stream(gc)),
               'esr_dconv_col2im')
    return gx


class _Im2ColFn(torch.autograd.Function):
    """_im2col with _col2im as its gradient (and _im2col as the gradient of that: the WGAN-GP double backward)."""

    @staticmethod
    def forward(ctx, xh, k, p):
        ctx.geom = (k, p) + tuple(xh.shape[1:])
        return _im2col(xh, k, p)

    @staticmethod
    def backward(ctx, g):
        return _Col2ImFn.apply(g.contiguous(), *ctx.geom), None, None


class _Col2ImFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gc, k, p, H, W, C):
        ctx.geom = (k, p)
        return _col2im(gc, k, p, H, W, C)

    @staticmethod
    def backward(ctx, gg):
        return _Im2ColFn.apply(gg.contiguous(), *ctx.geom), None, None, None, None, None


# ---- the first conv block fused (csrc/esr_dfirst.hip): Conv2d(3, 64, 3, stride 1, padding 1) + LeakyReLU, exact fp32 --
# (architecture.py:231, block.py:129-156); '0' = HipConv2d (im2col + 1x1 conv at PRECISION) + a separate LeakyReLU
FUSED_FIRST = os.environ.get('ESR_DFIRST', '1') != '0'
_DF_LRELU, _DF_MASK, _DF_ACC = 1, 2, 4
_DF_NW = 64 * 27 + 64  # weight-gradient partial: 64·27 weights (torch order), then 64 biases


def _ptr(t):
    return t.data_ptr() if t is not None else None


def _df_fwd(xh, w, b, slope, flags, mask=None, out=None):
    """esr_dfirst_fwd: [B][H][W][3] -> [B][H][W][64] (flags: LeakyReLU / mask by lrelu'(mask) / accumulate into out)."""
    B, H, W, _ = xh.shape
    y = out if out is not None else torch.empty(B, H, W, 64, device=xh.device, dtype=torch.float32)
    _lib.check(_lib.load().esr_dfirst_fwd(xh.data_ptr(), B, H, W, w.contiguous().data_ptr(), _ptr(b), slope, flags,
                                          _ptr(mask), y.data_ptr(), _stream(xh)), 'esr_dfirst_fwd')
    return y


def _df_bwd(xh, gy, mask, slope, w, need_x, need_w):
    """esr_dfirst_bwd + the ordered block reduction: (input gradient or None, [weight grads | bias grads] or None)
    for g' = gy·lrelu'(mask)."""
    lib = _lib.load()
    B, H, W, _ = gy.shape
    gx = torch.empty(B, H, W, 3, device=gy.device, dtype=torch.float32) if need_x else None
    part = None
    if need_w:
        nb = lib.esr_dfirst_bwd_blocks(B, H, W)
        part = torch.empty(nb * _DF_NW, device=gy.device, dtype=torch.float32)
    st = _stream(gy)
    _lib.check(lib.esr_dfirst_bwd(_ptr(xh), gy.data_ptr(), _ptr(mask), slope, B, H, W, w.contiguous().data_ptr(),
                                  _ptr(gx), _ptr(part), st), 'esr_dfirst_bwd')
    gwb = None
    if need_w:
        gwb = torch.empty(_DF_NW, device=gy.device, dtype=torch.float32)
        _lib.check(lib.esr_wgrad_reduce(part.data_ptr(), nb, _DF_NW, 1.0, gwb.data_ptr(), st), 'esr_wgrad_reduce')
    return gx, gwb


class _DFirstFn(torch.autograd.Function):
    """y = LeakyReLU(conv3x3(x, w) + b) on NHWC tensors (3 -> 64 channels); backward: _DFirstBwdFn."""

    @staticmethod
    def forward(ctx, xh, w, b, slope):
        y = _df_fwd(xh, w, b, slope, _DF_LRELU)
        ctx.save_for_backward(xh, w, y)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, gy):
        xh, w, y = ctx.saved_tensors
        nx, nw, nb = ctx.needs_input_grad[:3]
        gx, gw, gb = _DFirstBwdFn.apply(xh, gy.contiguous(), y, w, ctx.slope, nx, nw or nb)
        return gx if nx else None, gw if nw else None, gb if nb else None, None


class _DFirstBwdFn(torch.autograd.Function):
    """(x, gy, y, w) -> (gx, gw, gb) of _DFirstFn with g' = gy·lrelu'(y) (one esr_dfirst_bwd pass).  Its backward (the
    WGAN-GP double backward, loss.py:244-263): with ggx, ggw, ggb the gradients of the three outputs,
        d/dgy = lrelu'(y) · (conv(ggx; w) + conv(x; ggw) + ggb)      (esr_dfirst_fwd, masked)
        d/dw  = wgrad(ggx, g')     d/dx = dgrad(g'; ggw)             (esr_dfirst_bwd)
    and nothing through y (the mask is piecewise constant)."""

    @staticmethod
    def forward(ctx, xh, gy, y, w, slope, need_x, need_w):
        gx, gwb = _df_bwd(xh, gy, y, slope, w, need_x, need_w)
        ctx.save_for_backward(xh, gy, y, w)
        ctx.slope, ctx.need = slope, (need_x, need_w)
        ctx.set_materialize_grads(False)
        e = gy.new_zeros(0)
        if gwb is None:
            return (gx if need_x else e), e, e
        return (gx if need_x else e), gwb[:64 * 27].view(64, 3, 3, 3).clone(), gwb[64 * 27:].clone()

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, ggx, ggw, ggb):
        xh, gy, y, w = ctx.saved_tensors
        need_x, need_w = ctx.need
        ggx = ggx if need_x and ggx is not None else None
        ggw = ggw if need_w and ggw is not None else None
        ggb = ggb if need_w and ggb is not None else None
        slope = ctx.slope
        g_x = g_gy = g_w = None
        if ctx.needs_input_grad[1] and (ggx is not None or ggw is not None or ggb is not None):
            terms = []
            if ggx is not None:
                terms.append((ggx.contiguous(), w))
            if ggw is not None:
                terms.append((xh, ggw.contiguous()))
            if not terms:  # the bias term alone: a conv with zero weights plus ggb
                terms.append((xh, torch.zeros_like(w)))
            g_gy = torch.empty_like(gy)
            for i, (src, wt) in enumerate(terms):
                last = i == len(terms) - 1
                _df_fwd(src, wt, ggb.contiguous() if (i == 0 and ggb is not None) else None, slope,
                        (_DF_ACC if i else 0) | (_DF_MASK if last else 0), mask=y, out=g_gy)
        if ctx.needs_input_grad[3] and ggx is not None:
            g_w = _df_bwd(ggx.contiguous(), gy, y, slope, w, False, True)[1][:64 * 27].view(64, 3, 3, 3)
        if ctx.needs_input_grad[0] and ggw is not None:
            g_x = _df_bwd(None, gy, y, slope, ggw.contiguous(), True, False)[0]
        return g_x, g_gy, None, g_w, None, None, None


def dfirst_ok(conv):
    """Whether a HipConv2d is the first conv block's shape the fused kernels take."""
    return FUSED_FIRST and conv.in_channels == 3 and conv.out_channels == 64 and conv.kernel_size == (3, 3) and \
        conv.stride == (1, 1) and conv.padding == (1, 1) and conv.bias is not None


def dfirst_lrelu(x, conv, slope):
    """LeakyReLU(slope)(conv(x)) for a HipConv2d passing dfirst_ok, on the fused kernels: NCHW in (any memory format),
    NCHW with channels-last storage out, differentiable twice (the WGAN-GP penalty)."""
    _check_dev(x)
    if x.is_contiguous(memory_format=torch.channels_last):
        xh = x.permute(0, 2, 3, 1)
    else:
        xh = _ToNHWC.apply(x)
    return _DFirstFn.apply(xh, conv.weight, conv.bias, float(slope)).permute(0, 3, 1, 2)


class HipConv2d(nn.Conv2d):
    """nn.Conv2d of the discriminator (same parameters, state_dict and init) whose forward runs esr_dconv.

    Square kernel, equal stride and zero padding in both dimensions, no dilation / groups (what conv_block builds).
    Input: NCHW tensor (any memory format; channels-last avoids a copy); output: NCHW with channels-last storage."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        k, s, p = self.kernel_size, self.stride, self.padding
        if k[0] != k[1] or s[0] != s[1] or p[0] != p[1] or self.dilation != (1, 1) or self.groups != 1 or \
                self.padding_mode != 'zeros' or k[0] * k[1] > MAX_TAPS:
            raise NotImplementedError('HipConv2d: square zero-padded dense convolutions with <= %d taps' % MAX_TAPS)
        # few input channels (conv0: 3 channels x 9 taps = 27): gather the taps into channels once and run a 1x1 conv,
        # one 32-wide K step instead of one (mostly zero) K step per tap
        self._im2col = s[0] == 1 and self.in_channels * k[0] * k[1] <= 32 and self.in_channels < 8
        self.esr_precision = None  # this layer's precision ('x3' / 'x6' / 'f32'); None = the module default

    def forward(self, x):
        _check_dev(x)
        if x.is_contiguous(memory_format=torch.channels_last):
            xh = x.permute(0, 2, 3, 1)  # a view: NHWC storage already
        else:
            xh = _ToNHWC.apply(x)
        k, p = self.kernel_size[0], self.padding[0]
        self.weight._esr_dconv_param = True  # packed-weight memo (_packed); set per call: .to()/_apply may replace it
        if self._im2col:
            C = xh.shape[3]
            cols = _Im2ColFn.apply(xh, k, p)  # channel (ky*k + kx)*C + c
            w1 = F.pad(self.weight.permute(0, 2, 3, 1).reshape(self.out_channels, k * k * C), (0, 32 - k * k * C))
            y = DConvFn.apply(cols, w1.view(self.out_channels, 32, 1, 1), self.bias, 1, 1, 0, self.esr_precision)
        else:
            y = DConvFn.apply(xh, self.weight, self.bias, k, self.stride[0], p, self.esr_precision)
        return y.permute(0, 3, 1, 2)
