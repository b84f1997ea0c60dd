"""Training (autograd) path of the HIP generator: forward with retained activations + hand-written backward.

`generator_forward` in engine.py routes here whenever autograd needs parameter gradients (the reference's training
step: `fake_H = netG(model_input)` then `l_g_total.backward()`, SRRaGAN_model.py:348, 529).  The whole generator +
CEM is one torch.autograd.Function whose backward runs libesr_amd kernels (exact fp32):

  CEM (train mode)      d gen = g - Down^T Inv^T Up^T g        esr_cem_adjoint ×3 (exact replicate-pad adjoints)
  conv data gradient    esr_conv3x3_fwd with rot180, in/out-swapped packed weights, in 64-channel output slices,
                        accumulating into a concat-gradient buffer (the adjoint of the dense concatenations)
  conv weight gradient  esr_conv3x3_wgrad (split-K over pixel tiles) + esr_wgrad_reduce (deterministic)
  LeakyReLU / residuals esr_lrelu_bwd, esr_axpby;  nearest ×2 adjoint: esr_sum2x2
The reference's residual scales (0.2 in RDB and RRDB, block.py:235, 270) are folded into the packed backward weights
and the reduction scales.
"""
import ctypes

import torch

from . import _lib
from . import engine as E

WG_SPLITS_MAX = 128


def _z(dev, *s):
    return torch.zeros(*s, device=dev, dtype=torch.float32)


class TrainWorkspace:
    """Buffers of one training forward/backward at (B, H, W).  Same attribute names as engine._Workspace for the
    shared forward code, plus one concat buffer per RDB (`Q`) and the gradient buffers."""

    def __init__(self, dev, B, H, W, latent, nb):
        zc = 8 if latent else 0
        self.B, self.H, self.W, self.zc, self.nb = B, H, W, zc, nb
        self.first_cp = 16 if latent else 8
        self.first_lr_off = 8 if latent else 0
        self.cp = zc + 192
        self.hr_cp = zc + 64
        self.first = _z(dev, B, H + 2, W + 2, self.first_cp)
        self.fea = _z(dev, B, H + 2, W + 2, 64)
        self.Q = [_z(dev, B, H + 2, W + 2, self.cp) for _ in range(3 * nb + 1)]
        self.U0 = _z(dev, B, H + 2, W + 2, 64)
        self.U1 = _z(dev, B, 2 * H + 2, 2 * W + 2, 64)
        self.HR = [_z(dev, B, 4 * H + 2, 4 * W + 2, self.hr_cp) for _ in range(2)]
        self.lr = _z(dev, B, 3, H, W)
        self.overflow = torch.zeros(1, device=dev, dtype=torch.int32)
        # backward
        self.D = [_z(dev, B, H + 2, W + 2, self.cp) for _ in range(2)]
        self.GA = _z(dev, B, H + 2, W + 2, 64)
        self.G3 = _z(dev, B, H + 2, W + 2, 64)
        self.dU0 = _z(dev, B, H + 2, W + 2, 64)
        self.dU1 = _z(dev, B, 2 * H + 2, 2 * W + 2, 64)
        self.dUp1 = _z(dev, B, 2 * H + 2, 2 * W + 2, 64)
        self.dHR = [_z(dev, B, 4 * H + 2, 4 * W + 2, 64) for _ in range(2)]
        self.dgen_p = _z(dev, B, 4 * H + 2, 4 * W + 2, 8)
        self.wg_n_max = 9 * 224 * 64 + 64
        self.partial = torch.empty(WG_SPLITS_MAX * self.wg_n_max, device=dev, dtype=torch.float32)
        self.dw = torch.empty(self.wg_n_max, device=dev, dtype=torch.float32)


def _train_workspace(net, dev, B, H, W, latent):
    key = (str(dev), B, H, W, latent, net.nb)
    c = net._esr_cache.get('train_ws')
    if c is None or c[0] != key:
        net._esr_cache.pop('train_ws', None)
        c = (key, TrainWorkspace(dev, B, H, W, latent, net.nb))
        net._esr_cache['train_ws'] = c
    return c[1]


# ----------------------------------------------------------------------------------------------------------------------
# backward weight packing
# ----------------------------------------------------------------------------------------------------------------------
class _BwdConv:
    """Backward data of one conv: the forward-buffer channel map, dgrad weight slices and the wgrad index map."""

    def __init__(self, conv, cmap, scale=1.0, cin_k=None, dgrad_from=0):
        w = conv.weight.detach()
        cout, cin_ref = w.shape[:2]
        self.conv, self.cout, self.cmap, self.cin_buf = conv, cout, list(cmap), len(cmap)
        wf = w.flip(2, 3).transpose(0, 1)  # [Cin_ref][Cout][3][3]: rot180, swapped
        k = cin_k if cin_k is not None else cout  # channels of the gradient the dgrad reads (padded to 8)
        kmap = list(range(cout)) + [-1] * (k - cout)
        self.slices = []  # (first buffer channel, width, packed weights)
        n0 = dgrad_from  # input-gradient channels below this (the latent Z slot) are not needed
        while n0 < self.cin_buf:
            nw = min(64, self.cin_buf - n0)
            wt = torch.zeros(nw, cout, 3, 3, device=w.device, dtype=w.dtype)
            for o in range(nw):
                r = self.cmap[n0 + o]
                if r >= 0:
                    wt[o] = wf[r]
            self.slices.append((n0, nw, E.pack_conv_weight(wt * scale, kmap, 32 if nw <= 32 else 64)))
            n0 += nw
        dev = w.device
        self.ref_to_buf = torch.tensor([self.cmap.index(r) for r in range(cin_ref)], device=dev, dtype=torch.long)
        self.zero_bias = torch.zeros(64, device=dev)


class _BwdPacked:
    def __init__(self, net, latent):
        def lr_map(n):
            return list(range(n)) if not latent else [0, 1, 2] + [-1] * 5 + [3 + c for c in range(n)]
        m = net.model
        zc = 8 if latent else 0
        first_map = ([0, 1, 2] + [-1] * 5 + [3, 4, 5] + [-1] * 5) if latent else ([0, 1, 2] + [-1] * 5)
        self.first = _BwdConv(m[0], first_map, dgrad_from=len(first_map))  # no input gradient needed
        self.rdb = []
        for k in range(net.nb):
            rr = m[1].sub[k]
            for rdb in (rr.RDB1, rr.RDB2, rr.RDB3):
                self.rdb.append([_BwdConv(rdb.convs[i][0], lr_map(64 + 32 * i), 0.2 if i == 4 else 1.0,
                                          dgrad_from=zc) for i in range(5)])
        self.lr_conv = _BwdConv(m[1].sub[net.nb], lr_map(64), dgrad_from=zc)
        self.up = [_BwdConv(m[j][1], list(range(64))) for j in (2, 3)]
        self.hr0 = _BwdConv(m[4], lr_map(64), dgrad_from=zc)
        self.hr1 = _BwdConv(m[6], lr_map(64), cin_k=8, dgrad_from=zc)


def _bwd_packed(net, latent):
    key = (E._param_key(net), latent)
    c = net._esr_cache.get('packed_bwd')
    if c is None or c[0] != key:
        with torch.no_grad():
            c = (key, _BwdPacked(net, latent))
        net._esr_cache['packed_bwd'] = c
    return c[1]


# ----------------------------------------------------------------------------------------------------------------------
# backward sweep
# ----------------------------------------------------------------------------------------------------------------------
class _Runner:
    def __init__(self, ws, stream):
        self.lib = _lib.load()
        self.ws = ws
        self.B = ws.B
        self.stream = stream
        self.grads = {}

    def dgrad(self, bc, src, src_cp, src_coff, cin_k, h, w, dst, dst_cp, dst_base, accumulate, res=None):
        """dst[:, n0-dst_base ...] (+)= conv(src slice, rot180 W^T) for every output slice; `res` = (buf, cp, coff)
        is added to the first slice (a residual that bypasses the conv)."""
        for si, (n0, nw, wpk) in enumerate(bc.slices):
            coff = n0 - dst_base
            r1, r1_cp, r1_coff = (dst, dst_cp, coff) if accumulate else (None, 0, 0)
            if si == 0 and res is not None:
                assert not accumulate
                r1, r1_cp, r1_coff = res
            o = E._conv_out(dst, dst_cp, coff, h, w, False, r1=r1, r1_cp=r1_cp, r1_coff=r1_coff, s1=1.0)
            inp = src.data_ptr() + 4 * src_coff
            _lib.check(self.lib.esr_conv3x3_fwd(inp, self.B, h, w, src_cp, cin_k, wpk.data_ptr(),
                                                bc.zero_bias.data_ptr(), nw, ctypes.byref(o), self.stream), 'dgrad')

    def wgrad(self, bc, inp, in_cp, cin, up2, dout, d_cp, d_coff, h, w, scale=1.0):
        ws = self.ws
        cin_pad = (cin + 31) // 32 * 32
        cout_pad = 32 if bc.cout <= 32 else 64
        n = 9 * cin_pad * cout_pad + cout_pad
        chunks = cin_pad // 32
        ntiles = self.B * ((h + 7) // 8) * ((w + 31) // 32)
        splits = max(1, min(WG_SPLITS_MAX, -(-1024 // chunks), ntiles))
        _lib.check(self.lib.esr_conv3x3_wgrad(inp.data_ptr(), in_cp, cin, up2, dout.data_ptr(), d_cp, d_coff,
                                              bc.cout, self.B, h, w, splits, ws.partial.data_ptr(), self.stream),
                   'wgrad')
        _lib.check(self.lib.esr_wgrad_reduce(ws.partial.data_ptr(), splits, n, scale, ws.dw.data_ptr(),
                                             self.stream), 'wgrad_reduce')
        dw = ws.dw[:9 * cin_pad * cout_pad].view(9, cin_pad, cout_pad)
        g = dw[:, bc.ref_to_buf, :bc.cout].permute(2, 1, 0).reshape(bc.conv.weight.shape)
        self._acc(bc.conv.weight, g)
        self._acc(bc.conv.bias, ws.dw[9 * cin_pad * cout_pad:9 * cin_pad * cout_pad + bc.cout])

    def _acc(self, p, g):
        prev = self.grads.get(p)
        self.grads[p] = g.clone() if prev is None else prev + g

    def lrelu(self, d, d_cp, d_coff, y, y_cp, y_coff, C, h, w):
        _lib.check(self.lib.esr_lrelu_bwd(d.data_ptr(), d_cp, d_coff, y.data_ptr(), y_cp, y_coff, C, self.B, h, w,
                                          self.stream), 'lrelu_bwd')

    def axpby(self, out, o_cp, o_coff, a, x1, x1_cp, x1_coff, b=0.0, x2=None, x2_cp=0, x2_coff=0, C=64, h=0, w=0):
        _lib.check(self.lib.esr_axpby(out.data_ptr(), o_cp, o_coff, a, x1.data_ptr(), x1_cp, x1_coff, b,
                                      None if x2 is None else x2.data_ptr(), x2_cp, x2_coff, C, self.B, h, w,
                                      self.stream), 'axpby')


def _rdb_backward(R, P, dout, dcat, convs, zc, cp, H, W):
    """One ResidualDenseBlock_5C (block.py:230-235): h = 0.2·conv4(cat) + x, cat = [x, x1..x4], x_{i+1} =
    lrelu(conv_i(cat_{<=i})).  dout = (buffer, pitch, offset) of dL/dh.  On return dcat[zc:zc+64) = dL/dx."""
    dbuf, dcp, dcoff = dout
    # conv4 (0.2 folded into its packed dgrad weights and its wgrad scale); the x slice also receives dL/dh
    R.wgrad(convs[4], P, cp, zc + 192, 0, dbuf, dcp, dcoff, H, W, scale=0.2)
    R.dgrad(convs[4], dbuf, dcp, dcoff, 64, H, W, dcat, cp, 0, accumulate=False, res=(dbuf, dcp, dcoff))
    for i in (3, 2, 1, 0):
        s = zc + 64 + 32 * i
        R.lrelu(dcat, cp, s, P, cp, s, 32, H, W)
        R.wgrad(convs[i], P, cp, s, 0, dcat, cp, s, H, W)
        R.dgrad(convs[i], dcat, cp, s, 32, H, W, dcat, cp, 0, accumulate=True)


def generator_backward(net, cem, ws, d_out, latent, M):
    """dL/dparams of RRDBNet (+ CEM in train or eval mode) given dL/dout; returns {param: grad}."""
    dev = d_out.device
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    R = _Runner(ws, stream)
    lib = R.lib
    bp = _bwd_packed(net, latent)
    Bn, H, W, zc, cp, hcp = ws.B, ws.H, ws.W, ws.zc, ws.cp, ws.hr_cp
    HH, WW = E.SF * H, E.SF * W
    # ---- CEM adjoint: out = crop_M(gen + Up(Inv(LR - Down(gen)))) ----
    if cem is not None:
        g = d_out.contiguous()
        if M > 0:
            gfull = torch.zeros(Bn, 3, HH, WW, device=dev)
            gfull[:, :, M:HH - M, M:WW - M] = g
        else:
            gfull = g
        wd = cem.DownscaleOP.Filter_OP.weight[0, 0].contiguous()
        wi = cem.Conv_LR_with_Inv_hTh_OP.Filter_OP.weight[0, 0].contiguous()
        wu = cem.Upscale_OP.Filter_OP.weight[0, 0].contiguous()
        kd, ki = wd.shape[-1], wi.shape[-1]
        a1 = torch.empty(Bn, 3, H, W, device=dev)
        a2 = torch.empty_like(a1)
        _lib.check(lib.esr_cem_adjoint(gfull.data_ptr(), Bn * 3, HH, WW, wu.data_ptr(), kd, 1, 0, HH, WW, E.SF,
                                       E.CEM_PHASE, 1.0, 0, a1.data_ptr(), stream), 'cem_adjoint up')
        _lib.check(lib.esr_cem_adjoint(a1.data_ptr(), Bn * 3, H, W, wi.data_ptr(), ki, 1, 0, H, W, 1, 0, 1.0, 0,
                                       a2.data_ptr(), stream), 'cem_adjoint inv')
        dgen = gfull.clone()
        _lib.check(lib.esr_cem_adjoint(a2.data_ptr(), Bn * 3, H, W, wd.data_ptr(), kd, E.SF, E.CEM_PHASE, HH, WW, 1,
                                       0, -1.0, 1, dgen.data_ptr(), stream), 'cem_adjoint down')
    else:
        dgen = d_out.contiguous()
    _lib.check(lib.esr_nchw_to_padded(dgen.data_ptr(), 3, Bn, HH, WW, ws.dgen_p.data_ptr(), 8, 0, 0, stream),
               'nchw_to_padded')
    HR0, HR1 = ws.HR
    dA, dB = ws.dHR
    # HR_conv1 (no act): input HR1 = [Z_HR | x]
    R.wgrad(bp.hr1, HR1, hcp, hcp, 0, ws.dgen_p, 8, 0, HH, WW)
    R.dgrad(bp.hr1, ws.dgen_p, 8, 0, 8, HH, WW, dA, 64, zc, accumulate=False)
    # HR_conv0 + LReLU: output HR1.x
    R.lrelu(dA, 64, 0, HR1, hcp, zc, 64, HH, WW)
    R.wgrad(bp.hr0, HR0, hcp, hcp, 0, dA, 64, 0, HH, WW)
    R.dgrad(bp.hr0, dA, 64, 0, 64, HH, WW, dB, 64, zc, accumulate=False)
    # upconv 2: HR0.x = lrelu(conv(nearest2(U1)))
    R.lrelu(dB, 64, 0, HR0, hcp, zc, 64, HH, WW)
    R.wgrad(bp.up[1], ws.U1, 64, 64, 1, dB, 64, 0, HH, WW)
    R.dgrad(bp.up[1], dB, 64, 0, 64, HH, WW, dA, 64, 0, accumulate=False)
    _lib.check(lib.esr_sum2x2(ws.dU1.data_ptr(), 64, 0, dA.data_ptr(), 64, 0, 64, Bn, 2 * H, 2 * W, stream), 'sum2x2')
    # upconv 1: U1 = lrelu(conv(nearest2(U0)))
    R.lrelu(ws.dU1, 64, 0, ws.U1, 64, 0, 64, 2 * H, 2 * W)
    R.wgrad(bp.up[0], ws.U0, 64, 64, 1, ws.dU1, 64, 0, 2 * H, 2 * W)
    R.dgrad(bp.up[0], ws.dU1, 64, 0, 64, 2 * H, 2 * W, ws.dUp1, 64, 0, accumulate=False)
    _lib.check(lib.esr_sum2x2(ws.dU0.data_ptr(), 64, 0, ws.dUp1.data_ptr(), 64, 0, 64, Bn, H, W, stream), 'sum2x2')
    # LR_conv: U0 = conv(trunk[Z | x]) + fea
    Q = ws.Q
    trunk = Q[3 * net.nb]
    R.wgrad(bp.lr_conv, trunk, cp, zc + 64, 0, ws.dU0, 64, 0, H, W)
    R.dgrad(bp.lr_conv, ws.dU0, 64, 0, 64, H, W, ws.GA, 64, zc, accumulate=False)
    # RRDBs, last to first: o = 0.2·RDB3(RDB2(RDB1(x))) + x
    D0, D1 = ws.D
    for k in reversed(range(net.nb)):
        R.axpby(ws.G3, 64, 0, 0.2, ws.GA, 64, 0, C=64, h=H, w=W)
        _rdb_backward(R, Q[3 * k + 2], (ws.G3, 64, 0), D0, bp.rdb[3 * k + 2], zc, cp, H, W)
        _rdb_backward(R, Q[3 * k + 1], (D0, cp, zc), D1, bp.rdb[3 * k + 1], zc, cp, H, W)
        _rdb_backward(R, Q[3 * k], (D1, cp, zc), D0, bp.rdb[3 * k], zc, cp, H, W)
        R.axpby(ws.GA, 64, 0, 1.0, ws.GA, 64, 0, 1.0, D0, cp, zc, C=64, h=H, w=W)
    # conv_first: dL/dfea = trunk gradient + LR_conv skip
    R.axpby(ws.GA, 64, 0, 1.0, ws.GA, 64, 0, 1.0, ws.dU0, 64, 0, C=64, h=H, w=W)
    R.wgrad(bp.first, ws.first, ws.first_cp, ws.first_cp, 0, ws.GA, 64, 0, H, W)
    return R.grads


class _GeneratorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net, cem, *params):
        latent = net.latent_input is not None
        pre_pad = cem is not None and cem.pre_pad
        m = int(cem.margins_LR) if pre_pad else 0
        Bn, _, h, w = x.shape
        ws = _train_workspace(net, x.device, Bn, h + 2 * m, w + 2 * m, latent)
        out, _ = E._forward(net, x.detach().contiguous(), cem, 'f32', train_ws=ws)
        ctx.net, ctx.cem, ctx.ws, ctx.latent, ctx.M = net, cem, ws, latent, E.SF * m
        ctx.params = params
        return out

    @staticmethod
    def backward(ctx, d_out):
        grads = generator_backward(ctx.net, ctx.cem, ctx.ws, d_out, ctx.latent, ctx.M)
        return (None, None, None) + tuple(grads.get(p) for p in ctx.params)


def generator_forward_train(net, x, cem):
    params = [p for p in net.parameters()]
    return _GeneratorFn.apply(x, net, cem, *params)
