"""HIP executor for the RRDB ×4 generator (+ CEM) forward.

Replaces the PyTorch op graph of RRDBNet.forward (architecture.py:151-175) and CEM_PyTorch.forward (CEMnet.py:169-190)
with a fixed sequence of libesr_amd launches over preallocated padded-NHWC workspaces.

Precision modes (per call: `net.esr_precision`, default env ESR_PRECISION or 'x3'):
  'x3'  activations carried as f16 hi/lo pairs, products on f16 MFMA with fp32 accumulation (esr_conv_x3.hip);
        ~1e-6 relative error, 5.3× the MFMA rate of exact fp32.  If any activation leaves the f16 range the call is
        transparently recomputed in 'f32' (the overflow flag is checked once per forward).
  'f32' exact fp32 MFMA (esr_conv.hip).

Memory plan (per (device, B, H, W, latent) — H×W is the LR grid the generator runs on, i.e. after CEM pre-pad):
  ZC = 8 latent channels slot (3 used, 5 zero) in latent mode, 0 otherwise; XOFF = ZC.
  first [B][H+2][W+2][16|8]   conv_first input: Z_LR at 0..2, LR at 8..10 (latent) | LR at 0..2 (plain)
  fea   [B][H+2][W+2][64]     conv_first output, the ShortcutBlock skip (block.py:96)
  P0..2 [B][H+2][W+2][ZC+192] RDB concat buffers: [Z | x(64) | x1 | x2 | x3 | x4 (32 each)].  conv_i of an RDB reads
                              the channel prefix [0, ZC+64+32i) and writes its 32 growth channels right after it, so
                              torch.cat (block.py:234,265,92) never happens.  RRDB k: P0 -RDB1-> P1.x -RDB2-> P2.x
                              -RDB3-> P0.x (in place, pointwise residual), P0.x carrying the trunk.
  U0    [B][H+2][W+2][64]     LR_conv + skip output
  U1    [B][2H+2][2W+2][64]   upconv-1 output
  HR0/1 [B][4H+2][4W+2][ZC+64] upconv-2 / HR_conv0 outputs with Z_HR in the slot
  gen   [B][3][4H][4W]        HR_conv1 output (fp32 NCHW, consumed by the CEM stencils)
Every buffer holds 4 bytes per channel in either mode (fp32, or an f16 hi/lo pair).  Halos and unused channels are
zero from allocation and never written.
"""
import contextlib
import ctypes
import math
import operator
import os
import warnings

import numpy as np
import torch

from . import _lib

SF = 4
CEM_PHASE = SF - SF // 2 - 1  # calc_strides(None, 4) pre_stride (imresize_CEM.py:83-85)
_FOLD = (((1., 0., 0.), (0., 1., 1.)), ((1., 1., 0.), (0., 0., 1.)))  # nearest-×2 polyphase tap folding, phase 0/1
# nearest-×f upconv: output phase p of an upsampled axis is a 2-tap conv on the LR grid at offsets (t0 - 1, t0); its
# taps are the 3 conv taps k summed by the LR pixel floor((f·y + p + k - 1) / f) they read.  (fold rows, t0) per phase
_FOLDS = {2: ((_FOLD[0], 0), (_FOLD[1], 1))}


def cem_phase(sf):
    """calc_strides(None, sf) pre_stride (imresize_CEM.py:83-85): the sub-pixel phase of the CEM's strided filters."""
    return sf - sf // 2 - 1


def up_stages(net):
    """The upsampler stages of RRDBNet: [(module index, factor)] — two ×2 for ×4, one for ×2."""
    n, f = getattr(net, 'n_up', 2), getattr(net, 'up_factor', 2)
    return [(2 + i, f) for i in range(n)]
DEFAULT_PRECISION = os.environ.get('ESR_PRECISION', 'x3')
PRECISIONS = ('x3', 'f32')

# Optional per-launch profiling (bench.py): a list collecting (tag, algorithmic FLOPs, start event, end event).
_PROFILE = None
_TIMER_POOL = {}  # op count -> esr timers created ahead of a timed region (reserve_timers)


def reserve_timers(n_ops, count):
    """Create `count` per-op HIP-event timers for op lists of `n_ops` launches now, so that a profiled timed region
    takes them from the pool instead of creating n_ops + 1 events per forward inside it (hipEventCreate is a host call
    of several µs; ~360 per forward left the GPU idle ~3 % of a bench step)."""
    lib = _lib.load()
    pool = _TIMER_POOL.setdefault(int(n_ops), [])
    for _ in range(count):
        t = lib.esr_timer_create(int(n_ops))
        if not t:
            raise RuntimeError('esr_amd: esr_timer_create failed')
        pool.append(t)


def release_timers():
    """Destroy the timers reserve_timers created and no profiled forward used."""
    lib = _lib.load()
    for pool in _TIMER_POOL.values():
        while pool:
            lib.esr_timer_destroy(pool.pop())
# Number of forwards recomputed in f32 after an f16-range overflow (observability; tests read it).
OVERFLOW_RERUNS = 0
# Activation scale of the x3 forward (a power of two A): every split activation holds A·v (the prep kernel scales the
# inputs, every x3 conv adds its bias × A, LeakyReLU and the residual adds are homogeneous, the planar HR_conv1 output is
# divided by A), so that small activations keep their f16 lo parts in the normal range: a value v is carried to ~2^-22
# relative only while |A·v| >= 2^-3 (below, the lo part is an f16 subnormal with 2^-24 absolute steps).  A forward whose
# scaled activation leaves f16's range is redone in exact fp32 and the model's A is lowered 16× (lower_act_scale).
ACT_SCALE = float(os.environ.get('ESR_ACT_SCALE', '256'))


def act_scale(net):
    return getattr(net, '_esr_act_scale', ACT_SCALE)


# Number of activation-scale reductions (observability: each one trades small-activation precision for range, for
# the rest of the model's life; benchmarks record it, tests/test_gpu_state.py pins the behaviour).
ACT_SCALE_REDUCTIONS = 0


def lower_act_scale(net):
    """A scaled activation of an x3 forward left f16's range: the model's A drops 16× (floor 1) and stays there — a
    deliberate one-way ratchet, so a model fed out-of-range inputs does not overflow (and rerun in fp32) again and
    again; ACT_SCALE_REDUCTIONS counts the reductions that happened and each is reported once (an overflow at the floor
    A = 1 lowers nothing and reports nothing: the fp32 rerun is counted in OVERFLOW_RERUNS)."""
    global ACT_SCALE_REDUCTIONS
    old = act_scale(net)
    new = max(1.0, old / 16)
    if new >= old:
        return
    net._esr_act_scale = new
    ACT_SCALE_REDUCTIONS += 1
    warnings.warn('esr_amd: x3 activation scale of %s lowered %g -> %g after an f16-range overflow'
                  % (type(net).__name__, old, new), RuntimeWarning, stacklevel=2)


def _prof_begin(prof, tag, flops, nbytes=0.0):
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    prof.append((tag, flops, start, end, nbytes))
    return end


def _require_device(t, what):
    if not t.is_cuda:
        raise RuntimeError('esr_amd: %s must be a ROCm device tensor (this build has no CPU path)' % what)
    if t.dtype != torch.float32:
        raise RuntimeError('esr_amd: %s must be float32 (got %s)' % (what, t.dtype))


# ----------------------------------------------------------------------------------------------------------------------
# weight packing
# ----------------------------------------------------------------------------------------------------------------------
def pack_conv_weight(w, cmap, n_pad):
    """[Cout][Cin_ref][k][k] -> packed [nchunk][k*k][n_pad][32] (include/esr_amd.h); cmap[c] = reference input channel
    feeding buffer channel c, or -1 for a zero (padding) channel."""
    cout, cin_ref, kh, kw = w.shape
    T = kh * kw
    nch = (len(cmap) + 31) // 32
    src = w.detach().permute(1, 2, 3, 0).reshape(cin_ref, T, cout)
    out = torch.zeros(nch * 32, T, n_pad, device=w.device, dtype=w.dtype)
    cm = np.asarray(cmap)
    dst_idx = np.nonzero(cm >= 0)[0]
    out[torch.as_tensor(dst_idx, device=w.device), :, :cout] = src[torch.as_tensor(cm[dst_idx], device=w.device)]
    return out.view(nch, 32, T, n_pad).permute(0, 2, 3, 1).contiguous()


def split_f16(x):
    """fp32 -> (hi, lo) f16 with hi = f16(x), lo = f16(x - hi)."""
    hi = x.half()
    return hi, (x - hi.float()).half()


def pack_x3(packed):
    """fp32 packed weights [nch32][T][n_pad][32] -> x3 layout [nch16][T][n_pad][2 groups][hi 8 | lo 8] (f16): 16-channel
    K chunks (esr_conv_x3.hip), scaled by a power of two so that max|w|·scale lies in [2^14, 2^15) (lo parts stay out
    of the f16 subnormal range)."""
    amax = float(packed.abs().max())
    e = 0 if amax == 0.0 else 14 - math.floor(math.log2(amax))
    scale = 2.0 ** e
    n32, T, n_pad, _ = packed.shape
    p16 = packed.view(n32, T, n_pad, 2, 16).permute(0, 3, 1, 2, 4).reshape(2 * n32, T, n_pad, 16)
    hi, lo = split_f16(p16 * scale)
    sh = (2 * n32, T, n_pad, 2, 1, 8)
    out = torch.cat([hi.reshape(sh), lo.reshape(sh)], dim=4).contiguous()
    return out, scale


def to_split(x_nhwc):
    """fp32 [..., C] (C % 8 == 0) -> split-f16 layout with the same byte size, returned as float32 storage."""
    hi, lo = split_f16(x_nhwc)
    sh = x_nhwc.shape[:-1] + (x_nhwc.shape[-1] // 8, 1, 8)
    return torch.cat([hi.reshape(sh), lo.reshape(sh)], dim=-2).reshape(x_nhwc.shape[:-1] + (x_nhwc.shape[-1] * 2,)) \
        .view(torch.float32)


def from_split(buf):
    """Inverse of to_split: float32-storage [..., C] in split layout -> fp32 values."""
    h = buf.contiguous().view(torch.float16)
    sh = buf.shape[:-1] + (buf.shape[-1] // 8, 2, 8)
    h = h.reshape(sh).float()
    return (h[..., 0, :] + h[..., 1, :]).reshape(buf.shape)


FOLD_TERMS = 4  # a folded phase tap sums at most 2 × 2 of the 3×3 taps


def fold_terms(py, px, f=2):
    """Output phase (py, px) of a nearest-×f upconv: for each of its 2×2 LR taps (a, b), the 3×3 taps (y, x) summed
    into it, in the fixed order in which fold_upconv_phase and GatherPlan.reg_sum add them: x-major, i.e. the order of
    round 3's einsum fold on the GPU (tools/fold_order_probe.py), so that the folded weights are bitwise the same.  (A
    near-cancelling discriminator bias gradient of the config-3 grid test, an exact-fp32 run, moved from 81 % to 125 %
    of its bound under the row-major order: profiles/r4_c3_fold_order.txt.)"""
    Fy, Fx = _FOLDS[f][py][0], _FOLDS[f][px][0]
    return [[[(y, x) for x in range(3) for y in range(3) if Fy[a][y] and Fx[b][x]] for b in range(2)] for a in range(2)]


def fold_term_images(w, py, px, f=2):
    """fold_upconv_phase as FOLD_TERMS tensors [Cout][Cin][2][2] whose sum ((t0 + t1) + t2) + t3 is the folded weight:
    term k holds the k-th summed 3×3 tap of each phase tap, or 0."""
    terms = fold_terms(py, px, f)
    out = [w.new_zeros(w.shape[0], w.shape[1], 2, 2) for _ in range(FOLD_TERMS)]
    for a in range(2):
        for b in range(2):
            for k, (y, x) in enumerate(terms[a][b]):
                out[k][:, :, a, b] = w[:, :, y, x]
    return out


def fold_upconv_phase(w, py, px, f=2):
    """Nearest-×f upsample then 3×3 conv == per output phase (py,px) a 2×2 conv on the LR grid whose taps are sums of
    the 3×3 taps landing on the same source pixel (block.py:294-301)."""
    t = fold_term_images(w.detach(), py, px, f)
    return ((t[0] + t[1]) + t[2]) + t[3]


class _ConvW:
    """One conv's packed weights in both precisions (x3 built lazily) + its bias parameter (and, for the x3 forward,
    the bias × the activation scale: _Packed.act_bias)."""
    __slots__ = ('f32', 'bias', '_x3', 'bias_s')

    def __init__(self, f32, bias):
        self.f32, self.bias, self._x3, self.bias_s = f32, bias, None, None

    def x3(self):
        if self._x3 is None:
            self._x3 = pack_x3(self.f32)
        return self._x3


class GatherPlan:
    """Every packed weight layout of a network as ONE gather from its flattened parameters.

    The layouts (channel maps, padding, rot180/transpose for the data gradient, 0.2 residual scales) are pure
    permutations with zero fill, so they are derived once by running the packing code on *index images* of the
    parameters (float64 tensors holding 1-based flat positions; 0 = zero fill; +k·N selects the k-th scaled copy).
    `refresh()` then rebuilds all packed tensors in place after an optimiser step with one cat + one index_select,
    instead of thousands of small copies per step."""

    def __init__(self, params, scales=(1.0,)):
        self.params = list(params)
        self.scales = tuple(scales)
        self.N = sum(p.numel() for p in self.params)
        self._img, off = {}, 1
        for p in self.params:
            self._img[id(p)] = torch.arange(off, off + p.numel(), dtype=torch.float64).view(p.shape)
            off += p.numel()
        self._parts = []
        self._sums = []
        self.buf = self.idx = self.sidx = None
        self.n_gather = 0

    def w(self, p):
        return self._img[id(p)]

    def scaled(self, t, s):
        k = self.scales.index(s)
        return t if k == 0 else torch.where(t > 0, t + k * self.N, t)

    def reg(self, t):
        self._parts.append(t)
        return t

    def reg_sum(self, terms):
        """A packed tensor that is the sum ((t0 + t1) + t2) + t3 of FOLD_TERMS gathers (index images of one shape; 0 =
        a zero term): the nearest-×2 upconv phases (fold_term_images), refreshed with the rest instead of being folded
        and packed again after every optimiser step.  Returns the key (the first term) that finalize maps to the view."""
        assert len(terms) == FOLD_TERMS and all(t.shape == terms[0].shape for t in terms)
        self._sums.append(terms)
        return terms[0]

    def finalize(self, dev):
        """Allocate the packed buffer; returns {id(index tensor): device view} for the caller to swap in."""
        n = sum(t.numel() for t in self._parts)
        m = sum(ts[0].numel() for ts in self._sums)
        self.n_gather = n
        self.buf = torch.empty(n + m, device=dev, dtype=torch.float32)
        self.idx = torch.cat([t.reshape(-1) for t in self._parts]).to(torch.int64).to(dev)
        if self._sums:
            self.sidx = torch.stack([torch.cat([ts[k].reshape(-1) for ts in self._sums])
                                     for k in range(FOLD_TERMS)]).to(torch.int64).to(dev)
        views, o = {}, 0
        for t in self._parts:
            views[id(t)] = self.buf[o:o + t.numel()].view(t.shape)
            o += t.numel()
        for ts in self._sums:
            views[id(ts[0])] = self.buf[o:o + ts[0].numel()].view(ts[0].shape)
            o += ts[0].numel()
        self._parts = self._sums = None
        return views

    def _flat_source(self):
        """The FlatAdam buffer (flat_optim.py) if the parameters are exactly its consecutive views, else None.  The full
        check runs once per (buffer, parameter addresses); later calls compare the addresses only (~0.1 instead of
        ~0.4 ms of host time on RRDB-23's 702 parameters, several calls per training step)."""
        fl = getattr(self.params[0], '_esr_flat', None)
        if fl is None or fl.numel() != self.N:
            return None
        ptrs = list(map(_DATA_PTR, self.params))
        ok = self.__dict__.get('_flat_ok')
        if ok is not None and ok[0] is fl and ok[1] == ptrs:
            return fl.detach()
        base, o = fl.data_ptr(), 0
        for p, ptr in zip(self.params, ptrs):
            if getattr(p, '_esr_flat', None) is not fl or ptr != base + 4 * o or not p.is_contiguous():
                return None
            o += p.numel()
        self._flat_ok = (fl, ptrs)
        return fl.detach()

    def refresh(self):
        flat = self._flat_source()
        if flat is None:
            flat = torch.cat([p.detach().reshape(-1) for p in self.params])
        ext = torch.cat([flat.new_zeros(1)] + [flat * s if s != 1.0 else flat for s in self.scales])
        torch.index_select(ext, 0, self.idx, out=self.buf[:self.n_gather])
        if self.sidx is not None:
            g = ext[self.sidx]
            out = self.buf[self.n_gather:]
            torch.add(g[0], g[1], out=out)
            out.add_(g[2])
            out.add_(g[3])


class _Packed:
    """Packed weights of one generator: built once per parameter set (GatherPlan), refreshed in place when any
    parameter changes (in-place version bump, e.g. an optimiser step or load_state_dict)."""

    def __init__(self, net, latent):
        def lr_map(n_feat):  # [Z(3) pad(5)] + features, reference order [Z, features]
            if not latent:
                return list(range(n_feat))
            return [0, 1, 2] + [-1] * 5 + [3 + c for c in range(n_feat)]

        self.net = net
        plan = self.plan = GatherPlan(param_list(net))
        pk = lambda conv, cmap, n_pad: plan.reg(pack_conv_weight(plan.w(conv.weight), cmap, n_pad))  # noqa: E731
        m = net.model
        first_map = ([0, 1, 2] + [-1] * 5 + [3, 4, 5] + [-1] * 5) if latent else ([0, 1, 2] + [-1] * 5)
        self.first = _ConvW(pk(m[0], first_map, 64), m[0].bias)
        self.rdb = []
        for k in range(net.nb):
            rr = m[1].sub[k]
            for rdb in (rr.RDB1, rr.RDB2, rr.RDB3):
                self.rdb.append([_ConvW(pk(rdb.convs[i][0], lr_map(64 + 32 * i), 32 if i < 4 else 64),
                                        rdb.convs[i][0].bias) for i in range(5)])
        lrc = m[1].sub[net.nb]
        self.lr_conv = _ConvW(pk(lrc, lr_map(64), 64), lrc.bias)
        i0 = 2 + getattr(net, 'n_up', 2)  # HR_conv0, then its LeakyReLU, then HR_conv1
        self.hr0 = _ConvW(pk(m[i0], lr_map(64), 64), m[i0].bias)
        self.hr1 = _ConvW(pk(m[i0 + 2], lr_map(64), 32), m[i0 + 2].bias)
        # the upsampler phases: sums of taps (fold_upconv_phase), refreshed by the plan's summed gather
        self.up = []
        for j, f in up_stages(net):
            c = m[j][1]
            self.up.append([_ConvW(plan.reg_sum([pack_conv_weight(t, list(range(64)), 64)
                                                 for t in fold_term_images(plan.w(c.weight), py, px, f)]), c.bias)
                            for py in range(f) for px in range(f)])
        views = plan.finalize(net.model[0].weight.device)
        self.planned = [self.first, self.lr_conv, self.hr0, self.hr1] + [cw for r in self.rdb for cw in r]
        for cw in self.planned + [c for row in self.up for c in row]:
            cw.f32 = views[id(cw.f32)]

    def train_x3(self):
        """x3 weights for the training / Z-optimisation forward, rebuilt IN PLACE after every parameter change with no
        host sync: each layer keeps the power-of-two scale pack_x3 chose at the first build (so recorded launches and
        captured graphs stay valid), and all planned layers are split in one gather over the packed fp32 buffer.
        Returns a persistent device int32 flag, 1 if any scaled weight left the safe f16 range; the caller then falls
        back to fp32 for that step and calls reset_train_x3() so the next build picks new scales."""
        convs = self.planned + [c for row in self.up for c in row]
        if getattr(self, '_tx3', None) is None:
            scales = [pack_x3(cw.f32)[1] for cw in convs]  # one host sync per layer, at the first build only
            self._tx3_epoch = getattr(self, '_tx3_epoch', 0) + 1
            buf = self.plan.buf
            idx, sc, views, off = [], [], [], 0
            outs = []
            for cw, scl in zip(convs, scales):  # every layer is a view of the plan's buffer (upsampler phases too)
                n32, T, n_pad, _ = cw.f32.shape
                base = cw.f32.storage_offset() - buf.storage_offset()
                i = torch.arange(base, base + cw.f32.numel(), device=buf.device).view(cw.f32.shape)
                idx.append(i.view(n32, T, n_pad, 2, 16).permute(0, 3, 1, 2, 4).reshape(-1))
                sc.append(torch.full((cw.f32.numel(),), scl, device=buf.device))
                views.append((off, (2 * n32, T, n_pad, 2, 2, 8)))
                off += 2 * cw.f32.numel()
            self._tx3_idx, self._tx3_scale = torch.cat(idx), torch.cat(sc)
            self._tx3 = torch.empty(off, device=buf.device, dtype=torch.float16)
            for cw, scl, (o, shp) in zip(convs, scales, views):
                n = 1
                for d in shp:
                    n *= d
                outs.append((cw, self._tx3[o:o + n].view(shp), scl))
            self._tx3_layers = outs
            self._tx3_bad = torch.zeros(1, device=buf.device, dtype=torch.int32)
            self._tx3_version = None
        if self._tx3_version != getattr(self, 'version', 0):
            g = self.plan.buf[self._tx3_idx] * self._tx3_scale
            hi = g.half()
            lo = (g - hi.float()).half()
            G = g.numel() // 8
            self._tx3.view(G, 2, 8).copy_(torch.stack([hi.view(G, 8), lo.view(G, 8)], 1))
            self._tx3_bad.copy_((g.abs().amax() >= 61440.0).to(torch.int32).view(1))
            self._tx3_version = getattr(self, 'version', 0)
        for cw, view, scl in self._tx3_layers:
            cw._x3 = (view, scl)
        return self._tx3_bad

    def reset_train_x3(self):
        self._tx3 = None

    def act_bias(self, A):
        """The x3 forward's biases × A (the activation scale, act_scale): one persistent buffer, refreshed by one gather
        from the parameters when they or A change (pointers stay fixed for recorded op lists and captured graphs); sets
        every conv's bias_s.  HR_conv1 keeps its own bias: its planar output is divided by A instead."""
        convs = [cw for cw in self.planned if cw is not self.hr1] + [c for row in self.up for c in row]
        if getattr(self, '_bs', None) is None:
            offs, o = {}, 0
            for p in self.plan.params:
                offs[id(p)] = o
                o += p.numel()
            idx, spans, o = [], [], 0
            for cw in convs:
                n = cw.bias.numel()
                idx.append(torch.arange(offs[id(cw.bias)], offs[id(cw.bias)] + n))
                spans.append((o, n))
                o += n
            dev = self.plan.buf.device
            self._bs_idx = torch.cat(idx).to(dev)
            self._bs = torch.empty(o, device=dev, dtype=torch.float32)
            for cw, (a, n) in zip(convs, spans):
                cw.bias_s = self._bs[a:a + n]
            self._bs_key = None
        key = (getattr(self, 'version', 0), A)
        if self._bs_key != key:
            flat = self.plan._flat_source()
            if flat is None:
                flat = torch.cat([p.detach().reshape(-1) for p in self.plan.params])
            torch.index_select(flat, 0, self._bs_idx, out=self._bs)
            self._bs.mul_(A)
            self._bs_key = key
        self.hr1.bias_s = self.hr1.bias

    def refresh(self):
        self.plan.refresh()  # in place: recorded op lists and captured HIP graphs keep valid pointers
        self.version = getattr(self, 'version', 0) + 1  # invalidates recorded op lists (new x3 weight tensors)
        for cw in self.planned + [c for row in self.up for c in row]:
            cw._x3 = None


def param_list(m):
    """list(m.parameters()), cached on the module: walking RRDB-23's module tree for its 702 parameters costs ~5 ms
    of host time per call, and a training step needs the list several times.  The cache is revalidated on every
    call (each cached (module, name) slot must still hold the same Parameter object: ~0.09 ms for RRDB-23 as one
    C-level map, 0.13 as a generator expression); adding new submodules after the first call is not detected."""
    c = m.__dict__.get('_esr_plist')
    if c is not None:
        mods, names, plist = c
        if all(map(operator.is_, map(dict.get, map(_PARAMS, mods), names), plist)):
            return plist
    mods, names, plist, seen = [], [], [], set()
    for mod in m.modules():
        for n, q in mod._parameters.items():
            if q is not None and id(q) not in seen:
                seen.add(id(q))
                mods.append(mod)
                names.append(n)
                plist.append(q)
    m.__dict__['_esr_plist'] = (mods, names, plist)
    return plist


_PARAMS = operator.attrgetter('_parameters')
_VERSION = operator.attrgetter('_version')
_DATA_PTR = torch.Tensor.data_ptr


def _param_key(net):
    return _keys(net)[1]


def _struct_key(net):
    return _keys(net)[0]


def _keys(net):
    """(structure key: every parameter's address and shape; value key: their addresses and version counters) in one
    pass over the parameter list.  Parameters bound to a FlatAdam buffer (flat_optim.py) change when the buffer is
    updated in place, which bumps the buffer's version counter, not theirs."""
    ps = param_list(net)
    ptrs = list(map(_DATA_PTR, ps))
    c = net.__dict__.get('_esr_skey')  # the shapes are re-read only when a pointer changed (~0.5 ms per call saved)
    if c is not None and c[0] is ps and c[1] == ptrs:
        sk = c[2]
    else:
        sk = tuple(zip(ptrs, [p.shape for p in ps]))
        net.__dict__['_esr_skey'] = (ps, ptrs, sk)
    vk = [tuple(ptrs), tuple(map(_VERSION, ps))]
    fl = getattr(ps[0], '_esr_flat', None) if ps else None
    if fl is not None:
        vk.append((id(fl), fl._version))
    return sk, tuple(vk)


def _packed(net, latent):
    sk, vkey = _keys(net)
    skey = (sk, latent)
    c = net._esr_cache.get('packed')
    if c is None or c[0] != skey:
        net._esr_cache.pop('packed', None)
        with torch.no_grad():
            c = [skey, None, _Packed(net, latent)]
        net._esr_cache['packed'] = c
    if c[1] != vkey:
        with torch.no_grad():
            c[2].refresh()
        c[1] = vkey
    return c[2]


class _Workspace:
    def __init__(self, dev, B, H, W, latent, sf=4):
        zc = 8 if latent else 0
        z = lambda *s: torch.zeros(*s, device=dev, dtype=torch.float32)  # noqa: E731
        self.B, self.H, self.W, self.zc = B, H, W, zc
        self.first_cp = 16 if latent else 8
        self.first_lr_off = 8 if latent else 0
        self.cp = zc + 192
        self.hr_cp = zc + 64
        self.first = z(B, H + 2, W + 2, self.first_cp)
        self.fea = z(B, H + 2, W + 2, 64)
        self.P = [z(B, H + 2, W + 2, self.cp) for _ in range(3)]
        self.U0 = z(B, H + 2, W + 2, 64)
        self.U1 = z(B, 2 * H + 2, 2 * W + 2, 64) if sf == 4 else None  # between the two ×2 upconvs of ×4
        self.HR = [z(B, sf * H + 2, sf * W + 2, self.hr_cp) for _ in range(2)]
        self.lr = z(B, 3, H, W)
        self.overflow = torch.zeros(1, device=dev, dtype=torch.int32)
        self.Y = None  # x3 inference: HR_conv1's per-tap partial products (esr_hr_convs_x3), allocated on first use


# workspace slot of the inference forward being built: each batch part of a multi-stream forward (generator_forward)
# has buffers of its own
_WS_SLOT = [0]


def _workspace(net, dev, B, H, W, latent, precision, slot=None):
    # keyed by precision too: the zero padding channels of an fp32 workspace are not zero when read as split-f16 pairs
    sf = getattr(net, 'upscale', SF)
    key = (str(dev), B, H, W, latent, precision, sf)
    name = ('ws_' + slot) if slot else ('ws' if _WS_SLOT[0] == 0 else 'ws%d' % _WS_SLOT[0])
    c = net._esr_cache.get(name)
    if c is None or c[0] != key:
        net._esr_cache.pop(name, None)  # free the previous shape's buffers first
        c = (key, _Workspace(dev, B, H, W, latent, sf))
        net._esr_cache[name] = c
    return c[1]


def _conv_out(out, cp, coff, oh, ow, lrelu, sy=1, sx=1, oy=0, ox=0, planar=0, r1=None, r1_cp=0, r1_coff=0, s1=1.0,
              r2=None, r2_cp=0, r2_coff=0, s2=1.0, out2=None, out2_cp=0, out2_coff=0):
    return _lib.ConvOut(out.data_ptr(), cp, coff, oh, ow, sy, sx, oy, ox, planar, int(lrelu),
                        None if r1 is None else r1.data_ptr(), r1_cp, r1_coff, s1,
                        None if r2 is None else r2.data_ptr(), r2_cp, r2_coff, s2,
                        None if out2 is None else out2.data_ptr(), out2_cp, out2_coff)


# ----------------------------------------------------------------------------------------------------------------------
# op lists: a forward recorded once, replayed natively (esr_run_ops)
# ----------------------------------------------------------------------------------------------------------------------
class _Recorder:
    """Stands in for the library inside `_forward`: every launch becomes an esr_op record (include/esr_amd.h) instead
    of being issued.  Tensors allocated during recording are kept alive by the recorder (`keep`)."""

    def __init__(self):
        self.ops, self.tags, self.keep = [], [], []
        self._tag = None

    def tag(self, name, flops, nbytes=0.0):
        self._tag = (name, flops, nbytes)

    def _add(self, kind, p, i, f=(), o=None):
        op = _lib.EsrOp()
        op.kind = kind
        for k, v in enumerate(p):
            op.p[k] = v
        for k, v in enumerate(i):
            op.i[k] = v
        for k, v in enumerate(f):
            op.f[k] = v
        if o is not None:
            op.o = o._obj if hasattr(o, '_obj') else o
        self.ops.append(op)
        self.tags.append(self._tag)
        self._tag = None
        return 0

    def esr_conv3x3_fwd(self, inp, B, H, W, in_cp, cin, w, bias, cout, o, stream):
        return self._add(_lib.OP_CONV3X3, [inp, w, bias], [B, H, W, in_cp, cin, cout], o=o)

    def esr_conv3x3_fwd_x3(self, inp, B, H, W, in_cp, cin, w, bias, w_scale, cout, o, ovf, stream):
        return self._add(_lib.OP_CONV3X3_X3, [inp, w, bias, ovf], [B, H, W, in_cp, cin, cout], [w_scale], o=o)

    def esr_upconv2x_phase_fwd(self, inp, B, H, W, in_cp, cin, w, bias, cout, py, px, o, stream):
        return self._add(_lib.OP_UPCONV, [inp, w, bias], [B, H, W, in_cp, cin, cout, py, px], o=o)

    def esr_upconv2x_phase_fwd_x3(self, inp, B, H, W, in_cp, cin, w, bias, w_scale, cout, py, px, o, ovf, stream):
        return self._add(_lib.OP_UPCONV_X3, [inp, w, bias, ovf], [B, H, W, in_cp, cin, cout, py, px], [w_scale], o=o)

    def esr_prep_input_s(self, x, B, nz, h, w, sf, m, lr, first, first_cp, first_lr_off, zlr, zlr_cp, n_zlr, zhr,
                         zhr_cp, n_zhr, split, act_scale, stream):
        return self._add(_lib.OP_PREP, [x, lr, first] + [zlr[k] for k in range(4)] + [zhr[k] for k in range(2)],
                         [B, nz, h, w, sf, m, first_cp, first_lr_off] + [zlr_cp[k] for k in range(4)] + [n_zlr] +
                         [zhr_cp[k] for k in range(2)] + [n_zhr, split], [act_scale])

    def esr_cem_down(self, gen, lr, r, B, H, W, sf, ph, w, kd, negate, stream):
        return self._add(_lib.OP_CEM_DOWN, [gen, lr, r, w], [B, H, W, sf, ph, kd, negate])

    def esr_cem_inv(self, r, q, B, H, W, w, ki, stream):
        return self._add(_lib.OP_CEM_INV, [r, q, w], [B, H, W, ki])

    def esr_cem_up_add(self, q, gen, out, B, H, W, sf, ph, w, kd, M, stream):
        return self._add(_lib.OP_CEM_UP_ADD, [q, gen, out, w], [B, H, W, sf, ph, kd, M])

    def esr_hr_convs_x3(self, inp, B, H, W, in_cp, zc, w0, bias0, w0_scale, w1, y, ovf, stream):
        return self._add(_lib.OP_HR_CONVS_X3, [inp, w0, bias0, w1, y, ovf], [B, H, W, in_cp, zc], [w0_scale])

    def esr_hr1_sum(self, y, B, H, W, bias1, scale_inv, out, stream):
        return self._add(_lib.OP_HR1_SUM, [y, bias1, out], [B, H, W], [scale_inv])


class _OpPlan:
    """One recorded inference forward.  Between calls only the model-input pointer and the output pointer change;
    they are patched in place and the whole list runs in one esr_run_ops call."""

    def __init__(self, key, net, x, cem, precision):
        rec = _Recorder()
        out, ws = _forward(net, x, cem, precision, rec=rec)
        self.key, self.ws, self.keep, self.tags = key, ws, rec.keep, rec.tags
        self.n = len(rec.ops)
        self.ops = (_lib.EsrOp * self.n)(*rec.ops)
        self.out_shape = tuple(out.shape)
        xp, op_ = x.data_ptr(), out.data_ptr()
        self.x_sites, self.out_sites = [], []
        for k in range(self.n):
            for j in range(10):
                if self.ops[k].p[j] == xp:
                    self.x_sites.append((k, j))
                elif self.ops[k].p[j] == op_:
                    self.out_sites.append((k, j))
            if self.ops[k].o.out == op_:
                self.out_sites.append((k, -1))
        if not self.x_sites or not self.out_sites:
            raise RuntimeError('esr_amd: op-list recording did not find the input/output of the forward')

    def run(self, x, out=None):
        lib = _lib.load()
        if out is None:
            out = torch.empty(self.out_shape, device=x.device, dtype=torch.float32)
        elif tuple(out.shape) != self.out_shape or not out.is_contiguous():
            raise RuntimeError('esr_amd: op-list output view of the wrong shape')
        for k, j in self.x_sites:
            self.ops[k].p[j] = x.data_ptr()
        for k, j in self.out_sites:
            if j < 0:
                self.ops[k].o.out = out.data_ptr()
            else:
                self.ops[k].p[j] = out.data_ptr()
        timer = None
        if _PROFILE is not None:
            pool = _TIMER_POOL.get(self.n)
            timer = pool.pop() if pool else lib.esr_timer_create(self.n)
            if not timer:
                raise RuntimeError('esr_amd: esr_timer_create failed')
            _PROFILE.append(('ops', self.tags, timer, self.n))
        stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        _lib.check(lib.esr_run_ops(self.ops, self.n, timer, stream), 'esr_run_ops')
        return out


def profile_records(prof):
    """(tag, flops, ms) of every profiled launch in `prof` (engine._PROFILE list): op-list entries are read from
    their native HIP-event timers (and the timers freed), direct-launch entries from torch events."""
    lib = _lib.load()
    for entry in prof:
        if entry[0] == 'ops':
            _, tags, timer, n = entry
            ms = (ctypes.c_float * n)()
            _lib.check(lib.esr_timer_elapsed(timer, ms), 'esr_timer_elapsed')
            lib.esr_timer_destroy(timer)
            for k in range(n):
                if tags[k] is not None:
                    yield tags[k][0], tags[k][1], ms[k]
        else:
            tag, flops, start, end = entry[:4]
            yield tag, flops, start.elapsed_time(end)


class ProfileOrigin:
    """A time origin for profile_intervals: one native HIP event and one torch event, recorded back to back on the
    current stream at the start of a timed region."""

    def __init__(self, dev):
        lib = _lib.load()
        self.timer = lib.esr_timer_create(1)
        if not self.timer:
            raise RuntimeError('esr_amd: esr_timer_create failed')
        self.event = torch.cuda.Event(enable_timing=True)
        self.dev = dev

    def record(self):
        stream = torch.cuda.current_stream(self.dev)
        _lib.check(_lib.load().esr_timer_record(self.timer, 0, ctypes.c_void_p(stream.cuda_stream)),
                   'esr_timer_record')
        self.event.record(stream)

    def close(self):
        if self.timer:
            _lib.load().esr_timer_destroy(self.timer)
            self.timer = None


def profile_intervals(prof, origin):
    """(tag, flops, start_ms, end_ms, algorithmic bytes) of every profiled launch in `prof`, times from `origin` (a recorded
    ProfileOrigin): launches of several streams overlap, so a rate over them divides by the union of their intervals,
    not by the sum of their durations.  Frees the op-list timers like profile_records."""
    lib = _lib.load()
    for entry in prof:
        if entry[0] == 'ops':
            _, tags, timer, n = entry
            t = (ctypes.c_float * (n + 1))()
            _lib.check(lib.esr_timer_stamps(timer, origin.timer, t), 'esr_timer_stamps')
            lib.esr_timer_destroy(timer)
            for k in range(n):
                if tags[k] is not None:
                    yield tags[k][0], tags[k][1], t[k], t[k + 1], tags[k][2]
        else:
            tag, flops, start, end, nbytes = entry
            yield tag, flops, origin.event.elapsed_time(start), origin.event.elapsed_time(end), nbytes


def union_ms(intervals):
    """Length of the union of (start, end) intervals."""
    tot, hi = 0.0, None
    for a, b in sorted(intervals):
        if hi is None or a > hi:
            tot += b - a
            hi = b
        elif b > hi:
            tot += b - hi
            hi = b
    return tot


USE_OP_LISTS = os.environ.get('ESR_OP_LISTS', '1') != '0'
# x3 inference: HR_conv0 and HR_conv1 as esr_hr_convs_x3 + esr_hr1_sum (ESR_FUSE_HR1=0: the two convs as launched for
# training, HR_conv1 on the narrow-N kernel)
FUSE_HR1 = os.environ.get('ESR_FUSE_HR1', '1') != '0'


def _plan_key(net, x, cem, precision, pk):
    a = act_scale(net) if precision == 'x3' else 1.0
    pre_pad = cem is not None and cem.pre_pad
    cem_key = None
    if cem is not None:
        cem_key = (id(cem), pre_pad, int(cem.margins_LR),
                   cem.DownscaleOP.Filter_OP.weight.data_ptr(), cem.Conv_LR_with_Inv_hTh_OP.Filter_OP.weight.data_ptr(),
                   cem.Upscale_OP.Filter_OP.weight.data_ptr())
    return (id(pk), getattr(pk, 'version', 0), precision, tuple(x.shape), str(x.device), cem_key, a, FUSE_HR1)


def _plan(net, x, cem, precision, slot=0):
    pk = _packed(net, net.latent_input is not None)
    key = _plan_key(net, x, cem, precision, pk)
    if precision == 'x3':
        pk.act_bias(act_scale(net))  # (no-op unless the parameters or the scale changed)
    plans = net._esr_cache.setdefault('plans', {})
    plan = plans.get((precision, slot))
    if plan is None or plan.key != key:
        plans.pop((precision, slot), None)
        _WS_SLOT[0] = slot
        try:
            plan = _OpPlan(key, net, x, cem, precision)
        finally:
            _WS_SLOT[0] = 0
        plans[(precision, slot)] = plan
    return plan


def _planned_forward(net, x, cem, precision):
    plan = _plan(net, x, cem, precision)
    return plan.run(x), plan.ws


# Inference batches of at least STREAM_MIN_B images run as STREAMS parts on as many HIP streams at once (each part
# with its own workspace and op list): one part's kernels fill the GPU where another's are in their last, partly empty
# round of workgroups or between launches.  ESR_STREAMS=1: one stream (A/B).
# Only where each part alone still fills the chip for a round or more: measured at config 2 (two parts of 16 × 148²
# padded pixels each) +4.7 %; at 4 × 172² and 16 × 96² parts within ±1 %, at 4 × 154² 19 % slower
# (profiles/r5_streams_shapes.txt).
STREAMS = int(os.environ.get('ESR_STREAMS', '2'))
STREAM_MIN_B = 8
STREAM_MIN_PART_PIXELS = 300000
_SIDE_STREAMS = {}


def _side_stream(dev, k):
    key = (str(dev), k)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(dev)
    return _SIDE_STREAMS[key]


def use_streams(shape, cem):
    """Whether an inference forward of an input of `shape` runs as STREAMS batch parts (the padded LR pixels of a part
    at least STREAM_MIN_PART_PIXELS)."""
    B, _, h, w = shape
    m = 2 * int(cem.margins_LR) if (cem is not None and cem.pre_pad) else 0
    return STREAMS > 1 and B >= STREAM_MIN_B and (B // STREAMS) * (h + m) * (w + m) >= STREAM_MIN_PART_PIXELS


def _trim_slots(net, n):
    """Free the workspaces and op lists of inference slots >= n (those of a previous multi-stream forward): a later
    single-stream or smaller forward would otherwise keep a batch part's HR-resolution buffers allocated."""
    cache = net.__dict__.get('_esr_cache')
    if not cache:
        return
    for name in [k for k in cache if k.startswith('ws') and k[2:].isdigit() and int(k[2:]) >= n]:
        del cache[name]
    plans = cache.get('plans')
    if plans:
        for k in [k for k in plans if k[1] >= n]:
            del plans[k]


def _multistream_forward(net, x, cem, precision, n):
    """The batch in n parts, part k on stream k (part 0 on the current stream), results in one output tensor."""
    B = x.shape[0]
    bounds = [B * k // n for k in range(n + 1)]
    parts = [x[bounds[k]:bounds[k + 1]] for k in range(n)]
    plans = [_plan(net, parts[k], cem, precision, slot=k) for k in range(n)]  # (built once per shape)
    out = torch.empty((B,) + plans[0].out_shape[1:], device=x.device, dtype=torch.float32)
    cur = torch.cuda.current_stream(x.device)
    for k in list(range(1, n)) + [0]:  # the side streams first: each waits for the current stream's work so far only
        ok = out[bounds[k]:bounds[k + 1]]
        if k == 0:
            plans[0].run(parts[0], ok)
            continue
        st = _side_stream(x.device, k)
        st.wait_stream(cur)  # x is ready and out allocated on the current stream
        with torch.cuda.stream(st):
            plans[k].run(parts[k], ok)
        x.record_stream(st)
        out.record_stream(st)
    for k in range(1, n):
        cur.wait_stream(_side_stream(x.device, k))
    return out, [p.ws for p in plans]


# ----------------------------------------------------------------------------------------------------------------------
# forward
# ----------------------------------------------------------------------------------------------------------------------
def generator_forward(net, x, cem=None):
    """RRDBNet.forward, optionally wrapped by CEM_PyTorch.forward (cem = the CEM_PyTorch module)."""
    global OVERFLOW_RERUNS
    _require_device(x, 'generator input')
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in param_list(net))):
        # training step / Z optimisation: retained activations + HIP backward (×4 and ×2)
        from . import train_engine
        return train_engine.generator_forward_train(net, x.contiguous(), cem)
    precision = getattr(net, 'esr_precision', None) or DEFAULT_PRECISION
    if precision not in PRECISIONS:
        raise ValueError('esr_precision must be one of %s' % (PRECISIONS,))
    x = x.contiguous()
    multi = USE_OP_LISTS and use_streams(x.shape, cem)
    _trim_slots(net, STREAMS if multi else 1)
    if multi:
        out, wss = _multistream_forward(net, x, cem, precision, STREAMS)
    elif USE_OP_LISTS:
        out, ws = _planned_forward(net, x, cem, precision)
        wss = [ws]
    else:
        out, ws = _forward(net, x, cem, precision)
        wss = [ws]
    if precision == 'x3':
        flags = wss[0].overflow if len(wss) == 1 else torch.stack([w.overflow for w in wss]).amax()
        lag = _LAG[0]
        if lag is not None:  # lagged_overflow_checks(): read one forward later, after the next one is enqueued
            lag.push(net, x, cem, out, flags, wss)
        elif int(flags.item()):  # one 4-byte D2H per forward
            OVERFLOW_RERUNS += 1
            for w in wss:
                w.overflow.zero_()
            lower_act_scale(net)  # an activation (× the activation scale) left f16's range: smaller scale next time
            out, _ = _forward(net, x, cem, 'f32')
    return out


class _LaggedOverflow:
    """The x3 overflow flag of inference forward N read after forward N + 1 has been enqueued (lagged_overflow_checks):
    the host does not wait for the GPU to drain between forwards.  Forward N's flags go to pinned host memory by an
    async copy (its device flags are then cleared for N + 1) and its input is kept (a device copy: the caller may reuse
    its buffer); when N + 1 is enqueued, or the block ends, N's flags are read and an overflowed N is recomputed in exact
    fp32 INTO the tensor forward N returned (stream-ordered: every later read of it on the stream sees the fp32 result).
    The model's activation scale is lowered then — forward N + 1 was already enqueued at the old scale and is checked
    the same way."""

    def __init__(self):
        self.pending = None

    def push(self, net, x, cem, out, flags, wss):
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(flags.reshape(1).to(torch.int32), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        for w in wss:
            w.overflow.zero_()
        prev, self.pending = self.pending, (net, x.clone(), cem, out, host, ev)
        self._settle(prev)  # N - 1's flag: forward N is enqueued by now

    def _settle(self, item):
        global OVERFLOW_RERUNS
        if item is None:
            return
        net, x, cem, out, host, ev = item
        ev.synchronize()
        if int(host.item()):
            OVERFLOW_RERUNS += 1
            lower_act_scale(net)
            redo, _ = _forward(net, x, cem, 'f32', slot='redo')
            out.copy_(redo)

    def close(self):
        item, self.pending = self.pending, None
        self._settle(item)


_LAG = [None]


@contextlib.contextmanager
def lagged_overflow_checks():
    """Inference forwards in this block read their x3 overflow flag one forward late (_LaggedOverflow): a stream of
    forwards is enqueued back to back.  A tensor a forward returned holds its final (exact-fp32 if it overflowed) values
    for every reader that comes after the NEXT forward call or after the block, in stream order; read it earlier only
    after the block.  Default off: outside the block every forward checks its own flag before returning."""
    prev, _LAG[0] = _LAG[0], _LaggedOverflow()
    try:
        yield _LAG[0]
    finally:
        lag, _LAG[0] = _LAG[0], prev
        lag.close()


def _forward(net, x, cem, precision, train_ws=None, rec=None, slot=None):
    """One generator (+CEM) forward.  With `train_ws` (esr_amd.train_engine) every RDB's concat buffer is kept for
    the backward pass instead of the inference ping-pong, and the workspace comes from the caller.  With `rec` (a
    _Recorder) the launches are recorded as an op list instead of issued."""
    lib = rec if rec is not None else _lib.load()
    x3 = precision == 'x3'
    latent = net.latent_input is not None
    nz = net.nl if latent else 0
    sf = getattr(net, 'upscale', SF)
    Bn, C, h, w = x.shape
    if C != 3 + nz * sf * sf:
        raise RuntimeError('esr_amd: expected %d input channels (3 LR + %d rearranged HR latent), got %d'
                           % (3 + nz * sf * sf, nz * sf * sf, C))
    if latent and nz != 3:
        raise NotImplementedError('esr_amd latent path is built for 3 latent channels')
    pre_pad = cem is not None and cem.pre_pad
    m = int(cem.margins_LR) if pre_pad else 0
    H, W = h + 2 * m, w + 2 * m
    dev = x.device
    ws = train_ws if train_ws is not None else _workspace(net, dev, Bn, H, W, latent, precision, slot)
    pk = _packed(net, latent)
    _require_device(pk.first.bias, 'generator parameters')
    A = act_scale(net) if x3 else 1.0
    if x3:
        pk.act_bias(A)
    ws.act_scale = A
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    zc, cp, hcp = ws.zc, ws.cp, ws.hr_cp
    HR0, HR1 = ws.HR
    ovf = ws.overflow.data_ptr()
    if train_ws is None:
        P0, P1, P2 = ws.P

        def rrdb_bufs(k):  # (RRDB input, RDB1 out, RDB2 out, RRDB output): ping-pong, output in place
            return P0, P1, P2, P0
        lr_bufs = ws.P
    else:
        Q = ws.Q

        def rrdb_bufs(k):
            return Q[3 * k], Q[3 * k + 1], Q[3 * k + 2], Q[3 * k + 3]
        lr_bufs = Q

    # every concat buffer carries Z_LR in its slot; prep writes up to 4 destinations per call
    zhr = (ctypes.c_void_p * 2)(HR0.data_ptr(), HR1.data_ptr())
    zhr_cp = (ctypes.c_int32 * 2)(hcp, hcp)
    groups = [lr_bufs[i:i + 4] for i in range(0, len(lr_bufs), 4)] if nz else [[]]
    for gi, grp in enumerate(groups):
        zlr = (ctypes.c_void_p * 4)(*([t.data_ptr() for t in grp] + [None] * (4 - len(grp))))
        zlr_cp = (ctypes.c_int32 * 4)(*([cp] * 4))
        first = gi == 0
        _lib.check(lib.esr_prep_input_s(x.data_ptr(), Bn, nz, h, w, sf, m, ws.lr.data_ptr() if first else None,
                                        ws.first.data_ptr() if first else None, ws.first_cp, ws.first_lr_off, zlr,
                                        zlr_cp, len(grp), zhr, zhr_cp, 2 if (nz and first) else 0, int(x3), A, stream),
                   'esr_prep_input')
    prof = _PROFILE
    tagp = 'x3_' if x3 else ''

    def conv(inp, h_, w_, in_cp, cin, cw, cout, o, cin_ref):
        ev = None
        # timing tags: the N = 32 / 64 tile classes, and HR_conv1 (cout 3: the narrow-N kernel in x3) on its own
        ntag = '%sconv3x3_n%d' % (tagp, 3 if cout <= 3 else (32 if cout <= 32 else 64))
        # algorithmic HBM bytes: the input channels read once, the outputs (and residuals) once, the weights once
        # (4 bytes per value: fp32, or an f16 hi/lo pair)
        per_px = cin + cout * (1 + bool(o.r1) + bool(o.r2) + bool(o.out2))
        nbytes = 4.0 * (Bn * h_ * w_ * per_px + 9 * cin * cout)
        if rec is not None:
            rec.tag(ntag, 2.0 * Bn * h_ * w_ * 9 * cin_ref * cout, nbytes)
        elif prof is not None:
            ev = _prof_begin(prof, ntag, 2.0 * Bn * h_ * w_ * 9 * cin_ref * cout, nbytes)
        if x3:
            wx, scale = cw.x3()
            if rec is not None:  # the op list holds wx's pointer: keep it alive (train_x3 may swap cw._x3 later)
                rec.keep.append(wx)
            # activations carry × A: biases × A (bias_s); the planar HR_conv1 output is divided by A instead
            wsc = scale * A if cw is pk.hr1 else scale
            rc = lib.esr_conv3x3_fwd_x3(inp.data_ptr(), Bn, h_, w_, in_cp, cin, wx.data_ptr(), cw.bias_s.data_ptr(),
                                        wsc, cout, ctypes.byref(o), ovf, stream)
        else:
            rc = lib.esr_conv3x3_fwd(inp.data_ptr(), Bn, h_, w_, in_cp, cin, cw.f32.data_ptr(), cw.bias.data_ptr(),
                                     cout, ctypes.byref(o), stream)
        _lib.check(rc, 'esr_conv3x3_fwd' + ('_x3' if x3 else ''))
        if ev is not None:
            ev.record()

    nl = 3 if latent else 0  # reference latent channels concatenated into a conv input (FLOP accounting)
    # conv_first -> (RRDB 0 input).x and fea
    conv(ws.first, H, W, ws.first_cp, ws.first_cp, pk.first, 64,
         _conv_out(rrdb_bufs(0)[0], cp, zc, H, W, False, out2=ws.fea, out2_cp=64, out2_coff=0), 3 + nl)
    # nb RRDBs
    for k in range(net.nb):
        xin, b1, b2, xout = rrdb_bufs(k)
        for r, (pin, pout) in enumerate(((xin, b1), (b1, b2), (b2, xout))):
            convs = pk.rdb[3 * k + r]
            for i in range(4):
                coff = zc + 64 + 32 * i
                conv(pin, H, W, cp, coff, convs[i], 32, _conv_out(pin, cp, coff, H, W, True), nl + 64 + 32 * i)
            o = _conv_out(pout, cp, zc, H, W, False, r1=pin, r1_cp=cp, r1_coff=zc, s1=0.2,
                          r2=xin if r == 2 else None, r2_cp=cp, r2_coff=zc, s2=0.2)
            conv(pin, H, W, cp, zc + 192, convs[4], 64, o, nl + 192)
    # LR_conv + trunk skip
    trunk = rrdb_bufs(net.nb - 1)[3] if net.nb > 0 else rrdb_bufs(0)[0]
    conv(trunk, H, W, cp, zc + 64, pk.lr_conv, 64, _conv_out(ws.U0, 64, 0, H, W, False, r1=ws.fea, r1_cp=64, s1=1.0),
         nl + 64)
    # the nearest-×2 upconvs (two for ×4, one for ×2), one launch per output phase
    stages = [(ws.U0, H, W, ws.U1, 64, 0), (ws.U1, 2 * H, 2 * W, HR0, hcp, zc)] if sf == 4 else \
        [(ws.U0, H, W, HR0, hcp, zc)]
    for (src, sh, sw, dst, dcp, dcoff), phw, (_, f) in zip(stages, pk.up, up_stages(net)):
        for ph, cw in enumerate(phw):
            py, px = ph // f, ph % f
            ty, tx = _FOLDS[f][py][1], _FOLDS[f][px][1]  # tap origins of the phase's 2×2 LR conv
            o = _conv_out(dst, dcp, dcoff, f * sh, f * sw, True, sy=f, sx=f, oy=py, ox=px)
            ev = None  # reference FLOPs: a 3×3 conv at f× resolution, 1/f² of it per phase
            fl = 2.0 * Bn * (f * sh) * (f * sw) * 9 * 64 * 64 / (f * f)
            nb_ = 4.0 * (2 * Bn * sh * sw * 64 + 4 * 64 * 64)  # its LR source, its quarter of the output, weights
            if rec is not None:
                rec.tag(tagp + 'upconv2x_phase', fl, nb_)
            elif prof is not None:
                ev = _prof_begin(prof, tagp + 'upconv2x_phase', fl, nb_)
            if x3:
                wx, scale = cw.x3()
                if rec is not None:
                    rec.keep.append(wx)
                rc = lib.esr_upconv2x_phase_fwd_x3(src.data_ptr(), Bn, sh, sw, 64, 64, wx.data_ptr(),
                                                   cw.bias_s.data_ptr(), scale, 64, ty, tx, ctypes.byref(o), ovf,
                                                   stream)
            else:
                rc = lib.esr_upconv2x_phase_fwd(src.data_ptr(), Bn, sh, sw, 64, 64, cw.f32.data_ptr(),
                                                cw.bias.data_ptr(), 64, ty, tx, ctypes.byref(o), stream)
            _lib.check(rc, 'esr_upconv2x_phase_fwd')
            if ev is not None:
                ev.record()
    HH, WW = sf * H, sf * W
    gen = torch.empty(Bn, 3, HH, WW, device=dev, dtype=torch.float32)
    if rec is not None:
        rec.keep.append(gen)
    if x3 and train_ws is None and FUSE_HR1:
        # HR_conv0 + HR_conv1 without HR_conv0's activations in memory (esr_hr_convs_x3 / esr_hr1_sum); training keeps
        # them (the backward reads them)
        if ws.Y is None:
            ws.Y = torch.zeros(Bn, HH + 2, WW + 2, 32, device=dev, dtype=torch.float32)  # halo stays zero
        w0x, s0 = pk.hr0.x3()
        w1x, s1 = pk.hr1.x3()
        fl0 = 2.0 * Bn * HH * WW * 9 * (nl + 64) * 64
        fl1 = 2.0 * Bn * HH * WW * 9 * (nl + 64) * 3
        nb0 = 4.0 * (Bn * HH * WW * (zc + 64 + 32) + 9 * (zc + 64) * 64)  # HR0 in, 32 partial products out
        nb1 = 4.0 * Bn * HH * WW * (32 + 3)
        if rec is not None:
            rec.keep += [w0x, w1x]
            rec.tag(tagp + 'hr_conv0_hr1', fl0, nb0)
        ev = _prof_begin(prof, tagp + 'hr_conv0_hr1', fl0, nb0) if rec is None and prof is not None else None
        _lib.check(lib.esr_hr_convs_x3(HR0.data_ptr(), Bn, HH, WW, hcp, zc, w0x.data_ptr(), pk.hr0.bias_s.data_ptr(),
                                       s0, w1x.data_ptr(), ws.Y.data_ptr(), ovf, stream), 'esr_hr_convs_x3')
        if ev is not None:
            ev.record()
        if rec is not None:
            rec.tag(tagp + 'hr1_sum', fl1, nb1)
        ev = _prof_begin(prof, tagp + 'hr1_sum', fl1, nb1) if rec is None and prof is not None else None
        _lib.check(lib.esr_hr1_sum(ws.Y.data_ptr(), Bn, HH, WW, pk.hr1.bias.data_ptr(), 1.0 / (s1 * A),
                                   gen.data_ptr(), stream), 'esr_hr1_sum')
        if ev is not None:
            ev.record()
    else:
        conv(HR0, HH, WW, hcp, hcp, pk.hr0, 64, _conv_out(HR1, hcp, zc, HH, WW, True), nl + 64)
        conv(HR1, HH, WW, hcp, hcp, pk.hr1, 3, _conv_out(gen, 0, 0, HH, WW, False, planar=1), nl + 64)
    if cem is None:
        return gen, ws
    return cem_apply(lib, cem, gen, ws.lr, Bn, H, W, sf * m if pre_pad else 0, stream, sf), ws


def cem_apply(lib, cem, gen, lr, Bn, H, W, M, stream, sf=SF):
    """out = crop_M(gen + Up(Inv(lr - Down(gen))))  ==  CEMnet.py:186-190."""
    dev = gen.device
    ph = cem_phase(sf)
    wd = cem.DownscaleOP.Filter_OP.weight
    wi = cem.Conv_LR_with_Inv_hTh_OP.Filter_OP.weight
    wu = cem.Upscale_OP.Filter_OP.weight
    for t, n in ((wd, 'DownscaleOP'), (wi, 'Conv_LR_with_Inv_hTh_OP'), (wu, 'Upscale_OP')):
        _require_device(t, n + ' filter')
    kd, ki = wd.shape[-1], wi.shape[-1]
    r = torch.empty(Bn, 3, H, W, device=dev, dtype=torch.float32)
    q = torch.empty_like(r)
    if hasattr(lib, 'keep'):  # recording an op list: the intermediates must outlive this call
        lib.keep += [r, q]
    out = torch.empty(Bn, 3, sf * H - 2 * M, sf * W - 2 * M, device=dev, dtype=torch.float32)
    _lib.check(lib.esr_cem_down(gen.data_ptr(), lr.data_ptr(), r.data_ptr(), Bn, H, W, sf, ph,
                                wd[0, 0].contiguous().data_ptr(), kd, 0, stream), 'esr_cem_down')
    _lib.check(lib.esr_cem_inv(r.data_ptr(), q.data_ptr(), Bn, H, W, wi[0, 0].contiguous().data_ptr(), ki, stream),
               'esr_cem_inv')
    _lib.check(lib.esr_cem_up_add(q.data_ptr(), gen.data_ptr(), out.data_ptr(), Bn, H, W, sf, ph,
                                  wu[0, 0].contiguous().data_ptr(), kd, M, stream), 'esr_cem_up_add')
    return out


def cem_filter_op(layer, x):
    """A single CEM Filter_Layer applied on its own (CEMnet.py:139-140), e.g. `netG.module.DownscaleOP(HR)` from the
    GUI (GUI.py:1289,1900).  kind 'down': replicate-pad, xcorr, keep the stride phase (NCHW [B,3,sf*h,sf*w] ->
    [B,3,h,w]); 'inv': replicate-padded xcorr at LR; 'up': zero-stuff ×sf then xcorr ([B,3,h,w] -> [B,3,sf*h,sf*w])."""
    lib = _lib.load()
    _require_device(x, 'CEM filter input')
    if x.dim() != 4 or x.shape[1] != 3:
        raise RuntimeError('esr_amd: CEM filters take [B,3,H,W] input')
    x = x.contiguous()
    w = layer.Filter_OP.weight
    _require_device(w, 'CEM filter weight')
    k = w.shape[-1]
    wk = w[0, 0].contiguous()
    stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    Bn, _, Hx, Wx = x.shape
    sf = getattr(layer, 'sf', SF)
    ph = cem_phase(sf)
    if layer.kind == 'down':
        if Hx % sf or Wx % sf:
            raise RuntimeError('esr_amd: DownscaleOP input size must be divisible by %d' % sf)
        out = torch.empty(Bn, 3, Hx // sf, Wx // sf, device=x.device, dtype=torch.float32)
        _lib.check(lib.esr_cem_down(x.data_ptr(), None, out.data_ptr(), Bn, Hx // sf, Wx // sf, sf, ph,
                                    wk.data_ptr(), k, 1, stream), 'esr_cem_down')
    elif layer.kind == 'inv':
        out = torch.empty_like(x)
        _lib.check(lib.esr_cem_inv(x.data_ptr(), out.data_ptr(), Bn, Hx, Wx, wk.data_ptr(), k, stream), 'esr_cem_inv')
    elif layer.kind == 'up':
        zero = torch.zeros(Bn, 3, sf * Hx, sf * Wx, device=x.device, dtype=torch.float32)
        out = torch.empty_like(zero)
        _lib.check(lib.esr_cem_up_add(x.data_ptr(), zero.data_ptr(), out.data_ptr(), Bn, Hx, Wx, sf, ph,
                                      wk.data_ptr(), k, 0, stream), 'esr_cem_up_add')
    else:
        raise ValueError(layer.kind)
    return out


def set_precision(module, precision):
    """Select 'x3' or 'f32' for every RRDBNet inside `module` (CEM_PyTorch, DataParallel wrappers included)."""
    if precision not in PRECISIONS:
        raise ValueError('precision must be one of %s' % (PRECISIONS,))
    for m in module.modules():
        if hasattr(m, '_esr_cache'):
            m.esr_precision = precision
    return module
