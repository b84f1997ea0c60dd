"""Training (autograd) path of the HIP generator: forward with retained activations + hand-written backward.

`generator_forward` in engine.py routes here whenever autograd needs parameter gradients (the reference's training
step: `fake_H = netG(model_input)` then `l_g_total.backward()`, SRRaGAN_model.py:348, 529).  The whole generator +
CEM is one torch.autograd.Function whose backward runs libesr_amd kernels (exact fp32):

  CEM (train mode)      d gen = g - Down^T Inv^T Up^T g        esr_cem_adjoint ×3 (exact replicate-pad adjoints)
  conv data gradient    esr_conv3x3_fwd with rot180, in/out-swapped packed weights; inside an RDB one conv per
                        concat slice over the stacked output gradients of every conv that reads it (fused K),
                        LeakyReLU backward in its epilogue (the adjoint of the dense concatenations); elsewhere in
                        64-channel output slices
  conv weight gradient  esr_conv3x3_wgrad (split-K over pixel tiles) + esr_wgrad_reduce (deterministic)
  LeakyReLU / residuals esr_lrelu_bwd, esr_axpby;  nearest ×2 adjoint: esr_sum2x2
The reference's residual scales (0.2 in RDB and RRDB, block.py:235, 270) are folded into the packed backward weights
and the reduction scales.
"""
import contextlib
import ctypes
import math
import os
import weakref

import torch

from . import _lib
from . import engine as E

WG_SPLITS_MAX = 128
# The training forward and the backward sweep are ~400 and ~1200 launches per step; after a shape/flag combination has
# run once eagerly, it is captured into a HIP graph and replayed (one launch), with the parameter repack (GatherPlan
# refresh) kept outside the graph.  ESR_TRAIN_GRAPHS=0 keeps everything eager.
USE_GRAPHS = os.environ.get('ESR_TRAIN_GRAPHS', '1') != '0'
# Weight gradients of an x3 forward (split-f16 activations) on the x3 MFMA kernel (esr_conv3x3_wgrad flag 4); 0 keeps
# the exact-fp32 weight-gradient kernel reading the same split activations.
WGRAD_X3 = os.environ.get('ESR_WGRAD_X3', '1') != '0'
# Data gradients inside the residual blocks on the x3 conv (split-f16 gradients scaled per RRDB, include/esr_amd.h
# "x3 backward") when the forward ran in x3 and only parameter gradients are wanted (training); 0 keeps them fp32.
DGRAD_X3 = os.environ.get('ESR_DGRAD_X3', '1') != '0'
# with the x3 backward, also the trunk-level data gradients at 2x / 4x resolution (HR_conv0, the two upconvs) on the x3
# conv, each at its own gradient scale (Runner.dgrad_trunk_x3); '0' keeps them exact fp32
TRUNK_X3 = os.environ.get('ESR_TRUNK_X3', '1') != '0'
# weight gradients on a second stream, overlapping the data-gradient chain they do not feed (each wgrad forks from the
# main stream when its output gradient is ready; the main stream joins before it overwrites a buffer a pending wgrad
# reads).  Opt-in ('1'): on one box, order-balanced, the config-3 step took 159.8 ms with it and 156.3 ms without
# (profiles/r3_ab_stream.txt) — the concurrent kernels share the CUs and each runs longer than the overlap saves.
WGRAD_STREAM = os.environ.get('ESR_WGRAD_STREAM', '0') == '1'
# HR_conv1's data gradient (3 -> 64 channels, 3x3, at HR) on esr_dfirst_fwd_padded (exact fp32 on the VALU; the fp32
# MFMA conv pads its 3 input channels to a 32-wide K step: 0.86 ms at config 3); '0' = the MFMA conv (A/B)
HR1_DFIRST = os.environ.get('ESR_HR1_DFIRST', '1') != '0'
# x3 backward: each RRDB's closing trunk-gradient add also takes the next RRDB's gradient max (esr_axpby_gs_amax: one
# pass over the trunk gradient fewer per RRDB; bitwise the same scale); '0' = a separate esr_grad_amax (A/B)
AMAX_FUSED = os.environ.get('ESR_AMAX_FUSED', '1') != '0'
# SRRaGANModel's training forward with the generator optimiser's flat parameter as its one autograd input (the
# backward returns the flat gradient); '0' = the 702 parameters as inputs (A/B)
FLAT_FWD = os.environ.get('ESR_FLAT_FWD', '1') != '0'
_SIDE = {}


def _side_stream(dev):
    st = _SIDE.get(dev)
    if st is None:
        st = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return st


def _z(dev, *s):
    return torch.zeros(*s, device=dev, dtype=torch.float32)


class DeferredOverflow:
    """The x3 overflow flags of the training forwards / backwards run inside `deferred_overflow_checks()`: instead of
    a blocking 4-byte read right after each forward and backward (which drains the stream and leaves the GPU idle while
    the host enqueues the discriminator's many small kernels), the flags are copied aside on the device and read once,
    by the caller, after the whole training step is enqueued (SRRaGANModel.optimize_parameters, which then redoes the
    step in exact fp32 from a snapshot when one was set)."""

    def __init__(self):
        self.flags = []   # device int32 scalars (activation / gradient overflow, weight out of its scale)
        self.resets = []  # (weight-flag tensor, callback resetting the x3 weight scales)
        self.on_flag = []  # per flag: callback when it is set with no weight flag (forward: lower the activation scale)

    def add(self, overflow, bad, reset, on_overflow=None):
        self.flags.append(overflow.clone())
        self.resets.append((bad.clone(), reset))
        self.on_flag.append(on_overflow)

    def _stacked(self):
        return torch.stack([f.reshape(()).float() for f in self.flags] +
                           [b.reshape(()).float() for b, _ in self.resets])

    def start_read(self):
        """Start the flags' device-to-host copy now, stream-ordered after the work that set them (into pinned memory,
        with an event), so that overflowed() can be asked later — after more work is enqueued — without draining the
        stream.  Single-process only: across ranks overflowed() all-reduces the flags itself."""
        self._host = None
        if self.flags:
            t = self._stacked()
            self._host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
            self._host.copy_(t, non_blocking=True)
            self._event = torch.cuda.Event()
            self._event.record()

    def overflowed(self):
        """True if any deferred forward or backward overflowed (one device-to-host read; all-reduced over ranks)."""
        if not self.flags:
            return False
        if getattr(self, '_host', None) is not None:  # start_read(): wait for that copy only
            self._event.synchronize()
            vals = self._host.tolist()
        else:
            t = self._stacked()
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
                from .SRRaGAN_model import collective
                collective(dist.all_reduce, t, op=dist.ReduceOp.MAX)  # every rank redoes the step together
            vals = t.tolist()
        n = len(self.flags)
        for (_, reset), bad in zip(self.resets, vals[n:]):
            if bad:
                reset()  # new x3 weight scales at the next x3 forward / backward
        for cb, flag, bad in zip(self.on_flag, vals[:n], vals[n:]):
            if cb is not None and flag and not bad:
                cb()
        return any(v != 0 for v in vals)


_DEFERRED = [None]


@contextlib.contextmanager
def deferred_overflow_checks(on=True):
    """Collect (on=True) or check eagerly (on=False) the x3 overflow flags of the training passes in this block."""
    prev = _DEFERRED[0]
    _DEFERRED[0] = DeferredOverflow() if on else None
    try:
        yield _DEFERRED[0]
    finally:
        _DEFERRED[0] = prev


class TrainWorkspace:
    """Buffers of one training forward/backward at (B, H, W).  Same attribute names as engine._Workspace for the
    shared forward code, plus one concat buffer per RDB (`Q`) and the gradient buffers."""

    def __init__(self, dev, B, H, W, latent, nb, sf=4):
        zc = 8 if latent else 0
        self.B, self.H, self.W, self.zc, self.nb, self.sf = B, H, W, zc, nb, sf
        S = sf
        self.first_cp = 16 if latent else 8
        self.first_lr_off = 8 if latent else 0
        self.cp = zc + 192
        self.hr_cp = zc + 64
        self.first = _z(dev, B, H + 2, W + 2, self.first_cp)
        self.fea = _z(dev, B, H + 2, W + 2, 64)
        self.Q = [_z(dev, B, H + 2, W + 2, self.cp) for _ in range(3 * nb + 1)]
        self.U0 = _z(dev, B, H + 2, W + 2, 64)
        self.U1 = _z(dev, B, 2 * H + 2, 2 * W + 2, 64) if sf == 4 else None  # between the two ×2 upconvs of ×4
        self.HR = [_z(dev, B, S * H + 2, S * W + 2, self.hr_cp) for _ in range(2)]
        self.lr = _z(dev, B, 3, H, W)
        self.overflow = torch.zeros(1, device=dev, dtype=torch.int32)
        # backward
        # concat-gradient buffers: [Z | x | d_0 .. d_3 | d_4] with d_i = dL/d(conv i output) (after the LeakyReLU
        # backward) and d_4 = dL/d(RDB output), contiguous so that every slice's data gradient is ONE conv
        self.dcp = zc + 256
        self.D = [_z(dev, B, H + 2, W + 2, self.dcp) for _ in range(2)]
        self.GA = _z(dev, B, H + 2, W + 2, 64)
        self.dU0 = _z(dev, B, H + 2, W + 2, 64)
        self.dU1 = _z(dev, B, 2 * H + 2, 2 * W + 2, 64) if sf == 4 else None
        self.dUp1 = _z(dev, B, 2 * H + 2, 2 * W + 2, 64) if sf == 4 else None
        self.dHR = [_z(dev, B, S * H + 2, S * W + 2, 64) for _ in range(2)]
        self.dgen_p = _z(dev, B, S * H + 2, S * W + 2, 8)
        # generator-input gradient (Z optimisation)
        self.dZl = _z(dev, B, H + 2, W + 2, 8)
        self.dFirst = _z(dev, B, H + 2, W + 2, self.first_cp)
        self.dZh = _z(dev, B, S * H + 2, S * W + 2, 8) if latent else None
        self.dzs = _z(dev, B, H + 2, W + 2, 8) if latent else None  # x3 backward: split latent-slot gradient
        # per-RRDB max |gradient| bits (x3 backward), then one slot per x3 trunk-level data gradient (_trunk_dgrad_x3)
        self.gamax = torch.zeros(nb + 4, device=dev, dtype=torch.int32)
        self.bwd_overflow = torch.zeros(1, device=dev, dtype=torch.int32)
        self.wg_n_max = 9 * 224 * 64 + 64
        self.partial = torch.empty(WG_SPLITS_MAX * self.wg_n_max, device=dev, dtype=torch.float32)
        self.graphs = {}


class _Owner:
    """Held by the autograd context of one training forward; the workspace keeps a weak reference to it.  While it is
    alive and its backward has not run, the workspace's saved activations belong to that forward."""
    __slots__ = ('done', '__weakref__')

    def __init__(self):
        self.done = False


def _busy(ws):
    o = ws.owner() if getattr(ws, 'owner', None) is not None else None
    return o is not None and not o.done


def _train_workspace(net, dev, B, H, W, latent, precision='f32'):
    """The cached workspace of this shape, or — when its saved activations still await a backward (a second grad
    forward before the first one's backward: two generator calls in one loss, retained graphs) — a fresh one, so that
    no forward overwrites another's activations."""
    # keyed by precision too: an x3 forward leaves split-f16 records where an fp32 forward expects floats
    sf = getattr(net, 'upscale', E.SF)
    key = (str(dev), B, H, W, latent, net.nb, precision, sf)
    c = net._esr_cache.get('train_ws')
    if c is None or c[0] != key:
        if c is not None and _busy(c[1]):
            return TrainWorkspace(dev, B, H, W, latent, net.nb, sf)  # the cached one is still needed: keep it
        net._esr_cache.pop('train_ws', None)
        c = (key, TrainWorkspace(dev, B, H, W, latent, net.nb, sf))
        net._esr_cache['train_ws'] = c
    if _busy(c[1]):
        return TrainWorkspace(dev, B, H, W, latent, net.nb, sf)
    return c[1]


# ----------------------------------------------------------------------------------------------------------------------
# backward weight packing
# ----------------------------------------------------------------------------------------------------------------------
class _BwdConv:
    """Backward data of one conv: the forward-buffer channel map, dgrad weight slices (GatherPlan index images until
    finalised) and the location of its weight gradient in the flat wgrad buffer."""

    def __init__(self, plan, conv, cmap, scale=1.0, cin_k=None, dgrad_from=0, in_width=0):
        w = plan.w(conv.weight)
        cout, cin_ref = w.shape[:2]
        self.conv, self.cout, self.cmap, self.cin_buf = conv, cout, list(cmap), len(cmap)
        wf = w.flip(2, 3).transpose(0, 1)  # [Cin_ref][Cout][3][3]: rot180, swapped
        k = cin_k if cin_k is not None else cout  # channels of the gradient the dgrad reads (padded to 8)
        kmap = list(range(cout)) + [-1] * (k - cout)
        def dslice(n0, nw):
            rows = torch.tensor(self.cmap[n0:n0 + nw])
            wt = torch.zeros(nw, cout, 3, 3, dtype=w.dtype)
            wt[rows >= 0] = wf[rows[rows >= 0]]
            return n0, nw, plan.reg(E.pack_conv_weight(plan.scaled(wt, scale), kmap, 32 if nw <= 32 else 64))

        self.wf = wf
        self.slices = []  # (first buffer channel, width, packed weights)
        n0 = dgrad_from  # input-gradient channels below this (the latent Z slot) are not needed
        while n0 < self.cin_buf:
            nw = min(64, self.cin_buf - n0)
            self.slices.append(dslice(n0, nw))
            n0 += nw
        # generator-input gradient (Z optimisation): the channels below dgrad_from (latent Z slot / conv_first input)
        self.in_slices = [dslice(0, in_width)] if in_width else []
        self.ref_to_buf = [self.cmap.index(r) for r in range(cin_ref)]
        self.cin_pad = (self.cin_buf + 31) // 32 * 32
        self.cout_pad = 32 if cout <= 32 else 64
        self.wg_n = 9 * self.cin_pad * self.cout_pad + self.cout_pad
        self.wg_off = 0

    def grad_index(self):
        """Positions in this conv's wgrad region ([9][cin_pad][cout_pad] + bias[cout_pad]) of the reference-layout
        weight [Cout][Cin_ref][3][3] and bias [Cout]."""
        co = torch.arange(self.cout).view(-1, 1, 1)
        ci = torch.tensor(self.ref_to_buf).view(1, -1, 1)
        tap = torch.arange(9).view(1, 1, 9)
        wi = self.wg_off + (tap * self.cin_pad + ci) * self.cout_pad + co
        bi = self.wg_off + 9 * self.cin_pad * self.cout_pad + torch.arange(self.cout)
        return wi.reshape(-1), bi


class _BwdPacked:
    def __init__(self, net, latent):
        def lr_map(n):
            return list(range(n)) if not latent else [0, 1, 2] + [-1] * 5 + [3 + c for c in range(n)]
        m = net.model
        zc = 8 if latent else 0
        plan = self.plan = E.GatherPlan(E.param_list(net), scales=(1.0, 0.2))
        first_map = ([0, 1, 2] + [-1] * 5 + [3, 4, 5] + [-1] * 5) if latent else ([0, 1, 2] + [-1] * 5)
        self.first = _BwdConv(plan, m[0], first_map, dgrad_from=len(first_map), in_width=len(first_map))
        self.rdb, self.rdb_fused = [], []
        for k in range(net.nb):
            rr = m[1].sub[k]
            for rdb in (rr.RDB1, rr.RDB2, rr.RDB3):
                cv = [_BwdConv(plan, rdb.convs[i][0], lr_map(64 + 32 * i), 0.2 if i == 4 else 1.0,
                               dgrad_from=zc + 64 + 32 * i) for i in range(5)]  # data gradient: fused below
                self.rdb.append(cv)
                self.rdb_fused.append(_fused_rdb_weights(plan, cv, zc))
        self.lr_conv = _BwdConv(plan, m[1].sub[net.nb], lr_map(64), dgrad_from=zc, in_width=zc)
        n_up = getattr(net, 'n_up', 2)  # ×4: two nearest-×2 upconvs (model.2, model.3), ×2: one (architecture.py:132)
        self.up = [_BwdConv(plan, m[2 + j][1], list(range(64))) for j in range(n_up)]
        self.hr0 = _BwdConv(plan, m[2 + n_up], lr_map(64), dgrad_from=zc, in_width=zc)
        self.hr1 = _BwdConv(plan, m[4 + n_up], lr_map(64), cin_k=8, dgrad_from=zc, in_width=zc)
        convs = [self.first, self.lr_conv, self.hr0, self.hr1] + self.up + [c for r in self.rdb for c in r]
        dev = m[0].weight.device
        views = plan.finalize(dev)
        off = 0
        for c in convs:
            c.slices = [(n0, nw, views[id(t)]) for n0, nw, t in c.slices]
            c.in_slices = [(n0, nw, views[id(t)]) for n0, nw, t in c.in_slices]
            c.wf = None
            c.wg_off = off
            off += c.wg_n
        self.rdb_fused = [{k: views[id(t)] for k, t in f.items()} for f in self.rdb_fused]
        self.zero_bias = torch.zeros(64, device=dev)
        self.dw = torch.empty(off, device=dev, dtype=torch.float32)  # every conv's reduced wgrad, packed layout
        by_param = {}
        for c in convs:
            wi, bi = c.grad_index()
            by_param[id(c.conv.weight)], by_param[id(c.conv.bias)] = wi, bi
        self.params = plan.params
        assert all(id(p) in by_param for p in self.params), 'generator parameter without a backward rule'
        self.gidx = torch.cat([by_param[id(p)] for p in self.params]).to(dev)
        # flat-gradient offsets (reference parameter order) where the backward has finalised a suffix of the flat
        # gradient: after LR_conv (the convs behind it are done too), after each RRDB (last to first); 0 = all
        off, o = {}, 0
        for p in self.params:
            off[id(p)] = o
            o += p.numel()
        self.flat_n = o
        self.lr_conv_lo = off[id(m[1].sub[net.nb].weight)]
        self.rrdb_lo = [off[id(m[1].sub[k].RDB1.convs[0][0].weight)] for k in range(net.nb)]
        self._x3 = None

    def x3_fused(self):
        """The fused RDB data-gradient weights in the x3 layout (engine.pack_x3: [chunk16][tap][n][2 × (hi 8 | lo 8)]),
        rebuilt in place with one gather after every refresh of the fp32 packs.  Each weight keeps the power-of-two
        scale chosen at the first build (one host sync, then none: captured graphs stay valid); returns
        ([{target: (x3 tensor, scale)}] per RDB, device int32 flag = a weight left its scale's safe range)."""
        buf = self.plan.buf
        if self._x3 is None:
            views = [(i, k, v) for i, f in enumerate(self.rdb_fused) for k, v in f.items()]
            # the trunk-level data gradients at 2x / 4x resolution (HR_conv0, both upconvs): slices and, for
            # HR_conv0, the latent-slot (input) slice; keyed (conv, kind, slice index) in self._x3_trunk
            tconvs = (('hr0', self.hr0),) + ((('up1', self.up[1]),) if len(self.up) > 1 else ()) + \
                (('up0', self.up[0]),)
            trunk = [(name, kind, j, v) for name, c in tconvs
                     for kind, sl in (('s', c.slices), ('in', c.in_slices)) for j, (_, _, v) in enumerate(sl)]
            views += [(None, (name, kind, j), v) for name, kind, j, v in trunk]
            amax = torch.stack([v.abs().max() for _, _, v in views]).cpu().tolist()  # first build only
            idx, scl, out, off = [], [], [], 0
            for (i, k, v), a in zip(views, amax):
                n32, T, n_pad, _ = v.shape
                sc = 1.0 if a == 0.0 else 2.0 ** (14 - math.floor(math.log2(a)))
                pos = torch.arange(v.numel(), device=buf.device) + v.storage_offset()
                idx.append(pos.view(n32, T, n_pad, 2, 16).permute(0, 3, 1, 2, 4).reshape(-1))
                scl.append(torch.full((v.numel(),), sc, device=buf.device))
                out.append((i, k, off, v.numel(), sc))
                off += 2 * v.numel()
            self._x3_idx, self._x3_scl = torch.cat(idx), torch.cat(scl)
            self._x3_buf = torch.empty(off, device=buf.device, dtype=torch.float16)
            self._x3_w = [dict() for _ in self.rdb_fused]
            self._x3_trunk = {}
            for i, k, o, n, sc in out:
                (self._x3_trunk if i is None else self._x3_w[i])[k] = (self._x3_buf[o:o + 2 * n], sc)
            self._x3_bad = torch.zeros(1, device=buf.device, dtype=torch.int32)
            self._x3 = 'stale'
        if self._x3 == 'stale':
            g = buf[self._x3_idx] * self._x3_scl
            hi = g.half()
            lo = (g - hi.float()).half()
            G = g.numel() // 8
            self._x3_buf.view(G, 2, 8).copy_(torch.stack([hi.view(G, 8), lo.view(G, 8)], 1))
            self._x3_bad.copy_((g.abs().amax() >= 61440.0).to(torch.int32).view(1))
            self._x3 = 'fresh'
        return self._x3_w, self._x3_bad

    def reset_x3(self):
        self._x3 = None


def _fused_rdb_weights(plan, convs, zc):
    """Data-gradient weights of one RDB in the fused form: the gradient of concat slice t (buffer channels
    [t0, t0+nw)) is  sum over the convs i that read t of conv_i^T(d_i),  one conv over the contiguous d_i channels
    [d_lo, zc+256) of the concat-gradient buffer with the rot180/transposed weights of those convs stacked along K
    (conv 4 scaled by its 0.2 residual factor).  Targets: 'm1'..'m4' = x_1..x_4 (32 channels, from d_m..d_4),
    'x' = the block input (64 channels, from d_0..d_4), 'z' = the latent slot (zc channels, from d_0..d_4)."""
    def slice_w(t0, nw, i_lo):
        blocks = []
        for i in range(i_lo, 5):
            c = convs[i]
            blk = torch.zeros(nw, c.cout, 3, 3, dtype=c.wf.dtype)
            for r in range(nw):
                t = t0 + r
                if t < len(c.cmap) and c.cmap[t] >= 0:
                    blk[r] = c.wf[c.cmap[t]]
            blocks.append(plan.scaled(blk, 0.2) if i == 4 else blk)
        wt = torch.cat(blocks, 1)
        return plan.reg(E.pack_conv_weight(wt, list(range(wt.shape[1])), 32 if nw <= 32 else 64))
    out = {'m%d' % m: slice_w(zc + 64 + 32 * (m - 1), 32, m) for m in (1, 2, 3, 4)}
    out['x'] = slice_w(zc, 64, 0)
    if zc:
        out['z'] = slice_w(0, zc, 0)
    return out


def _bwd_packed(net, latent):
    sk, vkey = E._keys(net)
    skey = (sk, latent)
    c = net._esr_cache.get('packed_bwd')
    if c is None or c[0] != skey:
        net._esr_cache.pop('packed_bwd', None)
        with torch.no_grad():
            c = [skey, None, _BwdPacked(net, latent)]
        net._esr_cache['packed_bwd'] = c
    if c[1] != vkey:
        with torch.no_grad():
            c[2].plan.refresh()
        if c[2]._x3 is not None:
            c[2]._x3 = 'stale'
        c[1] = vkey
    return c[2]


# ----------------------------------------------------------------------------------------------------------------------
# backward sweep
# ----------------------------------------------------------------------------------------------------------------------
class _Runner:
    def __init__(self, ws, bp, stream, need_params=True, need_input=False, split=False):
        self.lib = _lib.load()
        self.ws = ws
        self.bp = bp
        self.B = ws.B
        self.stream = stream
        self.need_params, self.need_input = need_params, need_input
        self.split = split  # forward activations in the split-f16 layout (x3 forward)
        self.x3 = None  # x3 backward: (per-RDB x3 fused weights, gradient-amax buffer, overflow flag)
        self.act_scale = 1.0
        self.side = None  # WGRAD_STREAM: (main torch stream, side torch stream, side stream handle)

    def use_side_stream(self, dev):
        main = torch.cuda.current_stream(dev)
        side = _side_stream(dev)
        self.side = (main, side, ctypes.c_void_p(side.cuda_stream))

    def join(self):
        """The main stream waits for every weight gradient issued so far (before it overwrites what they read)."""
        if self.side is not None:
            self.side[0].wait_stream(self.side[1])

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
                                                self.bp.zero_bias.data_ptr(), nw, ctypes.byref(o), self.stream),
                       'dgrad')

    def dgrad_fused(self, wpk, src, src_cp, src_coff, cin_k, h, w, dst, dst_cp, dst_coff, nw, res=None, mask=None):
        """dst[:, dst_coff:+nw] = conv(src channels [src_coff, +cin_k), fused weights) (+ res) (then LeakyReLU
        backward through the saved activation `mask` = (buf, cp, coff)); res = (buf, cp, coff) or 'acc'."""
        r1, r1_cp, r1_coff = (None, 0, 0)
        if res == 'acc':
            r1, r1_cp, r1_coff = dst, dst_cp, dst_coff
        elif res is not None:
            r1, r1_cp, r1_coff = res
        r2, r2_cp, r2_coff = mask if mask is not None else (None, 0, 0)
        o = E._conv_out(dst, dst_cp, dst_coff, h, w, (3 if self.split else 2) if mask is not None else 0, r1=r1, r1_cp=r1_cp,
                        r1_coff=r1_coff, s1=1.0, r2=r2, r2_cp=r2_cp, r2_coff=r2_coff)
        _lib.check(self.lib.esr_conv3x3_fwd(src.data_ptr() + 4 * src_coff, self.B, h, w, src_cp, cin_k, wpk.data_ptr(),
                                            self.bp.zero_bias.data_ptr(), nw, ctypes.byref(o), self.stream),
                   'dgrad_fused')

    def dgrad_in(self, bc, src, src_cp, src_coff, cin_k, h, w, dst, dst_cp):
        """Generator-input gradient: dst[:, 0:nw] += conv(src slice, rot180 W^T) restricted to the input channels
        below the feature channels (latent Z slot; conv_first's [Z | LR] input)."""
        if not self.need_input:
            return
        for n0, nw, wpk in bc.in_slices:
            o = E._conv_out(dst, dst_cp, 0, h, w, False, r1=dst, r1_cp=dst_cp, r1_coff=0, s1=1.0)
            _lib.check(self.lib.esr_conv3x3_fwd(src.data_ptr() + 4 * src_coff, self.B, h, w, src_cp, cin_k,
                                                wpk.data_ptr(), self.bp.zero_bias.data_ptr(), nw, ctypes.byref(o),
                                                self.stream), 'dgrad_in')

    def wgrad(self, bc, inp, in_cp, cin, up2, dout, d_cp, d_coff, h, w, scale=1.0, amax=None):
        """Weight + bias gradient of one conv into its region of the flat packed-layout buffer bp.dw.  `amax` (a
        device pointer): the output gradient is split-f16, scaled by the gradient scale of that amax."""
        if not self.need_params:
            return
        assert cin == bc.cin_buf
        chunks = bc.cin_pad // 32
        ntiles = self.B * ((h + 7) // 8) * ((w + 31) // 32)
        x3 = self.split and (WGRAD_X3 or amax is not None)
        # split-K: the fp32 kernel at ~4 workgroups per CU; the x3 kernel (one 12-wave workgroup per CU) at ~1 — more
        # splits only add partial traffic for the reduction (tools/wgrad_ab.py)
        splits = max(1, min(WG_SPLITS_MAX, (256 // chunks) if x3 else -(-1024 // chunks), ntiles))
        assert splits * bc.wg_n <= self.ws.partial.numel()
        flags = up2 | ((6 if x3 else 2) if self.split else 0) | (8 if amax is not None else 0)
        st = self.stream
        if self.side is not None:  # fork: the side stream sees everything issued on the main stream so far
            self.side[1].wait_stream(self.side[0])
            st = self.side[2]
        _lib.check(self.lib.esr_conv3x3_wgrad(inp.data_ptr(), in_cp, cin, flags, dout.data_ptr(), d_cp, d_coff,
                                              bc.cout, self.B, h, w, splits, self.ws.partial.data_ptr(), st),
                   'wgrad')
        dst = self.bp.dw.data_ptr() + 4 * bc.wg_off
        A = self.act_scale if self.split else 1.0
        if A != 1.0:  # weights part x 1/A (the split activations hold A·v); the bias gradients do not read them
            _lib.check(self.lib.esr_wgrad_reduce2(self.ws.partial.data_ptr(), splits, bc.wg_n, bc.wg_n - bc.cout_pad,
                                                  scale / A, scale, amax, dst, st), 'wgrad_reduce2')
        elif amax is None:
            _lib.check(self.lib.esr_wgrad_reduce(self.ws.partial.data_ptr(), splits, bc.wg_n, scale, dst, st),
                       'wgrad_reduce')
        else:
            _lib.check(self.lib.esr_wgrad_reduce_gs(self.ws.partial.data_ptr(), splits, bc.wg_n, scale, amax, dst,
                                                    st), 'wgrad_reduce_gs')

    def dgrad_x3(self, wx, src, src_cp, src_coff, cin_k, h, w, dst, dst_cp, dst_coff, nw, res=None, mask=None):
        """dgrad_fused on the x3 conv: src / dst / res are split-f16 gradients at one scale (the conv is linear, so
        the scale passes through); the LeakyReLU backward reads the saved split activation `mask`."""
        wpk, w_scale = wx
        r1, r1_cp, r1_coff = res if res is not None else (None, 0, 0)
        r2, r2_cp, r2_coff = mask if mask is not None else (None, 0, 0)
        o = E._conv_out(dst, dst_cp, dst_coff, h, w, 3 if mask is not None else 0, r1=r1, r1_cp=r1_cp,
                        r1_coff=r1_coff, s1=1.0, r2=r2, r2_cp=r2_cp, r2_coff=r2_coff)
        _lib.check(self.lib.esr_conv3x3_fwd_x3(src.data_ptr() + 4 * src_coff, self.B, h, w, src_cp, cin_k,
                                               wpk.data_ptr(), self.bp.zero_bias.data_ptr(), w_scale, nw,
                                               ctypes.byref(o), self.x3[2].data_ptr(), self.stream), 'dgrad_x3')

    def dgrad_trunk_x3(self, name, bc, src, h, w, dst, dst_base, s_in, s_out, slot, dz=None):
        """dst[:, 0:64] (fp32) = the data gradient of trunk conv `name` from its fp32 64-channel output gradient
        `src`, on the x3 conv: src -> split × S(max |src|) into s_in, the conv into s_out (split, the same scale: the
        conv is linear), back to fp32 into dst.  s_in / s_out: padded 64-channel buffers of this grid that are free
        here (zero halos; s_in may be dst, s_out may be src).  dz = (fp32 buffer, pitch, 8-channel split scratch):
        also the input-slice (latent slot) gradient, accumulated into the buffer.  Gradient-scale slot `slot` of
        ws.gamax; an f16-range overflow sets ws.bwd_overflow (the backward is then redone in fp32)."""
        lib, ws, B = self.lib, self.ws, self.B
        amax = ws.gamax.data_ptr() + 4 * slot
        ovf = ws.bwd_overflow.data_ptr()
        _lib.check(lib.esr_grad_amax(src.data_ptr(), 64, 0, 64, B, h, w, amax, self.stream), 'grad_amax')
        _lib.check(lib.esr_axpby_gs(s_in.data_ptr(), 64, 0, 1, 1.0, src.data_ptr(), 64, 0, 0, 0.0, None, 0, 0, 0, 64,
                                    B, h, w, amax, ovf, self.stream), 'axpby_gs')
        tw = self.bp._x3_trunk
        if dz is not None and self.need_input:
            zbuf, z_cp, zscr = dz
            for j, (n0, nw, _) in enumerate(bc.in_slices):
                self.dgrad_x3(tw[(name, 'in', j)], s_in, 64, 0, 64, h, w, zscr, 8, n0, nw)
            _lib.check(lib.esr_axpby_gs(zbuf.data_ptr(), z_cp, 0, 0, 1.0, zbuf.data_ptr(), z_cp, 0, 0, 1.0,
                                        zscr.data_ptr(), 8, 0, 1, 8, B, h, w, amax, ovf, self.stream), 'axpby_gs')
        for j, (n0, nw, _) in enumerate(bc.slices):
            self.dgrad_x3(tw[(name, 's', j)], s_in, 64, 0, 64, h, w, s_out, 64, n0 - dst_base, nw)
        _lib.check(lib.esr_axpby_gs(dst.data_ptr(), 64, 0, 0, 1.0, s_out.data_ptr(), 64, 0, 1, 0.0, None, 0, 0, 0, 64,
                                    B, h, w, amax, ovf, self.stream), 'axpby_gs')

    def lrelu(self, d, d_cp, d_coff, y, y_cp, y_coff, C, h, w):
        fn = self.lib.esr_lrelu_bwd_split if self.split else self.lib.esr_lrelu_bwd
        _lib.check(fn(d.data_ptr(), d_cp, d_coff, y.data_ptr(), y_cp, y_coff, C, self.B, h, w, self.stream),
                   'lrelu_bwd')

    def axpby(self, out, o_cp, o_coff, a, x1, x1_cp, x1_coff, b=0.0, x2=None, x2_cp=0, x2_coff=0, C=64, h=0, w=0):
        _lib.check(self.lib.esr_axpby(out.data_ptr(), o_cp, o_coff, a, x1.data_ptr(), x1_cp, x1_coff, b,
                                      None if x2 is None else x2.data_ptr(), x2_cp, x2_coff, C, self.B, h, w,
                                      self.stream), 'axpby')


def _rdb_backward_x3(R, P, dcat, convs, fx3, zc, cp, H, W, dx, amax, z_first=False):
    """_rdb_backward with the concat-gradient buffers in the split-f16 layout at gradient scale S(amax): the fused
    data-gradient convs on the x3 conv, the weight gradients on the x3 kernel reading the split gradients.  The latent
    slot's gradient (Z optimisation) is summed over the RRDB's three blocks in the split scratch ws.dzs (z_first: this
    block starts the sum)."""
    dcp = R.ws.dcp
    d4 = zc + 192
    R.wgrad(convs[4], P, cp, zc + 192, 0, dcat, dcp, d4, H, W, scale=0.2, amax=amax)
    for m in (4, 3, 2, 1):
        s_in, t = zc + 64 + 32 * m, zc + 64 + 32 * (m - 1)
        R.dgrad_x3(fx3['m%d' % m], dcat, dcp, s_in, zc + 256 - s_in, H, W, dcat, dcp, t, 32, mask=(P, cp, t))
        R.wgrad(convs[m - 1], P, cp, t, 0, dcat, dcp, t, H, W, amax=amax)
    if R.need_input and zc:
        R.dgrad_x3(fx3['z'], dcat, dcp, zc + 64, 192, H, W, R.ws.dzs, 8, 0, zc,
                   res=None if z_first else (R.ws.dzs, 8, 0))
    R.join()  # dx's buffer is the previous block's concat gradient, which its pending weight gradients read
    R.dgrad_x3(fx3['x'], dcat, dcp, zc + 64, 192, H, W, dx[0], dx[1], dx[2], 64, res=(dcat, dcp, d4))


def _rdb_backward(R, P, dcat, convs, fused, zc, cp, H, W, dx):
    """One ResidualDenseBlock_5C (block.py:230-235): h = 0.2·conv4(cat) + x, cat = [x, x1..x4], x_{i+1} =
    lrelu(conv_i(cat_{<=i})).  On entry dcat[zc+192 : zc+256) = d_4 = dL/dh.  For m = 4..1 one fused conv computes
    dL/dx_m from d_m..d_4 and its epilogue applies the LeakyReLU backward, giving d_{m-1} in place; then one conv gives
    dL/dx (+ d_4 through the residual) into dx = (buffer, pitch, offset)."""
    dcp = R.ws.dcp
    d4 = zc + 192
    R.wgrad(convs[4], P, cp, zc + 192, 0, dcat, dcp, d4, H, W, scale=0.2)
    for m in (4, 3, 2, 1):
        s_in, t = zc + 64 + 32 * m, zc + 64 + 32 * (m - 1)
        R.dgrad_fused(fused['m%d' % m], dcat, dcp, s_in, zc + 256 - s_in, H, W, dcat, dcp, t, 32, mask=(P, cp, t))
        R.wgrad(convs[m - 1], P, cp, t, 0, dcat, dcp, t, H, W)
    if R.need_input and zc:
        R.dgrad_fused(fused['z'], dcat, dcp, zc + 64, 192, H, W, R.ws.dZl, 8, 0, zc, res='acc')
    R.join()  # dx's buffer is the previous block's concat gradient, which its pending weight gradients read
    R.dgrad_fused(fused['x'], dcat, dcp, zc + 64, 192, H, W, dx[0], dx[1], dx[2], 64, res=(dcat, dcp, d4))


def generator_backward(net, cem, ws, d_out, latent, M, need_params=True, need_input=False, split=False, x3=False,
                       act_scale=1.0):
    """dL/dparams of RRDBNet (+ CEM in train or eval mode) and/or dL/dinput given dL/dout.  x3 (with split, params
    only): the residual blocks' backward in the split-f16 scheme; ws.bwd_overflow then tells whether a scaled gradient
    or a weight left its f16 range (the caller reruns without x3).
    Returns (flat parameter gradient in the reference layout or None, input gradient [B, C_in, h, w] or None)."""
    it = backward_segments(net, cem, ws, d_out, latent, M, need_params, need_input, split, x3, act_scale)
    while True:
        try:
            next(it)
        except StopIteration as e:
            return e.value


def _emit_points(bp, lows):
    """The segment boundaries of a sliced backward: for each bucket's lower end `lo` (GradBuckets.emit_offsets), the
    first point of the backward at which flat[lo:] is final — after LR_conv (with the convs behind it), after RRDB k
    (last to first) — so that every bucket launches as early as the backward allows.  0 (conv_first) is the end."""
    cands = [bp.lr_conv_lo] + [bp.rrdb_lo[k] for k in reversed(range(len(bp.rrdb_lo)))]
    pts = set()
    for lo in lows:
        p = next((c for c in cands if c <= lo), 0)
        if p > 0:
            pts.add(p)
    return pts


def backward_segments(net, cem, ws, d_out, latent, M, need_params=True, need_input=False, split=False, x3=False,
                      act_scale=1.0, seg=None):
    """generator_backward as a generator.  With seg = (flat_grad, lows) (parameter gradients only): the weight
    gradients go straight into flat_grad (+=, reference layout) in slices — at each boundary of _emit_points(lows)
    the finished suffix flat_grad[lo:hi] gets its gather-add and the generator yields lo (the caller launches the
    all-reduces of the buckets now complete while the rest is enqueued); the returned flat gradient is then None and
    the last slice [0, hi) is added before returning."""
    dev = d_out.device
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    bp = _bwd_packed(net, latent)
    R = _Runner(ws, bp, stream, need_params, need_input, split)
    R.act_scale = act_scale  # the forward's split activations hold A·v: weight gradients read them (x 1/A)
    if WGRAD_STREAM and need_params:
        R.use_side_stream(dev)
    lib = R.lib
    if x3:
        assert split and (need_params or need_input)
        fx3, bad = bp.x3_fused()
        ws.gamax.zero_()
        ws.bwd_overflow.copy_(bad)
        R.x3 = (fx3, ws.gamax, ws.bwd_overflow)
    if need_input:
        ws.dZl.zero_()
        ws.dFirst.zero_()
        if latent:
            ws.dZh.zero_()
    Bn, H, W, zc, cp, hcp = ws.B, ws.H, ws.W, ws.zc, ws.cp, ws.hr_cp
    sf = ws.sf
    ph = E.cem_phase(sf)
    HH, WW = sf * H, sf * W
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
        _lib.check(lib.esr_cem_adjoint(gfull.data_ptr(), Bn * 3, HH, WW, wu.data_ptr(), kd, 1, 0, HH, WW, sf,
                                       ph, 1.0, 0, a1.data_ptr(), stream), 'cem_adjoint up')
        _lib.check(lib.esr_cem_adjoint(a1.data_ptr(), Bn * 3, H, W, wi.data_ptr(), ki, 1, 0, H, W, 1, 0, 1.0, 0,
                                       a2.data_ptr(), stream), 'cem_adjoint inv')
        dgen = gfull.clone()
        _lib.check(lib.esr_cem_adjoint(a2.data_ptr(), Bn * 3, H, W, wd.data_ptr(), kd, sf, ph, HH, WW, 1,
                                       0, -1.0, 1, dgen.data_ptr(), stream), 'cem_adjoint down')
    else:
        dgen = d_out.contiguous()
    _lib.check(lib.esr_nchw_to_padded(dgen.data_ptr(), 3, Bn, HH, WW, ws.dgen_p.data_ptr(), 8, 0, 0, stream),
               'nchw_to_padded')
    HR0, HR1 = ws.HR
    dA, dB = ws.dHR
    # HR_conv1 (no act): input HR1 = [Z_HR | x]
    R.wgrad(bp.hr1, HR1, hcp, hcp, 0, ws.dgen_p, 8, 0, HH, WW)
    R.dgrad_in(bp.hr1, ws.dgen_p, 8, 0, 8, HH, WW, ws.dZh, 8)
    if HR1_DFIRST:  # the 3 -> 64 data gradient on the VALU kernel of the D's first conv (flipped, transposed weights)
        wt = bp.hr1.conv.weight[:, -64:].detach().flip(2, 3).permute(1, 0, 2, 3).contiguous()
        _lib.check(lib.esr_dfirst_fwd_padded(ws.dgen_p.data_ptr(), 8, Bn, HH, WW, wt.data_ptr(), None, 0.0, 0,
                                             dA.data_ptr(), 64, 0, stream), 'hr1 data gradient')
    else:
        R.dgrad(bp.hr1, ws.dgen_p, 8, 0, 8, HH, WW, dA, 64, zc, accumulate=False)
    # HR_conv0 + LReLU: output HR1.x
    R.lrelu(dA, 64, 0, HR1, hcp, zc, 64, HH, WW)
    R.wgrad(bp.hr0, HR0, hcp, hcp, 0, dA, 64, 0, HH, WW)
    # the trunk-level data gradients at 2x / 4x on the x3 conv when the backward is x3 (TRUNK_X3), else exact fp32
    tx3 = x3 and TRUNK_X3
    R.join()  # (each trunk data gradient below overwrites buffers that the weight gradient before it reads)
    if tx3:
        R.dgrad_trunk_x3('hr0', bp.hr0, dA, HH, WW, dB, zc, dB, dA, net.nb, dz=(ws.dZh, 8, ws.dgen_p) if zc else None)
    else:
        R.dgrad_in(bp.hr0, dA, 64, 0, 64, HH, WW, ws.dZh, 8)
        R.dgrad(bp.hr0, dA, 64, 0, 64, HH, WW, dB, 64, zc, accumulate=False)
    if sf == 4:
        # upconv 2: HR0.x = lrelu(conv(nearest2(U1)))
        R.lrelu(dB, 64, 0, HR0, hcp, zc, 64, HH, WW)
        R.wgrad(bp.up[1], ws.U1, 64, 64, 1, dB, 64, 0, HH, WW)
        R.join()
        if tx3:
            R.dgrad_trunk_x3('up1', bp.up[1], dB, HH, WW, dA, 0, dA, dB, net.nb + 1)
        else:
            R.dgrad(bp.up[1], dB, 64, 0, 64, HH, WW, dA, 64, 0, accumulate=False)
        _lib.check(lib.esr_sum2x2(ws.dU1.data_ptr(), 64, 0, dA.data_ptr(), 64, 0, 64, Bn, 2 * H, 2 * W, stream),
                   'sum2x2')
        # upconv 1: U1 = lrelu(conv(nearest2(U0)))
        R.lrelu(ws.dU1, 64, 0, ws.U1, 64, 0, 64, 2 * H, 2 * W)
        R.wgrad(bp.up[0], ws.U0, 64, 64, 1, ws.dU1, 64, 0, 2 * H, 2 * W)
        R.join()
        if tx3:
            R.dgrad_trunk_x3('up0', bp.up[0], ws.dU1, 2 * H, 2 * W, ws.dUp1, 0, ws.dUp1, ws.dU1, net.nb + 2)
        else:
            R.dgrad(bp.up[0], ws.dU1, 64, 0, 64, 2 * H, 2 * W, ws.dUp1, 64, 0, accumulate=False)
        _lib.check(lib.esr_sum2x2(ws.dU0.data_ptr(), 64, 0, ws.dUp1.data_ptr(), 64, 0, 64, Bn, H, W, stream),
                   'sum2x2')
    else:
        # ×2: the one upconv, HR0.x = lrelu(conv(nearest2(U0))) (architecture.py:132-136)
        R.lrelu(dB, 64, 0, HR0, hcp, zc, 64, HH, WW)
        R.wgrad(bp.up[0], ws.U0, 64, 64, 1, dB, 64, 0, HH, WW)
        R.join()
        if tx3:
            R.dgrad_trunk_x3('up0', bp.up[0], dB, HH, WW, dA, 0, dA, dB, net.nb + 2)
        else:
            R.dgrad(bp.up[0], dB, 64, 0, 64, HH, WW, dA, 64, 0, accumulate=False)
        _lib.check(lib.esr_sum2x2(ws.dU0.data_ptr(), 64, 0, dA.data_ptr(), 64, 0, 64, Bn, H, W, stream), 'sum2x2')
    # LR_conv: U0 = conv(trunk[Z | x]) + fea
    Q = ws.Q
    trunk = Q[3 * net.nb]
    R.wgrad(bp.lr_conv, trunk, cp, zc + 64, 0, ws.dU0, 64, 0, H, W)
    R.dgrad_in(bp.lr_conv, ws.dU0, 64, 0, 64, H, W, ws.dZl, 8)
    R.dgrad(bp.lr_conv, ws.dU0, 64, 0, 64, H, W, ws.GA, 64, zc, accumulate=False)
    pts, hi = (_emit_points(bp, seg[1]), [bp.flat_n]) if seg is not None else (set(), [0])

    def slice_to(lo):  # the finished suffix's weight gradients into the flat gradient, reference layout
        R.join()
        seg[0][lo:hi[0]].add_(bp.dw.index_select(0, bp.gidx[lo:hi[0]]))
        hi[0] = lo
        return lo
    if bp.lr_conv_lo in pts:
        yield slice_to(bp.lr_conv_lo)
    # RRDBs, last to first: o = 0.2·RDB3(RDB2(RDB1(x))) + x
    D0, D1 = ws.D
    dcp, d4 = ws.dcp, zc + 192
    for k in reversed(range(net.nb)):
        R.join()  # D0 / D1 are about to be rewritten: the previous RRDB's weight gradients read them
        if x3:  # gradient scale of this RRDB from max |trunk gradient| at its output
            amax = ws.gamax.data_ptr() + 4 * k
            ovf = ws.bwd_overflow.data_ptr()
            if k == net.nb - 1 or not AMAX_FUSED:  # (else: taken by the previous RRDB's closing add, below)
                _lib.check(lib.esr_grad_amax(ws.GA.data_ptr(), 64, 0, 64, Bn, H, W, amax, stream), 'grad_amax')
            _lib.check(lib.esr_axpby_gs(D0.data_ptr(), dcp, d4, 1, 0.2, ws.GA.data_ptr(), 64, 0, 0, 0.0, None, 0, 0,
                                        0, 64, Bn, H, W, amax, ovf, stream), 'axpby_gs')
            for j, (dc, dn) in zip((2, 1, 0), ((D0, D1), (D1, D0), (D0, D1))):
                _rdb_backward_x3(R, Q[3 * k + j], dc, bp.rdb[3 * k + j], R.x3[0][3 * k + j], zc, cp, H, W,
                                 (dn, dcp, d4), amax, z_first=j == 2)
            if k > 0 and AMAX_FUSED:  # the trunk gradient at this RRDB's input, and its max for the next RRDB's scale
                _lib.check(lib.esr_axpby_gs_amax(ws.GA.data_ptr(), 64, 0, 1.0, ws.GA.data_ptr(), 64, 0, 0, 1.0,
                                                 D1.data_ptr(), dcp, d4, 1, 64, Bn, H, W, amax,
                                                 ws.gamax.data_ptr() + 4 * (k - 1), stream), 'axpby_gs_amax')
            else:
                _lib.check(lib.esr_axpby_gs(ws.GA.data_ptr(), 64, 0, 0, 1.0, ws.GA.data_ptr(), 64, 0, 0, 1.0,
                                            D1.data_ptr(), dcp, d4, 1, 64, Bn, H, W, amax, ovf, stream), 'axpby_gs')
            if need_input and zc:  # latent-slot gradient of this RRDB's blocks, back to fp32
                _lib.check(lib.esr_axpby_gs(ws.dZl.data_ptr(), 8, 0, 0, 1.0, ws.dZl.data_ptr(), 8, 0, 0, 1.0,
                                            ws.dzs.data_ptr(), 8, 0, 1, 8, Bn, H, W, amax, ovf, stream), 'axpby_gs')
        else:
            R.axpby(D0, dcp, d4, 0.2, ws.GA, 64, 0, C=64, h=H, w=W)
            for j, (dc, dn) in zip((2, 1, 0), ((D0, D1), (D1, D0), (D0, D1))):
                _rdb_backward(R, Q[3 * k + j], dc, bp.rdb[3 * k + j], bp.rdb_fused[3 * k + j], zc, cp, H, W,
                              (dn, dcp, d4))
            R.axpby(ws.GA, 64, 0, 1.0, ws.GA, 64, 0, 1.0, D1, dcp, d4, C=64, h=H, w=W)
        if bp.rrdb_lo[k] in pts:
            yield slice_to(bp.rrdb_lo[k])
    # conv_first: dL/dfea = trunk gradient + LR_conv skip
    R.axpby(ws.GA, 64, 0, 1.0, ws.GA, 64, 0, 1.0, ws.dU0, 64, 0, C=64, h=H, w=W)
    R.wgrad(bp.first, ws.first, ws.first_cp, ws.first_cp, 0, ws.GA, 64, 0, H, W)
    R.join()
    if seg is not None:
        slice_to(0)  # the last slice; the caller launches the rest of the buckets after this segment
        flat = None
    else:
        flat = bp.dw.index_select(0, bp.gidx) if need_params else None  # all parameter gradients, reference layout
    dx = None
    if need_input:
        R.dgrad_in(bp.first, ws.GA, 64, 0, 64, H, W, ws.dFirst, ws.first_cp)
        m = M // sf
        h, w = H - 2 * m, W - 2 * m
        d_lr = torch.empty(Bn, 3, h, w, device=dev)
        _lib.check(lib.esr_input_adjoint(ws.dFirst.data_ptr(), ws.first_cp, ws.first_lr_off, None, 0, 0, 0,
                                         a2.data_ptr() if cem is not None else None, 3, Bn, H, W, m,
                                         d_lr.data_ptr(), stream), 'input_adjoint lr')
        if latent:  # Z_LR = bilinear↓4(Z_HR) feeds conv_first and every LR conv; Z_HR feeds HR_conv0/1
            R.axpby(ws.dZl, 8, 0, 1.0, ws.dZl, 8, 0, 1.0, ws.dFirst, ws.first_cp, 0, C=8, h=H, w=W)
            d_z = torch.empty(Bn, 3, sf * h, sf * w, device=dev)
            _lib.check(lib.esr_input_adjoint(ws.dZh.data_ptr(), 8, 0, ws.dZl.data_ptr(), 8, 0, sf, None, 3, Bn,
                                             HH, WW, M, d_z.data_ptr(), stream), 'input_adjoint z')
            dx = torch.cat([d_z.view(Bn, 3 * sf * sf, h, w), d_lr], 1)  # raw view, SRRaGAN_model.py:252
        else:
            dx = d_lr
    return flat, dx


def _split_grads(bp, flat):
    grads, o = {}, 0
    for p in bp.params:
        grads[p] = flat[o:o + p.numel()].view(p.shape)
        o += p.numel()
    return grads


# how the training passes ran (observability: the benchmarks record the deltas of their timed regions)
GRAPH_COUNTS = {'eager': 0, 'captured': 0, 'replayed': 0}


def _run_graphed(ws, key, fn, *inputs):
    """fn(*inputs) eagerly the first time `key` is seen; captured into a HIP graph (static copies of the inputs) the
    second time; replayed from then on.  Returns fn's outputs, which for a graph live in its private pool (the caller
    clones what must outlive the next replay)."""
    if not USE_GRAPHS:
        GRAPH_COUNTS['eager'] += 1
        return fn(*inputs), False
    ent = ws.graphs.get(key)
    if ent is None:
        ws.graphs[key] = 'seen'
        GRAPH_COUNTS['eager'] += 1
        return fn(*inputs), False
    if ent == 'seen':
        static = [t.detach().clone() for t in inputs]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = fn(*static)
        ent = ws.graphs[key] = (g, static, out)
        GRAPH_COUNTS['captured'] += 1
    else:
        GRAPH_COUNTS['replayed'] += 1
    g, static, out = ent
    for st, t in zip(static, inputs):
        st.copy_(t)
    g.replay()
    return out, True


def _run_graphed_segments(ws, key, it_fn, d_out, on_seg):
    """_run_graphed for a backward that yields at segment boundaries (backward_segments with seg): the work up to each
    yield, and after the last one, is one HIP graph (all in one memory pool), and on_seg(lo) runs on the host after a
    segment is enqueued — eagerly the first time, captured the second (the captures enqueue nothing: every graph is
    replayed after them), replayed from then on — then on_seg(0) after the last segment.  Returns the backward's
    result (flat None, input gradient) and whether it came from graphs."""
    def eager(x):
        it = it_fn(x)
        while True:
            try:
                lo = next(it)
            except StopIteration as e:
                on_seg(0)
                return e.value
            on_seg(lo)
    if not USE_GRAPHS:
        GRAPH_COUNTS['eager'] += 1
        return eager(d_out), False
    ent = ws.graphs.get(key)
    if ent is None:
        ws.graphs[key] = 'seen'
        GRAPH_COUNTS['eager'] += 1
        return eager(d_out), False
    if ent == 'seen':
        static = d_out.detach().clone()
        pool = torch.cuda.graph_pool_handle()
        it = it_fn(static)
        segs, out = [], None
        while out is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool):
                try:
                    lo = next(it)
                except StopIteration as e:
                    lo, out = 0, (e.value,)
            segs.append((g, lo))
        ent = ws.graphs[key] = (segs, static, out[0])
        GRAPH_COUNTS['captured'] += 1
    else:
        GRAPH_COUNTS['replayed'] += 1
    segs, static, out = ent
    static.copy_(d_out)
    for g, lo in segs:
        g.replay()
        on_seg(lo)
    return out, True


def _cem_key(cem):
    if cem is None:
        return None
    return (id(cem), bool(cem.pre_pad), int(cem.margins_LR), cem.DownscaleOP.Filter_OP.weight.data_ptr(),
            cem.Conv_LR_with_Inv_hTh_OP.Filter_OP.weight.data_ptr(), cem.Upscale_OP.Filter_OP.weight.data_ptr())


class _GeneratorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, net, cem, *params):
        latent = net.latent_input is not None
        pre_pad = cem is not None and cem.pre_pad
        m = int(cem.margins_LR) if pre_pad else 0
        Bn, _, h, w = x.shape
        # The forward runs in the model's precision (x3 by default, as inference); the backward reads the split-f16
        # activations (weight-gradient inputs and LeakyReLU masks) and is exact fp32 itself.  Exception: weight
        # gradients through the eval-mode CEM pre-pad use the exact-fp32 forward — the replicated margin holds whole
        # lines of equal pre-activations, and an x3-rounded one near 0 flips its LeakyReLU slope along the line
        # (measured 7.6e-4 L2 on a weight gradient, tests/test_gpu_train.py X3_GRAD_FLOOR).
        prec = getattr(net, 'esr_precision', None) or E.DEFAULT_PRECISION
        if pre_pad and any(p.requires_grad for p in params):
            prec = 'f32'
        ws = _train_workspace(net, x.device, Bn, h + 2 * m, w + 2 * m, latent, prec)
        pk = E._packed(net, latent)  # parameter repack, outside any graph
        bad = pk.train_x3() if prec == 'x3' else None  # x3 weights refreshed in place, fixed per-layer scales
        A = E.act_scale(net) if prec == 'x3' else 1.0  # activation scale of the x3 forward (engine.ACT_SCALE)
        if prec == 'x3':
            pk.act_bias(A)  # biases × A, outside any graph

        def fwd(xs):
            if prec == 'x3':
                ws.overflow.copy_(bad)  # a weight outside its scale's safe range counts as an overflow
            return E._forward(net, xs, cem, prec, train_ws=ws)[0]
        key = ('fwd', prec, tuple(x.shape), _cem_key(cem), id(pk), getattr(pk, '_tx3_epoch', 0), A)
        xd = x.detach().contiguous()
        out, graphed = _run_graphed(ws, key, fwd, xd)
        split = prec == 'x3'
        if split and _DEFERRED[0] is not None:  # checked once after the whole training step (DeferredOverflow)
            _DEFERRED[0].add(ws.overflow, bad, pk.reset_train_x3, lambda: E.lower_act_scale(net))
        elif split and int(ws.overflow.item()):  # an activation (or weight) beyond the f16 range: redo in exact fp32
            E.OVERFLOW_RERUNS += 1
            if int(bad.item()):
                pk.reset_train_x3()  # new scales at the next x3 forward
            else:
                E.lower_act_scale(net)  # a scaled activation left f16's range: smaller activation scale next time
            ws = _train_workspace(net, x.device, Bn, h + 2 * m, w + 2 * m, latent, 'f32')
            out, graphed, split = E._forward(net, xd, cem, 'f32', train_ws=ws)[0], False, False
        ctx.net, ctx.cem, ctx.ws, ctx.latent, ctx.M, ctx.split = net, cem, ws, latent, ws.sf * m, split
        ctx.act_scale = A if split else 1.0  # (after an fp32 rerun the activations are unscaled)
        ctx.params = params
        ctx.flat_fg = getattr(net, '_esr_flat_fwd', None) if len(params) == 1 and \
            getattr(getattr(net, '_esr_flat_fwd', None), 'flat', None) is params[0] else None
        ctx.owner = _Owner()
        ws.owner = weakref.ref(ctx.owner)
        return out.clone() if graphed else out

    @staticmethod
    def backward(ctx, d_out):
        need_params = any(ctx.needs_input_grad[3:])
        need_input = ctx.needs_input_grad[0]
        if ctx.ws.owner() is not ctx.owner:  # cannot happen through _train_workspace; guards direct workspace reuse
            raise RuntimeError('esr_amd: the saved activations of this forward were overwritten by a later forward')
        bp = _bwd_packed(ctx.net, ctx.latent)  # parameter repack, outside any graph
        x3 = DGRAD_X3 and ctx.split and (need_params or need_input)
        if x3:
            bp.x3_fused()  # x3 repack of the data-gradient weights, outside any graph
        sink = getattr(ctx.net, '_esr_grad_sink', None)
        if ctx.flat_fg is not None and sink is not None and sink.armed and sink.flat_opt is ctx.flat_fg and \
                need_params and not need_input and (not x3 or _DEFERRED[0] is not None):
            return _GeneratorFn._sliced_backward(ctx, d_out, bp, x3, sink)

        def run(x3):
            key = ('bwd', tuple(d_out.shape), _cem_key(ctx.cem), ctx.M, need_params, need_input, id(bp), ctx.split,
                   x3, ctx.act_scale)
            return _run_graphed(
                ctx.ws, key, lambda g: generator_backward(ctx.net, ctx.cem, ctx.ws, g, ctx.latent, ctx.M,
                                                          need_params=need_params, need_input=need_input,
                                                          split=ctx.split, x3=x3, act_scale=ctx.act_scale),
                d_out.contiguous())
        (flat, dx), graphed = run(x3)
        if x3 and _DEFERRED[0] is not None:  # checked once after the whole training step (DeferredOverflow)
            _DEFERRED[0].add(ctx.ws.bwd_overflow, bp._x3_bad, bp.reset_x3)
        elif x3 and int(ctx.ws.bwd_overflow.item()):  # a scaled gradient (or weight) left f16's range: redo in fp32
            E.OVERFLOW_RERUNS += 1
            if int(bp._x3_bad.item()):
                bp.reset_x3()  # new weight scales at the next x3 backward
            (flat, dx), graphed = run(False)
        if graphed:
            flat = flat.clone() if flat is not None else None
            dx = dx.clone() if dx is not None else None
        # the generator's FlatAdam, set by SRRaGANModel.optimize_parameters only around its generator loss's
        # .backward() (every parameter's AccumulateGrad runs, no per-parameter hooks wait); None everywhere else
        if ctx.flat_fg is not None:  # the flat parameter was the input (generator_forward_train)
            ctx.owner.done = True
            if flat is not None:
                ctx.flat_fg._sync_views()  # (parameters / gradients replaced since the last bind are re-attached first)
                if not ctx.flat_fg.accepts_flat_grad(bp.params):
                    raise RuntimeError('esr_amd: flat gradient layout differs from the optimiser\'s buffer')
            return (dx, None, None, flat)
        fg = getattr(ctx.net, '_esr_flat_grad', None)
        if flat is not None and fg is not None and all(ctx.needs_input_grad[3:]) and fg.accepts_flat_grad(bp.params):
            # flat is laid out as the optimiser's buffer: one add instead of 702 per-parameter accumulations (the
            # parameters' .grad are views of fg.flat.grad, so every reader sees the sum)
            fg._sync_views()
            fg.flat.grad.add_(flat)
            grads = {}
            sink = getattr(ctx.net, '_esr_grad_sink', None)
            if sink is not None and sink.flat_opt is fg:
                sink.ready_from(0)  # (no per-parameter accumulation: the sink's hooks would not see this gradient)
        else:
            grads = _split_grads(bp, flat) if flat is not None else {}
        ctx.owner.done = True  # the workspace may be reused (a retained graph's second backward would then raise)
        return (dx, None, None) + tuple(grads.get(p) for p in ctx.params)

    @staticmethod
    def _sliced_backward(ctx, d_out, bp, x3, sink):
        """Across ranks (SRRaGANModel's generator step, last accumulation micro-step): the backward adds its weight
        gradients into the optimiser's flat gradient itself, slice by slice from the output end, and after each slice
        hands the finished range to the flat-mode GradBuckets `sink`, whose buckets' all-reduces then run while the
        rest of the backward does (the whole generator is one autograd node: through autograd the gradient would
        arrive only after all of it).  Only with the x3 overflow check deferred (a redo restores flat.grad from the
        step's snapshot) or an exact-fp32 backward."""
        fg = ctx.flat_fg
        fg._sync_views()
        if not fg.accepts_flat_grad(bp.params):
            raise RuntimeError('esr_amd: flat gradient layout differs from the optimiser\'s buffer')
        lows = tuple(sink.emit_offsets())
        key = ('bwdseg', tuple(d_out.shape), _cem_key(ctx.cem), ctx.M, id(bp), ctx.split, x3, ctx.act_scale,
               fg.flat.grad.data_ptr(), lows)
        it_fn = lambda g: backward_segments(ctx.net, ctx.cem, ctx.ws, g, ctx.latent, ctx.M, need_params=True,  # noqa
                                            need_input=False, split=ctx.split, x3=x3, act_scale=ctx.act_scale,
                                            seg=(fg.flat.grad, lows))
        _run_graphed_segments(ctx.ws, key, it_fn, d_out.contiguous(), sink.ready_from)
        if x3:
            _DEFERRED[0].add(ctx.ws.bwd_overflow, bp._x3_bad, bp.reset_x3)
        ctx.owner.done = True
        return (None, None, None, None)


def generator_forward_train(net, x, cem):
    params = E.param_list(net)
    if not any(p.requires_grad for p in params):  # a frozen generator (Z optimisation): only the input gradient, and
        return _GeneratorFn.apply(x, net, cem)     # no 702-input autograd node (~0.5 ms of host time per forward)
    fg = getattr(net, '_esr_flat_fwd', None)  # SRRaGANModel's own step, single-process: a FlatAdam over `params`
    if FLAT_FWD and fg is not None and fg.flat.requires_grad and fg.accepts_flat_grad(params) and \
            all(p.requires_grad for p in params):
        # one autograd input, the optimiser's flat parameter: the backward returns the flat gradient (laid out as the
        # flat buffer) and autograd adds it into flat.grad, of which every parameter's .grad is a view
        return _GeneratorFn.apply(x, net, cem, fg.flat)
    return _GeneratorFn.apply(x, net, cem, *params)
