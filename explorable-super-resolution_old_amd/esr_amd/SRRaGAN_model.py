"""SRRaGANModel — counterpart of reference codes/models/SRRaGAN_model.py (the north_star's "SRGAN_model").

Keeps the interface the reference's drivers use — `feed_data`, `ConcatLatent`, `GetLatent`, `optimize_parameters`,
`test`, `get_current_visuals`, `update_learning_rate(cur_step)`, `get_current_log`, `get_current_learning_rate`,
`perform_validation`, `save`/`load`/`save_log`, attributes `netG`, `netD`, `CEM_net`, `fake_H`, `var_L`, `var_H`, `model_input`,
`num_latent_channels`, `Z_size_factor`, `log_dict`, `step` — for the configuration the shipped JSONs select:
CEM_arch, latent `all_layers`/`HR_downscaled` (or no latent), WGAN-GP (relativistic or not), range loss, D_verification
'past'/'current'/None, fixed or adaptive D_update_ratio, gradient accumulation.  Options the shipped configs switch off (VGG feature loss — broken in the
reference, pixel/high-pass/shift-invariant/optimal-Z/latent losses, encoder, decomposed D input) raise
NotImplementedError instead of silently differing.  Checkpoints and logs keep the reference's formats
(base_model.py:86-144; SRRaGAN_model.py:695-719, 766-813): `{step}_G.pth` / `{step}_D.pth` dicts with
model_state_dict + optimizer_state_dict, the positional key-remapping loader with the latent-channel zero-prepend, and
logs.npz / lr.npz; checkpoints are read with torch.load(weights_only=True).  Plotting (display_log_figure) and
TensorBoard are out of scope: display_log_figure is a no-op, so codes/train.py runs unchanged.

Multi-GPU: one process per GPU (torch.distributed, RCCL).  The reference's nn.DataParallel computes every loss on the
gathered global batch; with equal per-rank batches the average of per-rank gradients equals that gradient, so the G / D
gradients of the last accumulation micro-step are averaged by bucketed asynchronous all-reduces launched from inside
the backward as each bucket's gradients become final (GradBuckets).  BatchNorm statistics stay
per-replica (as DataParallel's) and the running buffers are broadcast from rank 0 (DataParallel keeps replica 0's).
The per-image D statistics that gate the generator step are all-reduced so that every rank takes the same branch.
"""
import collections
import math
import os
import re
import struct
import warnings
import zlib
from collections import OrderedDict

import numpy as np
import torch
import torch.distributed as dist

from . import CEMnet
from . import dconv as D
from . import engine as E
from . import networks
from . import train_engine as TE
from .flat_optim import FlatAdam
from .loss import CreateRangeLoss, GANLoss, GradientPenaltyLoss


def Latent_channels_desc_2_num_channels(desc):
    """loss.py:14-21."""
    if isinstance(desc, int):
        return desc
    if desc == 'STD_1dir':
        return 2
    if desc == 'STD_directional' or 'structure_tensor' in desc:
        return 3
    raise ValueError(desc)


def SVD_2_LatentZ(SVD_values, max_lambda=1):
    """utils/util.py:137-143: (lambda0, lambda1, theta) -> structure-tensor latent channels."""
    l0, l1, th = SVD_values[:, 0, ...], SVD_values[:, 1, ...], SVD_values[:, -1, ...]
    s, c = torch.sin(th) ** 2, torch.cos(th) ** 2
    return torch.stack([2 * max_lambda * (l1 * s + l0 * c) - max_lambda,
                        2 * max_lambda * (l0 * s + l1 * c) - max_lambda,
                        2 * (l0 - l1) * torch.sin(th) * torch.cos(th)], 1)


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _host_collectives():
    """True when the process group is gloo (the CPU test path of the multi-rank code, and ranks sharing one GPU):
    it moves device tensors through host copies that are not ordered on the device stream the way RCCL's
    collectives are (tests/test_gpu_ddp.py saw noise-level gradient differences against the single-process run)."""
    return _world() > 1 and dist.get_backend() == 'gloo'


class _Done:
    def wait(self):
        return True


def collective(fn, t, *args, async_op=False, **kw):
    """dist.<fn>(t, ...) in place on the backend's terms: RCCL takes device tensors stream-ordered (asynchronous when
    async_op); with gloo a device tensor goes through an explicit host copy (synchronous: the copy out waits for the
    stream, the copy back is enqueued on it)."""
    if t.is_cuda and _host_collectives():
        c = t.detach().cpu()
        fn(c, *args, **kw)
        t.copy_(c)
        return _Done() if async_op else None
    return fn(t, *args, async_op=async_op, **kw)


def _allreduce_grads(params):
    """Average the .grad of `params` over ranks in one flat bucket (RCCL all-reduce over xGMI)."""
    if _world() == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    collective(dist.all_reduce, flat)
    flat /= _world()
    o = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[o:o + n].view_as(g))
        o += n


class GradBuckets:
    """DDP-style gradient averaging for one network over ranks (the reference's nn.DataParallel, networks.py:99-101,
    125-126, computes every loss on the gathered global batch; with equal per-rank batches the average of the per-rank
    gradients is that gradient).

    Parameters are grouped into buckets of at most `cap_bytes` in reverse registration order — the order a backward
    finalises them (output layers first).  While armed (the last micro-step of a gradient accumulation), a
    post-accumulate-grad hook marks each parameter whose gradient that backward has finished; when a bucket is
    complete its flattened gradients go out as one asynchronous all-reduce (RCCL over xGMI), overlapping the rest of the
    backward; buckets go out strictly in bucket order (the same collective sequence on every rank).  `finish()` launches
    the buckets still pending (parameters that got no gradient in this backward: requires_grad toggled off, or not
    reached), waits for every bucket, averages and writes back.  Buckets are ≥ a few MB so that each ring
    all-reduce runs near the per-link xGMI bandwidth rather than its latency.

    Flat mode (`flat_opt`: a FlatAdam over exactly these parameters, whose .grad are views of flat_opt.flat.grad, so a
    bucket is one contiguous range of it): a bucket is all-reduced in place on its range (no cat, no copy back).  A
    producer that writes the flat gradient itself — the HIP generator's backward, one autograd node over the
    optimiser's flat parameter (train_engine._GeneratorFn) — calls `ready_from(lo)` each time flat.grad[lo:] is final,
    so that the buckets launch while the rest of its backward runs (`emit_offsets()` tells it where a bucket
    completes).  A post-accumulate hook on the flat parameter launches everything when the flat gradient arrives
    through autograd instead."""

    def __init__(self, params, cap_bytes=16 << 20, flat_opt=None):
        self.params = list(params)
        self.buckets, cur, size = [], [], 0
        for p in reversed(self.params):
            n = p.numel() * p.element_size()
            if cur and size + n > cap_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += n
        if cur:
            self.buckets.append(cur)
        self.where = {id(p): b for b, ps in enumerate(self.buckets) for p in ps}
        self.flat_opt = flat_opt if flat_opt is not None and flat_opt.accepts_flat_grad(self.params) else None
        self.ranges = None
        if self.flat_opt is not None:
            off, o = {}, 0
            for p in self.params:
                off[id(p)] = o
                o += p.numel()
            self.ranges = [(off[id(ps[-1])], off[id(ps[0])] + ps[0].numel()) for ps in self.buckets]
        self.armed = False
        self.launched_in_backward = 0
        self._next = 0
        self._pending = [set() for _ in self.buckets]
        self._works = [None] * len(self.buckets)
        self.hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params] \
            if _world() > 1 else []
        if self.flat_opt is not None and _world() > 1:
            self.hooks.append(self.flat_opt.flat.register_post_accumulate_grad_hook(lambda _: self.ready_from(0)))
        # what went over the wire: collectives, bytes, and the stream time finish() left exposed (device events
        # around the waits, read lazily by comm_stats so no host sync is added to the step)
        self.n_allreduce = 0
        self.allreduce_bytes = 0
        self._exposed = []
        self._exposed_ms = 0.0

    def comm_stats(self):
        """{'allreduces', 'allreduce_bytes', 'exposed_ms'} since construction (exposed_ms: compute-stream time spent
        waiting in finish() for the collectives, i.e. the part not overlapped with the backward)."""
        for e0, e1 in self._exposed:
            e1.synchronize()
            self._exposed_ms += e0.elapsed_time(e1)
        self._exposed = []
        return {'allreduces': self.n_allreduce, 'allreduce_bytes': self.allreduce_bytes,
                'exposed_ms': round(self._exposed_ms, 3)}

    def arm(self):
        self.armed = _world() > 1
        self._pending = [set(id(p) for p in ps) for ps in self.buckets]
        self._works = [None] * len(self.buckets)
        self._next = 0
        self.launched_in_backward = 0

    def emit_offsets(self):
        """Flat mode: the flat-gradient offsets at which a producer finalising the gradient from its end should call
        ready_from (each bucket's lower end)."""
        return sorted({lo for lo, _ in self.ranges}) if self.ranges is not None else [0]

    def _launch(self, b):
        if self.ranges is not None:
            lo, hi = self.ranges[b]
            g = self.flat_opt.flat.grad[lo:hi]
            self._works[b] = (collective(dist.all_reduce, g, async_op=True), g, None)
            self.n_allreduce += 1
            self.allreduce_bytes += g.numel() * g.element_size()
            return
        grads = [p.grad for p in self.buckets[b] if p.grad is not None]
        if not grads:
            self._works[b] = ()
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        self._works[b] = (collective(dist.all_reduce, flat, async_op=True), flat, grads)
        self.n_allreduce += 1
        self.allreduce_bytes += flat.numel() * flat.element_size()

    def _launch_ready(self):
        # launch complete buckets strictly in bucket order (the same sequence of collectives on every rank, as RCCL
        # requires, whatever order the backward finalises the parameters in)
        while self._next < len(self.buckets) and not self._pending[self._next]:
            self._launch(self._next)
            self._next += 1
            self.launched_in_backward += 1

    def _on_grad(self, p):
        if not self.armed:
            return
        self._pending[self.where[id(p)]].discard(id(p))
        self._launch_ready()

    def ready_from(self, lo):
        """Flat mode: flat_opt.flat.grad[lo:] holds its final value for this backward (launches the buckets inside)."""
        if not self.armed:
            return
        for b in range(self._next, len(self.buckets)):
            if self.ranges[b][0] >= lo:
                self._pending[b].clear()
        self._launch_ready()

    def finish(self):
        if not self.armed:
            return
        self.armed = False
        for b in range(self._next, len(self.buckets)):  # the rest, still in bucket order
            self._launch(b)
        w = _world()
        items = [it for it in self._works if it]
        ev = None
        if items and items[0][1].is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for work, _, _ in items:
            work.wait()
        if ev is not None:
            ev[1].record()
            while self._exposed and self._exposed[0][1].query():  # fold the completed ones (no sync): bounded list
                e0, e1 = self._exposed.pop(0)
                self._exposed_ms += e0.elapsed_time(e1)
            self._exposed.append(ev)
        if self.ranges is not None:  # in place on flat.grad: one scaling of the whole buffer
            self.flat_opt.flat.grad.div_(w)
        else:
            for _, flat, grads in items:
                flat /= w
                o = 0
                for g in grads:
                    n = g.numel()
                    g.copy_(flat[o:o + n].view_as(g))
                    o += n
        self._works = [None] * len(self.buckets)


class FlatBuffers:
    """A module's floating-point buffers (the D BatchNorms' running means / variances) as views of one flat tensor, so
    that rank 0's values reach every rank in ONE broadcast (DataParallel keeps replica 0's buffers).
    num_batches_tracked stays as it is: every rank increments it identically.  The views are re-bound when something
    replaced a buffer (module.to(), load_state_dict(assign=True))."""

    def __init__(self, module):
        self.module = module
        self.flat = None
        self._ptrs = []

    def _entries(self):
        return [(m, n, b) for m in self.module.modules() for n, b in m._buffers.items()
                if b is not None and b.is_floating_point()]

    def sync(self):
        ents = self._entries()
        if self.flat is None or len(ents) != len(self._ptrs) or \
                any(b.data_ptr() != ptr for (_, _, b), ptr in zip(ents, self._ptrs)):
            flat = torch.cat([b.detach().reshape(-1) for _, _, b in ents])
            o = 0
            for m, n, b in ents:
                m._buffers[n] = flat[o:o + b.numel()].view_as(b)
                o += b.numel()
            self.flat = flat
            self._ptrs = [b.data_ptr() for _, _, b in self._entries()]
        return self.flat


def _broadcast_buffers(module, flat=None):
    """Rank 0's buffers everywhere: one broadcast of `flat` (a FlatBuffers of module), else one per buffer."""
    if _world() == 1:
        return
    if flat is not None:
        collective(dist.broadcast, flat.sync(), 0)
        return
    for b in module.buffers():
        collective(dist.broadcast, b, 0)


class _GlobalMean(torch.autograd.Function):
    """mean(t) over the GLOBAL batch (every rank's t, equal sizes), differentiable: the relativistic D terms
    (SRRaGAN_model.py:380-382, 521-524) subtract the mean over DataParallel's gathered batch.  Backward: the gradient
    reaching the global mean is all-reduced and spread over the local elements, so that the ranks' averaged parameter
    gradients are the gradient of the global-batch loss also for non-linear GAN losses (vanilla, lsgan); wgan-gp is
    linear, where rank-local means give the same average."""

    @staticmethod
    def forward(ctx, t):
        ctx.shape = t.shape
        m = t.detach().mean().reshape(1)
        collective(dist.all_reduce, m)
        return (m / _world()).reshape(())

    @staticmethod
    def backward(ctx, g):
        gs = g.detach().reshape(1).clone()
        collective(dist.all_reduce, gs)
        n = 1
        for d in ctx.shape:
            n *= d
        return (gs / (_world() * n)).reshape(()).expand(ctx.shape)


LATENT_WEIGHTS_RELATIVE_STD = 0.  # base_model.py:116
# x3 overflow checks of the training step read once per micro-step (optimize_parameters); 0 = after every pass
DEFER_OVERFLOW = os.environ.get('ESR_DEFER_OVERFLOW', '1') != '0'


class SRRaGANModel:
    def __init__(self, opt, accumulation_steps_per_batch=1, kernel=None, device=None):
        self.opt = opt
        self.is_train = bool(opt['is_train'])
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        opt_G = opt['network_G']
        li = opt_G.get('latent_input')
        self.latent_input = li if li not in (None, 'None') else None
        self.latent_input_domain = opt_G.get('latent_input_domain')
        self.num_latent_channels = Latent_channels_desc_2_num_channels(opt_G.get('latent_channels', 0) or 0) \
            if self.latent_input is not None else 0
        if self.latent_input is not None:
            self.Z_size_factor = opt['scale'] if 'HR' in self.latent_input_domain else 1
        self.CEM_arch = bool(opt_G.get('CEM_arch'))
        self.step = 0
        self.gradient_step_num = 0
        self.generator_step = False
        self.CEM_net = None
        paths = opt.get('path') or {}
        self.save_dir = paths.get('models')
        self.log_path = paths.get('log')
        if self.CEM_arch or self.latent_input is not None:
            conf = CEMnet.Get_CEM_Config(opt['scale'])
            conf.input_range = np.array(opt.get('range', [0, 1]))
            test_opt = opt.get('test') or {}
            if test_opt.get('kernel') == 'estimated':
                conf.lower_magnitude_bound = 0.1
            k = kernel if kernel is not None else test_opt.get('kernel')
            if isinstance(k, str) and k == 'estimated':
                k = None
            self.CEM_net = CEMnet.CEMnet(conf, upscale_kernel=k)
            if not self.CEM_arch:
                self.CEM_net.WrapArchitecture_PyTorch(only_padders=True)
        self.netG = networks.define_G(opt, CEM=self.CEM_net, num_latent_channels=self.num_latent_channels)
        self.netG.to(self.device)
        # the reference's log keys in its order (SRRaGAN_model.py:72-75): get_current_log reports them in this order
        keys = ['l_g_pix', 'l_g_fea', 'l_g_range', 'l_g_gan', 'l_d_real', 'l_d_fake', 'D_loss_STD', 'l_d_real_fake',
                'l_g_highpass', 'l_g_shift_invariant', 'D_real', 'D_fake', 'D_logits_diff', 'psnr_val',
                'D_update_ratio', 'LR_decrease', 'Correctly_distinguished', 'l_d_gp', 'l_e', 'l_g_optimalZ'] + \
            ['l_g_latent_%d' % i for i in range(self.num_latent_channels)]
        self.log_dict = OrderedDict((k, []) for k in keys)
        self.max_accumulation_steps = accumulation_steps_per_batch
        if self.is_train:
            self._init_training(opt, accumulation_steps_per_batch)
            self.generator_changed = True  # :243, so that train.py validates the initial state
        self.load()  # :244: resume / pretrained weights / the test model, as the options say

    # ------------------------------------------------------------------------------------------------------------------
    def _init_training(self, opt, accumulation_steps_per_batch):
        t = opt['train']
        for k in ('feature_weight', 'latent_weight', 'optimalZ_loss_weight', 'highpass_weight',
                  'shift_invariant_weight'):
            if t.get(k):
                raise NotImplementedError('%s > 0 is not part of the built training path (shipped configs use 0)' % k)
        # G pixel loss (SRRaGAN_model.py:108-120, 477-483): L1 / L2 between fake_H and var_H, in the HR domain or (not
        # with CEM_arch: the reference asserts that at construction, :61) between their bilinear resizes to the LR size
        self.cri_pix = None
        if (t.get('pixel_weight') or 0) > 0:
            crit = t.get('pixel_criterion')
            if crit == 'l1':
                self.cri_pix = torch.nn.functional.l1_loss
            elif crit == 'l2':
                self.cri_pix = torch.nn.functional.mse_loss
            else:
                raise NotImplementedError('Loss type [{}] not recognized.'.format(crit))
            self.l_pix_w = t['pixel_weight']
        self.pixel_domain = t.get('pixel_domain', 'HR')
        assert self.pixel_domain == 'HR' or not self.CEM_arch, \
            'Why should I use CEM_arch AND penalize MSE in the LR domain?'
        if opt['network_D'].get('decomposed_input'):
            raise NotImplementedError('decomposed D input')
        rel = opt['network_D'].get('relativistic')
        self.relativistic_D = rel is None or bool(rel)  # SRRaGAN_model.py:87: unset means relativistic
        self.D_verification = t.get('D_verification')
        assert self.D_verification in ['current', 'past', None]
        self.grad_accumulation_steps_G = t.get('grad_accumulation_steps_G', 1)
        self.grad_accumulation_steps_D = t.get('grad_accumulation_steps_D', 1)
        self.max_accumulation_steps = accumulation_steps_per_batch
        self.l_gan_w = t['gan_weight']
        self.D_exists = self.l_gan_w > 0
        # precision of the discriminator in the G step (its data gradient into fake_H seeds G's backward); None = the
        # dconv module default
        self.d_gstep_precision = os.environ.get('ESR_D_GSTEP_PRECISION') or None
        self.netG.train()
        self.cri_range = CreateRangeLoss(opt.get('range', [0, 1])) if t.get('range_weight', 0) > 0 else None
        self.l_range_w = t.get('range_weight', 0)
        self.optimizers = []
        gparams = [p for p in self.netG.parameters() if p.requires_grad]
        lr_G, lr_D = t['lr_G'], t.get('lr_D')
        lr_file = os.path.join(self.log_path, 'lr.npz') if self.log_path else None
        if lr_file and os.path.isfile(lr_file):  # SRRaGAN_model.py:212-216: learning rates decayed by a resumed run
            with np.load(lr_file) as f:
                lr_G, lr_D = float(f['lr_G']), float(f['lr_D'])
        if self.latent_input is not None:  # SRRaGAN_model.py:79-80
            self.latent_grads_multiplier = t['lr_latent'] / t['lr_G'] if t.get('lr_latent') else 1
            self.channels_idx_4_grad_amplification = [[] for _ in self.netG.parameters()]
        # one flat buffer for all generator parameters (flat_optim.py: the reference's per-element update)
        self.optimizer_G = FlatAdam(gparams, lr=lr_G, weight_decay=t.get('weight_decay_G') or 0,
                                    betas=(t['beta1_G'], 0.999))
        g = self.netG.module if isinstance(self.netG, torch.nn.DataParallel) else self.netG
        # the RRDBNet whose backward may add its flat gradient buffer straight into the optimiser's; armed only around
        # the generator loss's .backward() in optimize_parameters (single process: no bucket hooks wait)
        self._rrdb = g.generated_image_model if hasattr(g, 'generated_image_model') else g  # (CEM_arch or bare)
        self.optimizers.append(self.optimizer_G)
        if self.D_exists:
            self.netD = networks.define_D(opt, CEM=self.CEM_net).to(self.device)
            self.netD.train()
            self.cri_gan = GANLoss(t['gan_type'], 1.0, 0.0)
            r = t.get('D_update_ratio')
            self.global_D_update_ratio = r if r is not None else 1  # <= 0: adaptive ratio (optimize_parameters)
            self.D_init_iters = t.get('D_init_iters') or 0
            if t['gan_type'] == 'wgan-gp':
                self.cri_gp = GradientPenaltyLoss(device=self.device)
                self.l_gp_w = t['gp_weigth']
            # flat buffer too: ~40 tensors, but the per-tensor foreach Adam costs ~2 ms of host time per step
            self.optimizer_D = FlatAdam(list(self.netD.parameters()), lr=lr_D,
                                        weight_decay=t.get('weight_decay_D') or 0, betas=(t['beta1_D'], 0.999))
            self.optimizers.append(self.optimizer_D)
        else:
            self.global_D_update_ratio, self.D_init_iters = 1, 0
        self.schedulers = [torch.optim.lr_scheduler.MultiStepLR(o, t['lr_steps'], t['lr_gamma'])
                           for o in self.optimizers]
        # flat mode: the buckets are ranges of the FlatAdams' gradient buffers, all-reduced in place; the generator's
        # backward launches its buckets itself as it finalises them (train_engine._GeneratorFn, _esr_grad_sink)
        self._g_buckets = GradBuckets(gparams, flat_opt=self.optimizer_G)
        self._d_buckets = GradBuckets(list(self.netD.parameters()), flat_opt=self.optimizer_D) \
            if self.D_exists else None
        self._d_flat_buffers = FlatBuffers(self.netD) if self.D_exists else None

    # ------------------------------------------------------------------------------------------------------------------
    def ConcatLatent(self, LR_image, latent_input):
        """SRRaGAN_model.py:249-255: the HR latent is carried as a raw view into sf² LR-sized channels."""
        if latent_input is not None:
            if LR_image.size()[2:] != latent_input.size()[2:]:
                latent_input = latent_input.contiguous().view([latent_input.size(0)] + [
                    latent_input.size(1) * self.opt['scale'] ** 2] + list(LR_image.size()[2:]))
            self.model_input = torch.cat([latent_input, LR_image], dim=1)
        else:
            self.model_input = 1 * LR_image

    def AssignLatent(self, latent_input):
        """SRRaGAN_model.py:260-261."""
        self.netG.module.generated_image_model.Z = latent_input

    def GetLatent(self):
        latent = 1 * self.model_input[:, :-3, ...]
        if latent.size(1) != self.num_latent_channels:
            latent = latent.view([latent.size(0)] + [self.num_latent_channels] +
                                 [self.opt['scale'] * v for v in list(latent.size()[2:])])
        return latent

    def feed_data(self, data, need_HR=True):
        """SRRaGAN_model.py:269-302."""
        self.var_L = data['LR'].to(self.device)
        cur_Z = None
        if self.latent_input is not None:
            B = self.var_L.size(0)
            if 'Z' in data:
                cur_Z = data['Z']
            else:
                lc = self.opt['network_G']['latent_channels']
                cur_Z = torch.rand([B, self.num_latent_channels, 1, 1])
                if lc in ['SVD_structure_tensor', 'SVDinNormedOut_structure_tensor']:
                    cur_Z[:, -1, ...] = 2 * np.pi * cur_Z[:, -1, ...]
                    cur_Z = SVD_2_LatentZ(cur_Z).detach()
                else:
                    cur_Z = 2 * cur_Z - 1
            hw = [self.Z_size_factor * v for v in list(self.var_L.size()[2:])]
            # the spatial broadcasts happen on the device (the reference builds them on the host: a 28 MB CPU tensor
            # per step at config 3)
            if isinstance(cur_Z, (int, float)):
                cur_Z = torch.full([1, self.num_latent_channels] + hw, float(cur_Z), device=self.device)
            elif not torch.is_tensor(cur_Z) and np.ndim(cur_Z) < 4:
                cur_Z = cur_Z * np.ones([1, self.num_latent_channels] + hw)
            elif torch.is_tensor(cur_Z) and cur_Z.size(2) == 1:
                if not cur_Z.is_cuda and self.device.type == 'cuda':
                    # through a (cached) pinned buffer: a pageable host-to-device copy blocks the host until it is done
                    cur_Z = cur_Z.float().contiguous().pin_memory()
                cur_Z = cur_Z.to(self.device, non_blocking=True).float().expand(-1, -1, *hw).contiguous()
            if not torch.is_tensor(cur_Z):
                cur_Z = torch.from_numpy(np.asarray(cur_Z, dtype=np.float32))
            cur_Z = cur_Z.float().to(self.device)
        self.ConcatLatent(LR_image=self.var_L, latent_input=cur_Z)
        if need_HR:
            self.var_H = data['HR'].to(self.device)
            self.var_ref = (data['ref'] if 'ref' in data else data['HR']).to(self.device)

    # ------------------------------------------------------------------------------------------------------------------
    def _d_statistics_t(self, pred_real, pred_fake, means=()):
        """Per-image D logit differences, summed over ranks (global-batch semantics of DataParallel), as a device
        tensor [mean diff, fraction correctly distinguished, mean D(real), mean D(fake), *means] (no host sync).
        `means`: scalars (this micro-step's logged losses) averaged over ranks in the same all-reduce — a loss that
        is a mean over the local batch averages to the global batch's (equal per-rank batches)."""
        diff = torch.mean(pred_real.detach() - pred_fake.detach(), dim=list(range(1, pred_real.dim())))
        # (the image count as a device fill, not torch.tensor(): a pageable host-to-device copy waits for the stream)
        s = torch.stack([diff.sum(), (diff > 0).float().sum(), diff.new_full((), float(diff.numel())),
                         pred_real.detach().mean(), pred_fake.detach().mean()] +
                        [m.detach().reshape(()).to(diff.dtype) for m in means])
        if _world() > 1:
            collective(dist.all_reduce, s)
            s[3:] /= _world()
        return torch.cat([torch.stack([s[0] / s[2], s[1] / s[2]]), s[3:]])

    def _batch_mean(self, t):
        """torch.mean(t) over the batch DataParallel would have gathered: across ranks (differentiable) when the GAN
        loss is not linear in it; rank-local for wgan-gp, whose averaged gradients are then already the global ones
        and whose logged losses are averaged in _d_statistics_t."""
        if _world() > 1 and self.cri_gan.gan_type != 'wgan-gp':
            return _GlobalMean.apply(t)
        return torch.mean(t)

    def _global_log_means(self, vals):
        """Logged per-micro-step losses (device scalars) averaged over ranks: the global batch's values."""
        if _world() > 1 and vals:
            t = torch.stack([v.detach().reshape(()) for v in vals])
            collective(dist.all_reduce, t)
            t /= _world()
            return list(t.unbind())
        return [v.detach().reshape(()) for v in vals]

    def _d_statistics(self, pred_real, pred_fake):
        return tuple(float(v) for v in self._d_statistics_t(pred_real, pred_fake).tolist())

    # ---- logged scalars: device values are read back in one copy when someone needs them ----------------------------
    # The reference calls .item() on every logged loss right away (SRRaGAN_model.py:401-574); each call drains the GPU.
    # Here they queue (in step order) and are copied to the host together when log_dict is read (the training loop's
    # logging, the 'past' gate or the adaptive D_update_ratio) — same values, same order, no mid-step sync.
    @property
    def log_dict(self):
        self._flush_logs()
        return self._log_dict

    @log_dict.setter
    def log_dict(self, d):
        self._flush_logs()
        self._log_dict = d

    def _defer(self, tensor, fn):
        self.__dict__.setdefault('_pending_logs', []).append((tensor, fn))

    def _flush_logs(self):
        pend = self.__dict__.get('_pending_logs')
        if not pend:
            return
        self._pending_logs = []
        ts = [t.reshape(-1) for t, _ in pend if t is not None]
        vals = torch.cat(ts).tolist() if ts else []
        i = 0
        for t, fn in pend:
            if t is None:
                fn(None)
            else:
                fn(vals[i:i + t.numel()])
                i += t.numel()

    def _d_update_ratio(self, t):
        """SRRaGAN_model.py:314-324: the configured ratio, or (D_update_ratio <= 0) one adapted to the mean logged
        D_logits_diff of the last D_valid_Steps_4_G_update D steps (> 1: D steps per G step; < 1: G steps per D step)."""
        if self.global_D_update_ratio > 0:
            return self.global_D_update_ratio
        n = t['D_valid_Steps_4_G_update']
        if len(self.log_dict['D_logits_diff']) < n:
            return n
        log_mean = np.log(max(1e-5, np.mean([v[1] for v in self.log_dict['D_logits_diff'][-n:]])))
        if log_mean < -2:
            return int(-2 * np.ceil((log_mean + 1) * 2) / 2)
        return 1 / max(1, int(np.floor((log_mean + 2) * 20)))

    def _gate_generator_step(self, t, first_acc_D, diff, correct):
        """SRRaGAN_model.py:400-427: whether this micro-step also updates G.  `diff`/`correct` are this micro-step's
        D statistics over the GLOBAL batch (all-reduced by _d_statistics) and log_dict holds the all-reduced history,
        so every rank takes the same branch, as DataParallel's single process did."""
        if first_acc_D:
            self.generator_step = (self.gradient_step_num % max(1, self.cur_D_update_ratio) == 0 and
                                   self.gradient_step_num > self.D_init_iters)
            self.generator_step = self.generator_step and self.step % self.grad_accumulation_steps_D >= \
                self.grad_accumulation_steps_D - self.grad_accumulation_steps_G
            if self.generator_step and self.D_verification == 'past' and t.get('D_valid_Steps_4_G_update', 0) > 0:
                n = t['D_valid_Steps_4_G_update']
                self.generator_step = len(self.log_dict['D_logits_diff']) >= n and \
                    all(v[1] > np.log(t['min_D_prob_ratio_4_G']) for v in self.log_dict['D_logits_diff'][-n:]) and \
                    all(v[1] > t['min_mean_D_correct'] for v in self.log_dict['Correctly_distinguished'][-n:])
        if self.D_verification == 'current' and self.generator_step:
            self.generator_step = correct == 1.0 and diff > np.log(t['min_D_prob_ratio_4_G'])
        return self.generator_step

    def _interp_points(self, n):
        """WGAN-GP interpolation points, one per image (SRRaGAN_model.py:388-391, random_pt.uniform_())."""
        return torch.rand(n, 1, 1, 1, device=self.device)

    def optimize_parameters(self):
        """SRRaGAN_model.py:307-575 for the shipped training configuration.

        The x3 overflow checks of the generator's forward and backward (an activation or scaled gradient beyond the
        f16 range, or a weight outside its scale) are not read mid-step, where each read drained the stream and left
        the GPU idle while the host enqueued the discriminator's kernels: the flags are collected on the device
        (train_engine.deferred_overflow_checks) and read once after the whole micro-step is enqueued.  If one was set,
        the micro-step is undone from a device snapshot taken before it (both networks' flat parameters, gradients
        and Adam moments, the discriminator's BatchNorm buffers, the host-side counters, inputs and logs) and redone
        with the generator in exact fp32 — what the eager per-pass check did.  ESR_DEFER_OVERFLOW=0 keeps the eager
        checks."""
        if not DEFER_OVERFLOW or not self.D_exists:
            return self._optimize_step()
        self._flush_logs()  # (free: the previous step's check already synchronised)
        snap = self._snapshot()
        with TE.deferred_overflow_checks() as chk:
            self._optimize_step()
        if chk.overflowed():
            E.OVERFLOW_RERUNS += 1
            self._restore(snap)
            prev = getattr(self._rrdb, 'esr_precision', None)
            self._rrdb.esr_precision = 'f32'
            try:
                with TE.deferred_overflow_checks(on=False):
                    self._optimize_step()
            finally:
                self._rrdb.esr_precision = prev

    _SNAP_ATTRS = ('step', 'gradient_step_num', 'generator_step', 'generator_changed', 'cur_D_update_ratio', 'var_L',
                   'var_H', 'var_ref', 'model_input', 'fake_H', '_d_logs', '_g_logs')

    def _snapshot(self):
        """Everything one micro-step changes (see optimize_parameters): device copies are enqueued, not waited for."""
        host = {k: self.__dict__[k] for k in self._SNAP_ATTRS if k in self.__dict__}
        host['_d_logs_n'] = len(self.__dict__.get('_d_logs') or [])
        host['_g_logs_n'] = {k: len(v) for k, v in (self.__dict__.get('_g_logs') or {}).items()}
        host['_log_n'] = {k: len(v) for k, v in self._log_dict.items()}
        dev = []
        for o in self.optimizers:
            st = o.state.get(o.flat, {})
            dev.append((o, o.flat.data.clone(), o.flat.grad.clone(),
                        {k: (v.clone() if torch.is_tensor(v) else v) for k, v in st.items()}))
        bufs = [(b, b.clone()) for n, b in self.netD.named_buffers()]
        # the RNG streams (the WGAN-GP interpolation points): a redo draws the same points as the undone micro-step
        host['_rng'] = (torch.get_rng_state(),
                        torch.cuda.get_rng_state(self.device) if self.device.type == 'cuda' else None)
        return host, dev, bufs

    def _restore(self, snap):
        host, dev, bufs = snap
        cpu_rng, dev_rng = host['_rng']
        torch.set_rng_state(cpu_rng)
        if dev_rng is not None:
            torch.cuda.set_rng_state(dev_rng, self.device)
        for k in self._SNAP_ATTRS:
            if k in host:
                self.__dict__[k] = host[k]
            else:
                self.__dict__.pop(k, None)
        if host.get('_d_logs') is not None:
            del host['_d_logs'][host['_d_logs_n']:]
        for k, n in host['_g_logs_n'].items():
            del self._g_logs[k][n:]
        self._pending_logs = []  # this micro-step's deferred log values (flushed before the snapshot)
        for k, v in self._log_dict.items():
            del v[host['_log_n'].get(k, 0):]
        with torch.no_grad():
            for o, data, grad, st in dev:
                o.flat.data.copy_(data)
                o.flat.grad.copy_(grad)
                o._sync_views()
                if st:
                    cur = o.state[o.flat]
                    for k, v in st.items():
                        if torch.is_tensor(v):
                            cur[k].copy_(v)
                        else:
                            cur[k] = v
                else:
                    o.state.pop(o.flat, None)
            for b, v in bufs:
                b.copy_(v)

    def _optimize_step(self):
        t = self.opt['train']
        self.gradient_step_num = self.step // self.max_accumulation_steps
        first_acc_G = self.step % self.grad_accumulation_steps_G == 0
        last_acc_G = self.step % self.grad_accumulation_steps_G == self.grad_accumulation_steps_G - 1
        first_acc_D = self.step % self.grad_accumulation_steps_D == 0
        last_acc_D = self.step % self.grad_accumulation_steps_D == self.grad_accumulation_steps_D - 1
        if first_acc_D:
            self.cur_D_update_ratio = self._d_update_ratio(t)
        G_grads_retained = first_acc_D or self.generator_step
        for p in E.param_list(self.netG):
            if not getattr(p, '_esr_frozen', False) and p.requires_grad != G_grads_retained:
                p.requires_grad = G_grads_retained
        if self.CEM_net is not None:
            self.var_H, self.var_ref = self.CEM_net.HR_unpadder(self.var_H), self.CEM_net.HR_unpadder(self.var_ref)
        static_Z = self.GetLatent() if self.latent_input is not None else None
        self.ConcatLatent(LR_image=self.var_L, latent_input=static_Z)
        # the generator's training forward takes the optimiser's flat parameter as its one autograd input (its backward
        # returns the flat gradient, or across ranks writes it in bucket-sized slices: train_engine) instead of 702
        self._rrdb._esr_flat_fwd = self.optimizer_G if G_grads_retained else None
        try:
            self.fake_H = self.netG(self.model_input)
        finally:
            self._rrdb._esr_flat_fwd = None
        if self.CEM_net is not None:
            self.fake_H = self.CEM_net.HR_unpadder(self.fake_H)
        # ---- D step ----
        if not self.D_exists:
            self.generator_step = self.gradient_step_num > 0
        elif self.gradient_step_num % max(1, math.ceil(1 / self.cur_D_update_ratio)) == 0 and \
                self.gradient_step_num > -self.D_init_iters:
            for p in self.netD.parameters():
                p.requires_grad = True
            if first_acc_D:
                self.optimizer_D.zero_grad()
                self._d_logs = []
            pred_d_real = self.netD(self.var_ref)
            pred_d_fake = self.netD(self.fake_H.detach())
            if self.relativistic_D:
                l_d_real = self.cri_gan(pred_d_real - self._batch_mean(pred_d_fake), True)
                l_d_fake = self.cri_gan(pred_d_fake - self._batch_mean(pred_d_real), False)
            else:
                l_d_real = 2 * self.cri_gan(pred_d_real, True)
                l_d_fake = 2 * self.cri_gan(pred_d_fake, False)
            l_d_total = (l_d_real + l_d_fake) / 2
            l_d_gp = None
            if t['gan_type'] == 'wgan-gp':
                rp = self._interp_points(self.var_ref.size(0))
                interp = rp * self.fake_H.detach() + (1 - rp) * self.var_ref
                interp.requires_grad = True
                l_d_gp = self.l_gp_w * self.cri_gp(interp, self.netD(interp))
                l_d_total = l_d_total + l_d_gp
            # [l_d_real, l_d_fake, D_real, D_fake, D_logits_diff, Correctly_distinguished] of this micro-step, the losses
            # (and l_d_gp) averaged over ranks in the statistics' all-reduce
            st = self._d_statistics_t(pred_d_real, pred_d_fake,
                                      (l_d_real, l_d_fake) + ((l_d_gp,) if l_d_gp is not None else ()))
            vals = torch.stack([st[4], st[5], st[2], st[3], st[0], st[1]])
            if l_d_gp is not None:
                l_d_gp_log = st[6]
            if self.D_verification == 'current':  # the gate needs this micro-step's statistics now
                v = vals.tolist()
                self._d_logs.append(v)
                diff, correct = v[4], v[5]
            else:
                self._defer(vals, self._d_logs.append)
                diff = correct = None
            self._gate_generator_step(t, first_acc_D, diff, correct)
            if G_grads_retained and not self.generator_step:
                self.fake_H = self.fake_H.detach()
            if last_acc_D:
                self._d_buckets.arm()  # bucket all-reduces launch from inside this backward
            (l_d_total / self.grad_accumulation_steps_D).backward(retain_graph=self.generator_step)
            if last_acc_D:
                self._d_buckets.finish()
                self.optimizer_D.step()
                _broadcast_buffers(self.netD, self._d_flat_buffers)

                def log_d(_, rows=self._d_logs, g=self.gradient_step_num, ratio=self.cur_D_update_ratio):
                    a = np.mean(np.array(rows), axis=0)
                    for k, v in (('l_d_real', a[0]), ('l_d_fake', a[1]), ('l_d_real_fake', a[0] + a[1]),
                                 ('D_real', a[2]), ('D_fake', a[3]), ('D_logits_diff', a[4]),
                                 ('Correctly_distinguished', a[5]), ('D_update_ratio', ratio)):
                        self._log_dict[k].append((g, float(v)))
                self._defer(None, log_d)
                if l_d_gp is not None:
                    self._defer(l_d_gp_log.reshape(1),
                                lambda v, g=self.gradient_step_num: self._log_dict['l_d_gp'].append((g, v[0])))
        # ---- G step ----
        if self.generator_step:
            if self.D_exists:
                for p in self.netD.parameters():
                    p.requires_grad = False
            if first_acc_G:
                self.optimizer_G.zero_grad()
                self._g_logs = {'l_g_pix': [], 'l_g_range': [], 'l_g_gan': []}
            l_g_total = 0
            if self.cri_pix is not None:  # :477-483
                if self.pixel_domain == 'LR':  # Convert_2_LR (:304-305): bilinear resize to the LR size
                    size = list(self.var_L.size()[-2:])
                    rs = lambda v: torch.nn.functional.interpolate(v, size=size, mode='bilinear')  # noqa: E731
                    l_g_pix = self.cri_pix(rs(self.fake_H), rs(self.var_H))
                else:
                    l_g_pix = self.cri_pix(self.fake_H, self.var_H)
                l_g_total = l_g_total + self.l_pix_w * l_g_pix / self.grad_accumulation_steps_G
            if self.cri_range is not None:
                l_g_range = self.cri_range(self.fake_H)
                l_g_total = l_g_total + self.l_range_w * l_g_range / self.grad_accumulation_steps_G
            if self.D_exists:
                # (the D's forward here fixes the precision of its backward into fake_H, which seeds G's backward)
                prev = D.set_precision(self.d_gstep_precision) if self.d_gstep_precision else None
                try:
                    pred_g_fake = self.netD(self.fake_H)
                finally:
                    if prev is not None:
                        D.set_precision(prev)
                if self.relativistic_D:
                    pred_d_real = self.netD(self.var_ref).detach()
                    l_g_gan = self.l_gan_w * (self.cri_gan(pred_d_real - self._batch_mean(pred_g_fake), False) +
                                              self.cri_gan(pred_g_fake - self._batch_mean(pred_d_real), True)) / 2
                else:
                    l_g_gan = self.l_gan_w * self.cri_gan(pred_g_fake, True)
                l_g_gan = l_g_gan / self.grad_accumulation_steps_G  # logged divided, as the reference (:526, 539)
                l_g_total = l_g_total + l_g_gan
            if last_acc_G:
                self._g_buckets.arm()
            # the flat-gradient fast path (train_engine._GeneratorFn.backward) only for this backward: a full
            # .backward() into every generator parameter; across ranks the backward also launches the G buckets
            # itself as it finalises them (flat-mode GradBuckets as its gradient sink)
            self._rrdb._esr_flat_grad = self.optimizer_G
            self._rrdb._esr_grad_sink = self._g_buckets if (last_acc_G and _world() > 1) else None
            try:
                l_g_total.backward()
            finally:
                self._rrdb._esr_flat_grad = None
                self._rrdb._esr_grad_sink = None
            logged = [(k, v) for k, v in (('l_g_pix', l_g_pix if self.cri_pix is not None else None),
                                          ('l_g_range', l_g_range if self.cri_range is not None else None),
                                          ('l_g_gan', l_g_gan if self.D_exists else None)) if v is not None]
            for (k, _), v in zip(logged, self._global_log_means([v for _, v in logged])):
                self._defer(v.reshape(1), lambda x, rows=self._g_logs[k]: rows.append(x[0]))
            if last_acc_G:
                self._g_buckets.finish()
                if self.latent_input is not None and self.latent_grads_multiplier != 1:  # :543-546
                    for idx, p in zip(self.channels_idx_4_grad_amplification, E.param_list(self.netG)):
                        for c in idx:
                            p.grad[:, c, ...] *= self.latent_grads_multiplier
                self.optimizer_G.step()
                self.generator_changed = True  # :548

                def log_g(_, logs=self._g_logs, g=self.gradient_step_num):
                    for k, v in logs.items():  # means over the accumulated micro-batches (:566-574)
                        if v:
                            self._log_dict[k].append((g, float(np.mean(v))))
                self._defer(None, log_g)
        self.step += 1

    def update_learning_rate(self, cur_step=None):
        """SRRaGAN_model.py:637-683 (the LOSS_BASED branch the reference runs; returns lr_too_low).  Once
        D_logits_diff holds steps_4_loss_std entries, logs D_loss_STD = the std of (l_d_real + l_d_fake) / 2 over the
        entries logged at steps >= cur_step - steps_4_loss_std.  Nothing more happens until the log holds
        2 * steps_4_loss_std entries and its first entry is at least steps_4_loss_std steps old; then, if that std
        exceeds std_4_lr_drop, training rolls back to the newest checkpoint at or before cur_step - steps_4_loss_std
        (weights, optimiser states, step counter and logs), every learning rate becomes lr_gamma × its value before the
        rollback, lr.npz is written and the drop is logged in LR_decrease; True as soon as a learning rate falls below
        1e-8.  The MultiStepLR schedulers (self.schedulers, :236-239) are never stepped here: the reference's
        override replaces base_model's scheduler stepping (train.py steps them itself only without a D)."""
        t = self.opt['train']
        n = t['steps_4_loss_std']
        log = self.log_dict
        reduce_lr = False
        if len(log['D_logits_diff']) >= n:
            vals = [(v[1] + log['l_d_fake'][i][1]) / 2 for i, v in enumerate(log['l_d_real']) if v[0] >= cur_step - n]
            log['D_loss_STD'].append([self.gradient_step_num, np.std(vals)])
            reduce_lr = t.get('std_4_lr_drop') is not None and log['D_loss_STD'][-1][1] > t['std_4_lr_drop']
        if len(log['D_logits_diff']) < 2 * n or log['D_logits_diff'][0][0] > cur_step - n:
            return False
        if reduce_lr:
            cur_lr = [o.param_groups[0]['lr'] for o in self.optimizers]
            self.load(max_step=cur_step - n, resume_train=True)
            for lr, o in zip(cur_lr, self.optimizers):
                for group in o.param_groups:
                    group['lr'] = lr * t['lr_gamma']
                    if group['lr'] < 1e-8:
                        return True
            lr_G, lr_D = self.optimizer_G.param_groups[0]['lr'], self.optimizer_D.param_groups[0]['lr']
            print('LR(D) reduced to %.2e, LR(G) reduced to %.2e.' % (lr_D, lr_G))
            self.save_lr(cur_step)
            self.log_dict['LR_decrease'].append([self.step // self.max_accumulation_steps,
                                                 {'lr_G': lr_G, 'lr_D': lr_D}])
        return False

    def get_current_log(self):
        """SRRaGAN_model.py:685-693: the latest value of every non-empty log series."""
        out = OrderedDict()
        for k, v in self.log_dict.items():
            if len(v) > 0:
                out[k] = v[-1][1] if isinstance(v[-1], tuple) or len(v[-1]) > 1 else v[-1]
        return out

    def get_current_learning_rate(self):
        """base_model.py:44-45."""
        return self.optimizers[0].param_groups[0]['lr']

    def display_log_figure(self):
        """base_model.py:160-215 plots the logs with matplotlib: out of scope here (no-op)."""

    def perform_validation(self, data_loader, cur_Z, print_rlt, save_GT_HR, save_images):
        """SRRaGAN_model.py:586-635: batch-1 `test()` of every validation image with latent value cur_Z, PSNR of
        the 0-255 float images (utils/util.py:80-104 tensor2img, :168-175 calculate_psnr) averaged into
        print_rlt['psnr']; with save_images, the centre crops (the smallest HR size - 2) of the SR (and, with
        save_GT_HR, the HR) images as a collage PNG under path.val_images.  Returns the SR images (HWC BGR float32
        0-255)."""
        psnrs, sr_images, collage, gt_collage = [], [], [], []
        if save_images:
            n_img = len(data_loader.dataset)
            rows = int(np.floor(np.sqrt(n_img)))
            while rows > 1 and np.round(n_img / rows) != n_img / rows:
                rows -= 1
            patch = min([min(im['HR'].shape[1:]) for im in data_loader.dataset]) - 2
        for idx, val_data in enumerate(data_loader):
            if save_images and idx % rows == 0:
                collage.append([])
                gt_collage.append([])
            val_data['Z'] = cur_Z
            self.feed_data(val_data)
            self.test()
            visuals = self.get_current_visuals()
            sr_img = 255 * _tensor2img(visuals['SR'])
            gt_img = 255 * _tensor2img(visuals['HR'])
            sr_images.append(sr_img)
            psnrs.append(_psnr(sr_img, gt_img))
            if save_images:
                m = ((np.array(sr_img.shape[:2]) - patch) / 2).astype(np.int32)
                crop = lambda im: np.clip(im[m[0]:-m[0], m[1]:-m[1], ...], 0, 255).astype(np.uint8)  # noqa: E731
                collage[-1].append(crop(sr_img))
                if save_GT_HR:
                    gt_collage[-1].append(crop(gt_img))
        avg_psnr = float(np.mean(psnrs))
        if save_images:
            out_dir = self.opt['path']['val_images']
            latent = self.opt['network_G'].get('latent_input')
            _save_png(np.concatenate([np.concatenate(c, 0) for c in collage], 1), os.path.join(
                out_dir, '{:d}_{}PSNR{:.3f}.png'.format(self.gradient_step_num, ('Z' + str(cur_Z)) if latent else '',
                                                        avg_psnr)))
            if save_GT_HR:
                _save_png(np.concatenate([np.concatenate(c, 0) for c in gt_collage], 1),
                          os.path.join(out_dir, 'GT_HR.png'))
        print_rlt['psnr'] += avg_psnr
        return sr_images

    # ------------------------------------------------------------------------------------------------------------------
    def test(self, prevent_grads_calc=True):
        """SRRaGAN_model.py:577-584 (leaves the net in train mode afterwards, like the reference)."""
        self.netG.eval()
        if prevent_grads_calc:
            with torch.no_grad():
                self.fake_H = self.netG(self.model_input)
        else:
            self.fake_H = self.netG(self.model_input)
        self.netG.train()

    def get_current_visuals(self, need_HR=True, entire_batch=False):
        out = OrderedDict()
        sel = slice(None) if entire_batch else 0
        out['LR'] = self.var_L.detach()[sel].float().cpu()
        out['SR'] = self.fake_H.detach()[sel].float().cpu()
        if need_HR:
            out['HR'] = self.var_H.detach()[sel].float().cpu()
        return out

    # ------------------------------------------------------------------------------------------------------------------
    # checkpoints and logs (base_model.py:86-144; SRRaGAN_model.py:695-719, 766-813)
    # ------------------------------------------------------------------------------------------------------------------
    def save_network(self, save_dir, network, network_label, iter_label, optimizer):
        """base_model.py:86-97: `{iter}_{label}.pth` = {'model_state_dict' (CPU tensors), 'optimizer_state_dict'}."""
        path = os.path.join(save_dir, '{}_{}.pth'.format(iter_label, network_label))
        if hasattr(network, 'module'):
            network = network.module
        sd = network.state_dict()
        for k in sd:
            sd[k] = sd[k].cpu()
        torch.save({'model_state_dict': sd, 'optimizer_state_dict': optimizer.state_dict()}, path)
        return path

    def load_network(self, load_path, network, strict=False, optimizer=None):
        """base_model.py:100-111.  Plain state dicts (pretrained ESRGAN files) and {model, optimizer} dicts both load;
        the file is read with torch.load(weights_only=True) (no pickled code is executed)."""
        if hasattr(network, 'module'):
            network = network.module
        loaded = torch.load(load_path, map_location='cpu', weights_only=True)
        if 'optimizer_state_dict' in loaded:
            if optimizer is not None:
                optimizer.load_state_dict(loaded['optimizer_state_dict'])
            loaded = loaded['model_state_dict']
        if self.CEM_arch:
            loaded = CEMnet.Adjust_State_Dict_Keys(loaded, network.state_dict())
        loaded = self.process_loaded_state_dict(loaded_state_dict=loaded, current_state_dict=network.state_dict())
        network.load_state_dict(loaded, strict=strict)  # bumps the parameter versions: packed weights refresh

    def process_loaded_state_dict(self, loaded_state_dict, current_state_dict):
        """base_model.py:113-144: keys are matched by POSITION (old non-ModuleList checkpoints have other names; the
        shapes must agree up to the input-channel dim).  A weight whose current input-channel count is the loaded one
        plus num_latent_channels (× 1 or × scale²) gets zero weights prepended for the latent channels
        (LATENT_WEIGHTS_RELATIVE_STD = 0) and its channels recorded for latent gradient amplification.  CEM filter
        weights are never loaded (the current design is kept)."""
        out = collections.OrderedDict()
        cur_keys = list(current_state_dict.keys())
        assert len(cur_keys) == len(loaded_state_dict), 'Loaded model and current one should have the same number of ' \
                                                        'parameters'
        renamed = 0
        op_names = getattr(self.CEM_net, 'OP_names', []) if self.CEM_net is not None else []
        for i, key in enumerate(loaded_state_dict.keys()):
            ck = cur_keys[i]
            lv, cv = loaded_state_dict[key], current_state_dict[ck]
            ls, cs = tuple(lv.size()), tuple(cv.size())
            if key != ck:
                assert ls[:1] + ls[2:] == cs[:1] + cs[2:], 'Unmatching parameter sizes after changing parameter key name'
                renamed += 1
            if self.latent_input is not None and 'weight' in key and lv.dim() > 1 and \
                    cs[1] in list(ls[1] + self.num_latent_channels * np.array([1, self.opt['scale'] ** 2])):
                extra = cs[1] - ls[1]
                # the reference's expression (base_model.py:130-134): 0 x (loaded std / current std) x current
                # weights, so the prepended zeros carry the current weights' signs (and NaN if their std is 0)
                cur = cv[:, :extra].detach().cpu()
                out[ck] = torch.cat([LATENT_WEIGHTS_RELATIVE_STD * lv.std() / cur.std() * cur.to(lv.dtype),
                                     lv.cpu()], 1)
                if hasattr(self, 'channels_idx_4_grad_amplification'):
                    self.channels_idx_4_grad_amplification[i] = list(range(extra))
            elif self.CEM_arch and any(op in key for op in op_names):
                continue
            else:
                out[ck] = lv
        if renamed:
            warnings.warn('Modified %d key names due to the change to using ModuleLists' % renamed)
        return out

    @staticmethod
    def _step_of(name):
        return int(re.search(r'(\d)+(?=_G.pth)', name).group(0))

    def load(self, max_step=None, resume_train=None):
        """SRRaGAN_model.py:766-805: the latest (or latest <= max_step) `{step}_G.pth` under path.models when resuming
        or testing, else path.pretrain_model_G / _D."""
        resume = resume_train if resume_train is not None else (self.is_train and self.opt['train'].get('resume'))
        paths = self.opt.get('path') or {}
        if max_step is not None or resume or not self.is_train:
            if not self.is_train and not (self.save_dir and os.path.isdir(self.save_dir) and
                                          any('_G.pth' in n for n in os.listdir(self.save_dir))):
                return  # built programmatically (GUI / Z_optimizer / tests) with no checkpoint directory to load
            names = sorted([n for n in os.listdir(self.save_dir) if '_G.pth' in n], key=self._step_of)
            if max_step is not None:
                names = [n for n in names if self._step_of(n) <= max_step]
            name = names[-1]
            step = self._step_of(name)
            if self.is_train:
                self.step = (step + 1) * self.max_accumulation_steps
                self.load_network(os.path.join(self.save_dir, name), self.netG, optimizer=self.optimizer_G)
                if self.log_path and os.path.isfile(os.path.join(self.log_path, 'logs.npz')):
                    self.load_log(max_step=step)
                if self.D_exists:
                    self.load_network(os.path.join(self.save_dir, '%d_D.pth' % step), self.netD,
                                      optimizer=self.optimizer_D)
            else:
                self.load_network(os.path.join(self.save_dir, name), self.netG)
                if getattr(self, 'netD', None) is not None:
                    self.load_network(os.path.join(self.save_dir, name.replace('_G', '_D')), self.netD)
                self.gradient_step_num = step
        else:
            if paths.get('pretrain_model_G') is not None:
                self.load_network(paths['pretrain_model_G'], self.netG)
            if self.is_train and paths.get('pretrain_model_D') is not None and getattr(self, 'netD', None) is not None:
                self.load_network(paths['pretrain_model_D'], self.netD, optimizer=self.optimizer_D)

    def save(self, iter_label):
        """SRRaGAN_model.py:807-813."""
        path = self.save_network(self.save_dir, self.netG, 'G', iter_label, self.optimizer_G)
        if getattr(self, 'D_exists', False):
            self.save_network(self.save_dir, self.netD, 'D', iter_label, self.optimizer_D)
        return path

    def save_log(self):
        """SRRaGAN_model.py:695-698: logs.npz, one array of (step, value) rows per log key (LR_decrease's
        [step, {lr_G, lr_D}] rows as the object array the reference writes; load_log skips it: it needs unpickling)."""
        arrays = {}
        for k, v in self.log_dict.items():
            if any(isinstance(r[1], dict) for r in v):
                arrays[k] = np.array([[r[0], r[1]] for r in v], dtype=object)
            else:
                arrays[k] = np.asarray(v, dtype=np.float64).reshape(-1, 2)
        np.savez(os.path.join(self.log_path, 'logs.npz'), **arrays)

    def save_lr(self, step_num):
        """The lr.npz the reference writes when it decays the learning rates (SRRaGAN_model.py:676-681), read back by
        the optimizer set-up of a resumed run."""
        np.savez(os.path.join(self.log_path, 'lr.npz'), step_num=step_num, lr_G=self.optimizer_G.param_groups[0]['lr'],
                 lr_D=self.optimizer_D.param_groups[0]['lr'])

    def load_log(self, max_step=None):
        """SRRaGAN_model.py:700-714 (logs entries the reference stored as pickled objects are skipped: the file is read
        with allow_pickle=False)."""
        self.log_dict = OrderedDict((k, []) for k in self.log_dict)
        with np.load(os.path.join(self.log_path, 'logs.npz')) as f:
            for key in f.files:
                try:
                    arr = f[key]
                except ValueError:
                    warnings.warn('logs.npz: skipping %r (object array)' % key)
                    self.log_dict[key] = []
                    continue
                rows = [tuple(r) for r in np.asarray(arr).reshape(len(arr), -1).tolist()] if len(arr) else []
                if max_step is not None:
                    rows = [r for r in rows if r[0] <= max_step]
                self.log_dict[key] = rows


def _tensor2img(t):
    """utils/util.py:80-104 for a CHW tensor, out_type float32: clamp to [0, 1], HWC, BGR."""
    a = t.squeeze().float().cpu().clamp_(0, 1).numpy()
    if a.ndim == 3:
        a = np.transpose(a[[2, 1, 0], :, :], (1, 2, 0))
    return a.astype(np.float32)


def _psnr(img1, img2):
    """utils/util.py:168-175 (images in [0, 255])."""
    mse = np.mean((img1.astype(np.float64) - img2.astype(np.float64)) ** 2)
    return float('inf') if mse == 0 else 20 * math.log10(255.0 / math.sqrt(mse))


def _save_png(img, path):
    """cv2.imwrite of an HWC BGR (or HW gray) uint8 image (utils/util.py:107-108), as an 8-bit RGB/gray PNG written
    with zlib (OpenCV is not a dependency here)."""
    img = np.ascontiguousarray(img[..., ::-1] if img.ndim == 3 else img, dtype=np.uint8)
    h, w = img.shape[:2]
    color = 2 if img.ndim == 3 else 0
    raw = b''.join(b'\x00' + img[r].tobytes() for r in range(h))

    def chunk(tag, data):
        return struct.pack('>I', len(data)) + tag + data + struct.pack('>I', zlib.crc32(tag + data) & 0xffffffff)
    with open(path, 'wb') as f:
        f.write(b'\x89PNG\r\n\x1a\n' + chunk(b'IHDR', struct.pack('>IIBBBBB', w, h, 8, color, 0, 0, 0)) +
                chunk(b'IDAT', zlib.compress(raw, 6)) + chunk(b'IEND', b''))
