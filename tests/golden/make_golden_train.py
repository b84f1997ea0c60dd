"""Golden fixtures for the training loop and the checkpoint formats, made by running the REFERENCE's own
SRRaGANModel (read-only at /root/reference) in this container.  Run once here; only the small outputs are committed.

    python tests/golden/make_golden_train.py

Uses the in-memory shims of make_golden.py plus, for importing models/SRRaGAN_model.py:
  * stub modules for what its imports pull in but the training step never calls (torchvision.utils, GPUtil,
    skimage.transform, skimage.color): attribute access returns a function that raises if called;
  * `networks.define_D` builds Discriminator_VGG_128_(nb=n_layers) — the shipped `discriminator_vgg_128` + n_layers
    combination passes nb= to a class without it; this is the class DESIGN.md pins the port's D to;
  * `torch.Tensor.cuda` is the identity while process_loaded_state_dict runs (base_model.py:133-135 moves the
    latent-widened weights to CUDA; this container has no GPU);
  * the WGAN-GP interpolation points (SRRaGAN_model.py:391, `self.random_pt.uniform_()`) are drawn from a NumPy PCG64
    stream instead of torch's CPU generator, so that the GPU test can feed the port the same points.
Fixtures (tests/golden/):
  train_*.npz  — per micro-step generator_step flags, every log_dict series, and digests of the G/D parameter updates
                 (per-key L2 norms of the final parameters and of their change, projections of the change on a seeded
                 random direction, the full change of the small keys), for the reference run in float32 and float64
                 (the float64 run is the accuracy yardstick: the port's error is judged against the reference's own
                 float32 error, as conftest.grad_parity does for gradients).
  ckpt_remap.npz — base_model.load_network + process_loaded_state_dict of a plain (no latent, no CEM prefix) RRDBNet
                 state dict into the latent CEM generator: output key order, per-key SHA-256, the gradient-amplified
                 channel lists.
  lr_schedule.npz — SRRaGAN_model.update_learning_rate driven per gradient step as train.py:187-189 does
                 (train_recipe.drive_lr_schedule): the D_loss_STD log, the std_4_lr_drop test, the rollback through
                 load(max_step=cur_step-steps_4_loss_std, resume_train=True), the LR x lr_gamma, lr.npz, LR_decrease and
                 the lr_too_low return.
  ckpt/7_G.pth — written by base_model.save_network (model_state_dict on the CPU + Adam optimizer_state_dict with
                 state for three parameters), read back by the test with torch.load(weights_only=True).
"""
import hashlib
import json
import os
import sys
import types

sys.dont_write_bytecode = True
sys.pycache_prefix = '/tmp/esr_golden_pycache'

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
from oracle.recipe import seeded_params  # noqa: E402
from train_recipe import (C3_GRID_CFG, CKPT_CFG, LR_CFG, TRAIN_CFGS, VAL_CFG, VAL_ZS, drive_lr_schedule,  # noqa: E402
                          grad_projections, random_points, step_data, train_opt, val_items)

SMALL = 4096  # keys with at most this many elements get their full parameter change stored


class _Stub(types.ModuleType):
    __path__ = []

    def __getattr__(self, k):
        if k.startswith('__'):
            raise AttributeError(k)

        def f(*a, **kw):
            raise RuntimeError('stub %s.%s called' % (self.__name__, k))
        return f


def _stub(name):
    m = _Stub(name)
    sys.modules[name] = m
    parent, _, child = name.rpartition('.')
    if parent in sys.modules:
        setattr(sys.modules[parent], child, m)


def install_train_shims():
    MG.install_shims()
    sys.modules.pop('torchvision', None)
    for n in ('torchvision', 'torchvision.utils', 'GPUtil', 'skimage', 'skimage.transform', 'skimage.color'):
        _stub(n)


class FixedRP(torch.Tensor):
    """random_pt whose uniform_() takes the next row of a preset NumPy stream (results of ops are plain tensors)."""
    __torch_function__ = torch._C._disabled_torch_function_impl
    stream = None

    def uniform_(self, *a, **k):
        v = next(FixedRP.stream)
        with torch.no_grad():
            self.copy_(torch.from_numpy(v).to(self.dtype).view(self.shape))
        return self


def build_reference(cfg, dtype):
    import models.networks as networks
    import models.modules.architecture as arch
    import models.SRRaGAN_model as R

    def define_D(opt, CEM=None):
        o = opt['network_D']
        patch = opt['datasets']['train']['patch_size'] - (2 * CEM.invalidity_margins_HR if CEM is not None else 0)
        D = arch.Discriminator_VGG_128_(in_nc=o['in_nc'], base_nf=o['nf'], norm_type=o['norm_type'],
                                        act_type=o['act_type'], mode=o['mode'], input_patch_size=patch,
                                        nb=o['n_layers'])
        networks.init_weights(D, init_type='kaiming', scale=1)
        return D
    networks.define_D = define_D
    R.networks.define_D = define_D
    os.makedirs('/tmp/esr_golden_train_models', exist_ok=True)
    # the reference's constructor resumes the learning rates from <log>/lr.npz (SRRaGAN_model.py:212-216): never let
    # one left by the lr_schedule fixture leak into a training fixture
    for f in ('/tmp/esr_golden_train_log/lr.npz', '/tmp/esr_golden_train_log/logs.npz'):
        if os.path.exists(f):
            os.remove(f)
    torch.set_default_dtype(dtype)
    torch.cuda.FloatTensor = torch.DoubleTensor if dtype == torch.float64 else torch.FloatTensor
    try:
        model = R.SRRaGANModel(train_opt(cfg), accumulation_steps_per_batch=cfg['acc'])
    finally:
        torch.set_default_dtype(torch.float32)
    gsd, dsd = model.netG.state_dict(), model.netD.state_dict()
    gp = seeded_params([(k, tuple(v.shape)) for k, v in gsd.items()], cfg['seed'], w_scale=cfg.get('w_scale_G', 1.0))
    dp = seeded_params([(k, tuple(v.shape)) for k, v in dsd.items() if 'running' not in k and 'num_batches' not in k],
                       cfg['seed'] + 1, w_scale=1.0)
    model.netG.load_state_dict({k: torch.from_numpy(v) for k, v in gp.items()}, strict=False)
    model.netD.load_state_dict({k: torch.from_numpy(v) for k, v in dp.items()}, strict=False)
    if dtype == torch.float64:
        model.netG.double()
        model.netD.double()
    # optimisers were built over the same Parameter objects; the load copied into them in place
    B = cfg['batch']
    model.random_pt = torch.zeros(B, 1, 1, 1, dtype=dtype).as_subclass(FixedRP)
    return model


def run_reference(cfg, dtype, perturb=None):
    """perturb = seed: every G and D parameter multiplied by (1 + 2^-24·N(0,1)) before the run — a rounding-level
    kick, to sample how far the reference's own float32 trajectory moves under perturbations of that size."""
    model = build_reference(cfg, dtype)
    if perturb is not None:
        gen = torch.Generator().manual_seed(perturb)
        with torch.no_grad():
            for p in list(model.netG.parameters()) + list(model.netD.parameters()):
                p.mul_(1 + 2.0 ** -24 * torch.randn(p.shape, generator=gen, dtype=p.dtype))
    g0 = {k: v.detach().clone() for k, v in model.netG.named_parameters()}
    d0 = {k: v.detach().clone() for k, v in model.netD.named_parameters()}
    FixedRP.stream = random_points(cfg)
    flags = []
    for k in range(cfg['steps']):
        lr, hr, z = step_data(cfg, k)
        cast = lambda a: torch.from_numpy(a).to(dtype)  # noqa: E731
        model.feed_data({'LR': cast(lr), 'HR': cast(hr), 'Z': cast(z)})
        model.optimize_parameters()
        flags.append(bool(model.generator_step))
    return model, g0, d0, flags


def digest(prefix, final, init, d, proj_seed):
    rng = np.random.default_rng(proj_seed)
    for k in final:
        f = final[k].detach().double().numpy()
        delta = f - init[k].double().numpy()
        p = rng.standard_normal(f.shape)
        d['%s_norm:%s' % (prefix, k)] = np.float64(np.linalg.norm(f))
        d['%s_dnorm:%s' % (prefix, k)] = np.float64(np.linalg.norm(delta))
        d['%s_dproj:%s' % (prefix, k)] = np.float64((p * delta).sum())
        if f.size <= SMALL:
            d['%s_delta:%s' % (prefix, k)] = delta.astype(np.float64)


# float32 reference runs from rounding-level perturbed weights (f32p0 ..): the loop test takes the largest float32
# distance to the float64 run over them and the plain run as its yardstick (the plain f32 / f64 entries are unchanged
# by adding them: regenerated bit for bit).
N_PERTURBED = int(os.environ.get('ESR_GOLDEN_PERTURBED', '6'))


def train_fixture(name, cfg):
    d = {'cfg': np.str_(json.dumps(cfg))}
    runs = [('f32', torch.float32, None), ('f64', torch.float64, None)] + \
        [('f32p%d' % i, torch.float32, 7000 + i) for i in range(N_PERTURBED)]
    for tag, dtype, perturb in runs:
        model, g0, d0, flags = run_reference(cfg, dtype, perturb)
        d['%s_generator_step' % tag] = np.array(flags)
        for k, v in model.log_dict.items():
            if v:
                d['%s_log:%s' % (tag, k)] = np.array(v, dtype=np.float64)
        digest(tag + '_G', dict(model.netG.named_parameters()), g0, d, cfg['seed'] + 400)
        digest(tag + '_D', dict(model.netD.named_parameters()), d0, d, cfg['seed'] + 401)
        for k, v in model.netD.state_dict().items():
            if 'running' in k:
                d['%s_Dbuf:%s' % (tag, k)] = v.double().numpy()
        print('train_%s [%s]: generator_step %s, logs %s' % (
            name, tag, flags, {k: ['%.4g' % x[1] for x in v] for k, v in model.log_dict.items() if v}))
    np.savez_compressed(os.path.join(HERE, 'train_%s.npz' % name), **d)


def c3_grid_fixture():
    """Config 3 at its production grid (train_recipe.C3_GRID_CFG), float64 then float32, one model at a time.  The
    reference's RRDB.forward (block.py:262-270) runs under torch.utils.checkpoint so that the float64 generator's
    activations fit this container's memory (~75 GB without): the same ops on the same values, recomputed in the
    backward — a memory-only wrapper, the results are the reference's own."""
    import gc
    import torch.utils.checkpoint as ckpt
    import models.modules.block as blk
    if not getattr(blk.RRDB, '_esr_ckpt', False):
        fwd = blk.RRDB.forward
        blk.RRDB.forward = lambda self, x: ckpt.checkpoint(fwd, self, x, use_reentrant=False)
        blk.RRDB._esr_ckpt = True
    cfg = dict(C3_GRID_CFG)
    d = {'cfg': np.str_(json.dumps(cfg))}
    for tag, dtype in (('f64', torch.float64), ('f32', torch.float32)):
        model, g0, d0, flags = run_reference(cfg, dtype)
        d['%s_generator_step' % tag] = np.array(flags)
        for k, v in model.log_dict.items():
            if v:
                d['%s_log:%s' % (tag, k)] = np.array(v, dtype=np.float64)
        for net, t in ((model.netG, 'G'), (model.netD, 'D')):
            for i, (k, p) in enumerate(net.named_parameters()):
                if p.grad is None:
                    continue
                g = p.grad.detach().double().numpy()
                d['%s_%s_gproj:%s' % (tag, t, k)] = grad_projections(g, cfg['seed'] + (10 if t == 'G' else 11), i,
                                                                     cfg['proj'])
                d['%s_%s_gnorm:%s' % (tag, t, k)] = np.float64(np.linalg.norm(g))
        for k, v in model.netD.state_dict().items():
            if 'running' in k:
                d['%s_Dbuf:%s' % (tag, k)] = v.double().numpy()
        print('c3_grid [%s]: generator_step %s, logs %s' % (
            tag, flags, {k: ['%.6g' % x[1] for x in v] for k, v in model.log_dict.items() if v}), flush=True)
        del model, g0, d0
        gc.collect()
    np.savez_compressed(os.path.join(HERE, 'grid_c3_train.npz'), **d)


def c3_grid_perturbed(n=None):
    """Adds n rounding-perturbed float32 runs of the reference (run_reference(perturb=7100 + i): every G and D
    parameter × (1 + 2^-24·N(0,1))) to grid_c3_train.npz as f32p<i>_* entries (gradient projections, logs, D buffers),
    leaving the f64 / f32 entries as they are.  tests/grid_parity.py then bounds each quantity by FACTOR × the
    LARGEST float32 distance to the float64 run over the plain and the perturbed runs: the spread of the reference's
    own float32 result under rounding-level changes, which is what a legal summation order amounts to (VERDICT r4
    weak #1: a single float32 sample is noise for the near-cancelling bias gradients)."""
    import gc
    import torch.utils.checkpoint as ckpt
    import models.modules.block as blk
    if not getattr(blk.RRDB, '_esr_ckpt', False):
        fwd = blk.RRDB.forward
        blk.RRDB.forward = lambda self, x: ckpt.checkpoint(fwd, self, x, use_reentrant=False)
        blk.RRDB._esr_ckpt = True
    n = int(os.environ.get('ESR_GOLDEN_PERTURBED', '4')) if n is None else n
    path = os.path.join(HERE, 'grid_c3_train.npz')
    d = dict(np.load(path))
    cfg = json.loads(str(d['cfg']))
    for i in range(n):
        tag = 'f32p%d' % i
        if any(k.startswith(tag + '_') for k in d):
            continue
        model, g0, d0, flags = run_reference(cfg, torch.float32, 7100 + i)
        d['%s_generator_step' % tag] = np.array(flags)
        for k, v in model.log_dict.items():
            if v:
                d['%s_log:%s' % (tag, k)] = np.array(v, dtype=np.float64)
        for net, t in ((model.netG, 'G'), (model.netD, 'D')):
            for j, (k, p) in enumerate(net.named_parameters()):
                if p.grad is None:
                    continue
                d['%s_%s_gproj:%s' % (tag, t, k)] = grad_projections(
                    p.grad.detach().double().numpy(), cfg['seed'] + (10 if t == 'G' else 11), j, cfg['proj'])
        for k, v in model.netD.state_dict().items():
            if 'running' in k:
                d['%s_Dbuf:%s' % (tag, k)] = v.double().numpy()
        print('c3_grid [%s]: generator_step %s' % (tag, flags), flush=True)
        del model, g0, d0
        gc.collect()
        np.savez_compressed(path, **d)  # after every run: a long job keeps what it has made


def _sha(t):
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()


def checkpoint_fixtures():
    """base_model.py:86-144 on the reference model: load a plain checkpoint into the latent CEM generator; write a
    {step}_G.pth."""
    import models.modules.architecture as arch
    cfg = dict(CKPT_CFG)
    model = build_reference(cfg, torch.float32)
    plain = arch.RRDBNet(in_nc=3, out_nc=3, nf=64, nb=cfg['nb'], gc=32, upscale=4, norm_type=None,
                         act_type='leakyrelu', mode='CNA', upsample_mode='upconv', latent_input=None,
                         num_latent_channels=0)
    psd = seeded_params([(k, tuple(v.shape)) for k, v in plain.state_dict().items()], 900, w_scale=1.0)
    path = '/tmp/esr_golden_plain_G.pth'
    torch.save({k: torch.from_numpy(v) for k, v in psd.items()}, path)
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self
    try:
        model.load_network(path, model.netG)
    finally:
        torch.Tensor.cuda = cuda
    sd = model.netG.state_dict()
    d = dict(keys=np.str_(json.dumps(list(sd.keys()))), sha=np.str_(json.dumps({k: _sha(v) for k, v in sd.items()})),
             amplified=np.str_(json.dumps(model.channels_idx_4_grad_amplification)), plain_seed=np.int64(900),
             cfg=np.str_(json.dumps(cfg)))
    np.savez_compressed(os.path.join(HERE, 'ckpt_remap.npz'), **d)
    print('ckpt_remap: %d keys, %d amplified' % (len(sd), sum(1 for c in model.channels_idx_4_grad_amplification if c)))
    # save_network after one Adam step on three small parameters (optimizer state for those only)
    model = build_reference(cfg, torch.float32)
    names = ['generated_image_model.model.0.bias', 'generated_image_model.model.4.bias',
             'generated_image_model.model.6.bias']
    named = dict(model.netG.named_parameters())
    rng = np.random.default_rng(901)
    model.optimizer_G.zero_grad()
    for n in names:
        named[n].grad = torch.from_numpy(rng.standard_normal(tuple(named[n].shape)).astype(np.float32))
    model.optimizer_G.step()
    os.makedirs(os.path.join(HERE, 'ckpt'), exist_ok=True)
    p = model.save_network(os.path.join(HERE, 'ckpt'), model.netG, 'G', 7, model.optimizer_G)
    ref = {n: named[n].detach().numpy() for n in names}
    st = model.optimizer_G.state_dict()
    np.savez_compressed(os.path.join(HERE, 'ckpt_save.npz'), names=np.str_(json.dumps(names)),
                        param_seed=np.int64(cfg['seed']), cfg=np.str_(json.dumps(cfg)),
                        **{'after:' + n: v for n, v in ref.items()},
                        **{'exp_avg:%d' % i: s['exp_avg'].numpy() for i, s in st['state'].items()},
                        **{'exp_avg_sq:%d' % i: s['exp_avg_sq'].numpy() for i, s in st['state'].items()})
    print('ckpt_save: %s (%d bytes), state for params %s' % (p, os.path.getsize(p), sorted(st['state'])))


class ValLoader:
    """What train.py's val_loader hands perform_validation: batch-1 dicts and .dataset (CHW tensors)."""
    def __init__(self, items):
        self.dataset = [{'LR': torch.from_numpy(it['LR']), 'HR': torch.from_numpy(it['HR']), 'HR_path': it['HR_path']}
                        for it in items]

    def __len__(self):
        return len(self.dataset)

    def __iter__(self):
        for it in self.dataset:
            yield {'LR': it['LR'][None], 'HR': it['HR'][None], 'HR_path': [it['HR_path']]}


def validation_fixture():
    """The reference's own perform_validation (SRRaGAN_model.py:586-635) for three latent values: the returned SR
    images (HWC BGR float32 0-255) and print_rlt['psnr'] after each call (save_images off: its PNG writer is cv2)."""
    cfg = dict(VAL_CFG)
    model = build_reference(cfg, torch.float32)
    loader = ValLoader(val_items())
    rlt = {'psnr': 0}
    d = {'cfg': np.str_(json.dumps(cfg)), 'zs': np.array(VAL_ZS, dtype=np.float64)}
    for z in VAL_ZS:
        srs = model.perform_validation(loader, z, rlt, save_GT_HR=False, save_images=False)
        d['psnr_after:%g' % z] = np.float64(rlt['psnr'])
        for i, sr in enumerate(srs):
            d['sr:%g:%d' % (z, i)] = np.asarray(sr, dtype=np.float32)
        print('validation Z=%g: psnr sum %.6f, SR shapes %s' % (z, rlt['psnr'], [s.shape for s in srs]))
    np.savez_compressed(os.path.join(HERE, 'validation.npz'), **d)


def lr_schedule_fixture():
    import shutil
    cfg = dict(LR_CFG)
    for d in ('/tmp/esr_golden_train_models', '/tmp/esr_golden_train_log'):
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d)
    model = build_reference(cfg, torch.float32)
    records, dec = drive_lr_schedule(model, cfg)
    with np.load('/tmp/esr_golden_train_log/lr.npz') as f:
        lr_file = np.array([f['step_num'], f['lr_G'], f['lr_D']], dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, 'lr_schedule.npz'), cfg=np.str_(json.dumps(cfg)), records=records,
                        lr_decrease=dec, lr_file=lr_file)
    print('lr_schedule: %d calls, returns %s, LR_decrease %s, lr.npz %s' % (
        len(records), records[:, 1].tolist(), dec.tolist(), lr_file.tolist()))


def main():
    install_train_shims()
    torch.set_num_threads(8)
    which = sys.argv[1:] or list(TRAIN_CFGS) + ['ckpt', 'lr']
    for name in which:
        if name == 'ckpt':
            checkpoint_fixtures()
        elif name == 'lr':
            lr_schedule_fixture()
        elif name == 'val':
            validation_fixture()
        elif name == 'c3':
            c3_grid_fixture()
        elif name == 'c3p':
            c3_grid_perturbed()
        else:
            train_fixture(name, TRAIN_CFGS[name])


if __name__ == '__main__':
    main()
