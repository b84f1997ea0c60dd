"""The data-parallel training step (config 4's path: one process per GPU, SRRaGAN_model.GradBuckets all-reducing the G
and D gradients from inside the backward, the D statistics that steer generator_step all-reduced, BN buffers from
rank 0) with the real HIP kernels: two ranks sharing the box's one GPU over gloo (RCCL needs one GPU per rank; the
driver's 8-GPU run takes the same code path with the nccl backend).  The reference's counterpart is
nn.DataParallel over the GPUs (models/networks.py:99-101,125-126) with batch_size *= nGPU (options/options.py:85-87).

* identical batches on both ranks: the ranks agree bit for bit, and they agree with the single-process run to
  rounding level.  Asserted thresholds: the averaged gradient of each optimiser's FIRST step within 1e-5 relative L2
  of the single-process one; every parameter after the 6 micro-steps within 1e-3 relative L2 (Adam amplifies
  rounding-level gradient differences into lr-sized steps for elements whose gradient is ~0; run to run the two-rank
  step is not bitwise reproducible, ~1e-7 relative in the weights); the biases of the discriminator convs that feed a
  BatchNorm within 2·lr·steps absolute (their gradient is analytically zero, its computed value the rounding noise
  of a cancelling sum, observed 1e-3..6e-1 relative), and the BN running means, which carry those biases, within
  1e-3 relative or that absolute bound;
* different batches per rank: the ranks end with the same parameters and took the same generator_step decisions.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
if os.path.join(HERE, 'golden') not in __import__('sys').path:
    __import__('sys').path.insert(0, os.path.join(HERE, 'golden'))


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cfg_name, same_data, q):
    import sys
    for p_ in (HERE, os.path.join(HERE, 'golden'), os.path.dirname(HERE),
               os.path.join(os.path.dirname(HERE), 'explorable-super-resolution_old_amd')):
        if p_ not in sys.path:
            sys.path.insert(0, p_)
    import torch.distributed as dist
    from train_recipe import TRAIN_CFGS, random_points, step_data, train_opt
    from oracle.recipe import seeded_params
    from esr_amd import dconv, engine
    from esr_amd.SRRaGAN_model import SRRaGANModel
    try:
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        if world > 1:
            os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
            dist.init_process_group('gloo', rank=rank, world_size=world)
        if os.environ.get('DDP_PROBE_NANFILL') == '1':  # diagnostic: every torch.empty filled with NaN
            torch.use_deterministic_algorithms(True, warn_only=True)
            torch.utils.deterministic.fill_uninitialized_memory = True
        cfg = dict(TRAIN_CFGS[cfg_name])
        torch.manual_seed(0)
        model = SRRaGANModel(train_opt(cfg), accumulation_steps_per_batch=cfg['acc'], device=dev)
        gsd, dsd = model.netG.state_dict(), model.netD.state_dict()
        gp = seeded_params([(k, tuple(v.shape)) for k, v in gsd.items()], cfg['seed'], w_scale=1.0)
        dp = seeded_params([(k, tuple(v.shape)) for k, v in dsd.items() if 'running' not in k and 'num_batches' not in k],
                           cfg['seed'] + 1, w_scale=1.0)
        model.netG.load_state_dict({k: torch.from_numpy(v) for k, v in gp.items()}, strict=False)
        model.netD.load_state_dict({k: torch.from_numpy(v) for k, v in dp.items()}, strict=False)
        engine.set_precision(model.netG, 'x3')
        dconv.set_precision('x3')
        pts = random_points(cfg)
        model._interp_points = lambda n: torch.from_numpy(next(pts)).to(dev).view(n, 1, 1, 1)
        flags = []
        first = {}  # the flat gradient each optimiser applies at its first step (before Adam has amplified anything)
        for o, tag in ((model.optimizer_G, 'G'), (model.optimizer_D, 'D')):
            def step(*a, _o=o, _step=o.step, _tag=tag, **kw):
                if _tag not in first:
                    _o._sync_views()
                    first[_tag] = _o.flat.grad.detach().double().cpu().numpy()
                return _step(*a, **kw)
            o.step = step
        if os.environ.get('DDP_PROBE_SYNC_STEP') == '1':  # diagnostic (tools/ddp_probe.py): drain before each step
            for o in (model.optimizer_G, model.optimizer_D):
                def synced(*a, _step=o.step, **kw):
                    torch.cuda.synchronize()
                    return _step(*a, **kw)
                o.step = synced
        for k in range(6):
            lr, hr, z = step_data(cfg, k if same_data else 1000 * rank + k)
            t = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
            model.feed_data({'LR': t(lr), 'HR': t(hr), 'Z': t(z)})
            model.optimize_parameters()
            flags.append(bool(model.generator_step))
        h = hashlib.sha256()
        per = {}
        for tag, net in (('G', model.netG), ('D', model.netD)):
            for k, v in net.state_dict().items():
                b = v.detach().cpu().contiguous().numpy().tobytes()
                h.update(b)
                per[tag + ':' + k] = (hashlib.sha256(b).hexdigest()[:16], float(v.double().norm()),
                                      v.detach().double().cpu().numpy())
        comm = [b.comm_stats() for b in (model._g_buckets, model._d_buckets) if b is not None]
        logs = {k: [x[1] for x in v] for k, v in model.log_dict.items() if v}
        logs['_reruns'] = (engine.OVERFLOW_RERUNS, engine.ACT_SCALE_REDUCTIONS)
        logs['_first_grads'] = first
        logs['_nonfinite'] = [tag + ':' + k for tag, net in (('G', model.netG), ('D', model.netD))
                              for k, v in net.state_dict().items() if v.is_floating_point() and
                              not bool(torch.isfinite(v).all())]
        q.put((rank, h.hexdigest(), flags, comm, None, per, logs))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, None, None, repr(e), None, None))
    finally:
        if world > 1 and dist.is_initialized():
            dist.destroy_process_group()


def _run(world, cfg_name, same_data, procs_n=None):
    """world ranks (procs_n > world: that many independent single-process runs at once, world must be 1)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    n = procs_n or world
    procs = [ctx.Process(target=_worker, args=(r if world > 1 else 0, world, port, cfg_name, same_data, q))
             for r in range(n)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(n)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    for r in res:
        assert r[4] is None, r[4]
    return res


def _zero_grad_bias(key, keys):
    """A discriminator conv bias followed by BatchNorm ('D:features.2.bias' -> 'D:features.3.running_mean')."""
    if not key.startswith('D:') or not key.endswith('.bias'):
        return False
    parts = key[:-len('.bias')].split('.')
    if not parts[-1].isdigit():
        return False
    return '.'.join(parts[:-1] + [str(int(parts[-1]) + 1), 'running_mean']) in keys


@pytest.mark.parametrize('cfg_name', ['past_ratio2_acc2', 'adaptive_rel'])
def test_ddp_two_ranks_on_the_gpu(cfg_name):
    """past_ratio2_acc2: gradient accumulation 2 and the 'past' D verification (all-reduced D statistics gate
    generator_step); adaptive_rel: the relativistic D and the adaptive update ratio."""
    from train_recipe import TRAIN_CFGS
    lr, n_steps = TRAIN_CFGS[cfg_name]['lr'], 6
    single = _run(1, cfg_name, True)[0]
    same = _run(2, cfg_name, True)
    assert same[0][1] == same[1][1], 'ranks fed the same batches diverged'
    assert same[0][2] == same[1][2] == single[2], 'generator_step decisions'
    # the averaged gradient of each network's first optimiser step: the all-reduce path itself (a lost, stale or
    # double-counted bucket shows at O(1)), before Adam amplifies anything
    assert set(single[6]['_first_grads']) == set(same[0][6]['_first_grads']) and 'D' in single[6]['_first_grads']
    for tag in sorted(single[6]['_first_grads']):  # (no G step in past_ratio2_acc2's six micro-steps)
        g1, g2 = single[6]['_first_grads'][tag], same[0][6]['_first_grads'][tag]
        rel = float(np.linalg.norm(g1 - g2) / np.linalg.norm(g1))
        print('%s: first %s step, averaged two-rank gradient vs one process: %.1e relative L2' % (cfg_name, tag, rel))
        assert rel <= 1e-5, (tag, rel)
    # the parameters after the loop: Adam (m / sqrt(v)) turns rounding-level gradient differences into
    # learning-rate-sized steps for elements whose gradient is ~0, most of all the biases that feed a BatchNorm
    keys = set(single[5])
    worst = (-1.0, '')
    for k in sorted(keys):
        a, b = single[5][k][2], same[0][5][k][2]
        if _zero_grad_bias(k, keys):
            assert np.abs(a - b).max() <= 2 * lr * n_steps, (k, np.abs(a - b).max())
            continue
        rel = float(np.linalg.norm(a - b) / max(np.linalg.norm(a), 1e-30))
        if k.endswith('running_mean'):
            # a running mean averages (momentum-weighted) batch means that carry those biases' Adam noise: the same
            # absolute bound, or 1e-3 relative
            assert rel <= 1e-3 or np.abs(a - b).max() <= 2 * lr * n_steps, (k, rel, np.abs(a - b).max())
            continue
        assert rel <= 1e-3, (k, rel)
        if not k.endswith('running_mean'):
            worst = max(worst, (rel, k))
    print('%s: parameters after %d micro-steps, two ranks vs one process, worst relative L2 (all but the pre-BN conv '
          'biases and running means): %.1e %s' % (cfg_name, n_steps, worst[0], worst[1]))
    assert sum(c['allreduces'] for c in same[0][3]) > 0 and sum(c['allreduce_bytes'] for c in same[0][3]) > 0
    diff = _run(2, cfg_name, False)
    assert diff[0][1] == diff[1][1], 'ranks fed different batches must still hold the same parameters'
    assert diff[0][2] == diff[1][2], 'and take the same generator_step decisions'
    assert diff[0][1] != single[1]
