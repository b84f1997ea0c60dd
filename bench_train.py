#!/usr/bin/env python3
"""Training-step benchmark (BASELINE.json configs 3 and 4): one SRRaGANModel.optimize_parameters() with a D step and
a G step, RRDB-23 (latent all_layers/HR_downscaled) + CEM generator on the HIP path (forward + hand-written fp32
backward), Discriminator_VGG_128_(nb=6) + WGAN-GP (gp 10) + range loss (5000), Adam on both.

    python bench_train.py [--gpus N --steps K --warmup W]     (N>1 via torch.distributed.run: DP over RCCL, B per rank)

One JSON line on rank 0: value = HR Mpixels/s of training images (all ranks), step time = max over ranks.  The VGG
feature loss of the config-3 wording is off in the shipped config (feature_weight 0) and broken in the reference.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def make_opt(args):
    patch = 4 * args.lr_size
    return {
        'is_train': True, 'scale': 4, 'gpu_ids': [0], 'range': [0, 1],
        'datasets': {'train': {'patch_size': patch, 'batch_size': args.batch}},
        'network_G': {'which_model_G': 'RRDB_net', 'CEM_arch': 1, 'latent_input': 'all_layers' if args.latent else None,
                      'latent_input_domain': 'HR_downscaled', 'latent_channels': 'SVDinNormedOut_structure_tensor',
                      'norm_type': None, 'mode': 'CNA', 'nf': 64, 'nb': args.nb, 'in_nc': 3, 'out_nc': 3, 'gc': 32},
        'network_D': {'which_model_D': 'discriminator_vgg_128', 'relativistic': 0, 'decomposed_input': 0,
                      'norm_type': 'batch', 'act_type': 'leakyrelu', 'mode': 'CNA', 'n_layers': 6, 'nf': 64,
                      'in_nc': 3},
        'train': {'lr_G': 1e-5, 'weight_decay_G': 0, 'beta1_G': 0.9, 'lr_D': 1e-5, 'weight_decay_D': 0,
                  'beta1_D': 0.9, 'lr_steps': [50000], 'lr_gamma': 0.5, 'gan_type': 'wgan-gp', 'gan_weight': 1,
                  'gp_weigth': 10, 'range_weight': 5000, 'D_update_ratio': 1, 'D_verification': None,
                  'D_init_iters': 0, 'pixel_weight': 0, 'feature_weight': 0, 'latent_weight': 0,
                  'optimalZ_loss_weight': 0},
    }


GC_POLICY = ('Python GC: gc.collect() + gc.freeze() after the warm-up (settle(): the models, op lists and packed '
             'weights leave the collector, as in a serving process after model load), collector otherwise on; gc_gen2 / '
             'gc_ms count the collections and time inside the timed steps')
_GC_PAUSE = [0.0, None]  # total seconds Python's cyclic GC has run, start of the current collection


def _gc_timer(phase, info):
    if phase == 'start':
        _GC_PAUSE[1] = time.perf_counter()
    elif _GC_PAUSE[1] is not None:
        _GC_PAUSE[0] += time.perf_counter() - _GC_PAUSE[1]
        _GC_PAUSE[1] = None


def settle():
    """End of a leg's warm-up: one full collection, then the surviving objects (models, op lists, packed weights) are
    frozen out of the collector's generations, as a serving process does after loading its model — a generation-2
    collection inside the timed region then scans only the objects created since (without it one such collection cost
    a C5 iteration ≈150 ms: BENCH r4 records, `timed_region.gc_ms`)."""
    import gc
    gc.collect()
    gc.freeze()


def unsettle():
    """After the timed region: the frozen objects rejoin the collector (so that this leg's models, once dropped, are
    collected even if they sit in reference cycles)."""
    import gc
    gc.unfreeze()


def observe():
    """Counters that explain a timed region (record the delta of two calls): x3 overflow reruns, how the training
    passes ran (eager / graph capture / replay), the caching allocator's device allocations and retries, and Python's
    generation-2 garbage collections and the time the collector ran."""
    import gc
    from esr_amd import engine, train_engine
    if _gc_timer not in gc.callbacks:
        gc.callbacks.append(_gc_timer)
    ms = torch.cuda.memory_stats()
    return {'overflow_reruns': engine.OVERFLOW_RERUNS, 'act_scale_reductions': engine.ACT_SCALE_REDUCTIONS,
            **{'graph_' + k: v for k, v in train_engine.GRAPH_COUNTS.items()},
            'device_allocs': ms.get('num_device_alloc', 0), 'device_frees': ms.get('num_device_free', 0),
            'alloc_retries': ms.get('num_alloc_retries', 0), 'gc_gen2': gc.get_stats()[2]['collections'],
            'gc_ms': round(_GC_PAUSE[0] * 1e3, 2)}


def observed(a, b):
    return {k: round(b[k] - a[k], 2) for k in a}


def leg_args(**kw):
    """Default arguments of this benchmark (BASELINE config 3 per GPU), for callers such as bench.py."""
    # warmup 6: the caching allocator grows over the first calls (HIP graph captures in calls 2-3), returns memory to
    # the device in call 4 and makes its last device allocations (9, in the discriminator's double backward) in calls
    # 5-6; from call 7 on a step allocates nothing (tools/alloc_probe.py, profiles/r5_c3_alloc_steps.txt)
    d = dict(gpus=1, steps=10, warmup=6, batch=16, lr_size=96, nb=23, latent=True)
    d.update(kw)
    return argparse.Namespace(**d)


def run(args, dev, world, rank):
    """Build the model, run args.warmup + args.steps optimize_parameters() calls (timed: the steps, bracketed by
    barrier + synchronize, max over ranks), return the JSON record."""
    from esr_amd import engine
    from esr_amd.SRRaGAN_model import SRRaGANModel, collective
    torch.manual_seed(1000 + rank)
    model = SRRaGANModel(make_opt(args), device=dev)
    if world > 1:  # identical initial weights on every rank (DataParallel replicates rank 0's)
        for p in list(model.netG.parameters()) + list(model.netD.parameters()):
            collective(dist.broadcast, p.data, 0)
    g = torch.Generator(device='cpu').manual_seed(7 + rank)
    hr = 4 * args.lr_size
    data = {'LR': torch.rand(args.batch, 3, args.lr_size, args.lr_size, generator=g).to(dev),
            'HR': torch.rand(args.batch, 3, hr, hr, generator=g).to(dev)}
    gsteps = 0
    rrdb = model._rrdb
    reruns0, a0 = engine.OVERFLOW_RERUNS, engine.act_scale(rrdb)
    for _ in range(args.warmup):
        model.feed_data(data)
        model.optimize_parameters()
    reruns1, a1 = engine.OVERFLOW_RERUNS, engine.act_scale(rrdb)
    settle()
    obs0 = observe()
    comm0 = comm_stats(model)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stamps = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        model.feed_data(data)
        model.optimize_parameters()  # ends with its deferred overflow-flag read (a device sync)
        gsteps += int(model.generator_step)
        stamps.append(time.perf_counter())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    step_ms = [round((b - a) * 1e3, 2) for a, b in zip([t0] + stamps[:-1], stamps)]
    obs = observed(obs0, observe())
    comm = {k: round((v - comm0[k]) / args.steps, 3) for k, v in comm_stats(model).items()}
    unsettle()
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    value = world * args.batch * hr * hr * args.steps / dt / 1e6
    fwd = getattr(model.netG.module if hasattr(model.netG, 'module') else model.netG, 'generated_image_model',
                  None)
    fwd = getattr(fwd, 'esr_precision', engine.DEFAULT_PRECISION) if fwd is not None else engine.DEFAULT_PRECISION
    from esr_amd import dconv, train_engine
    bwd = 'x3' if fwd == 'x3' and train_engine.DGRAD_X3 and train_engine.WGRAD_X3 else 'f32'
    return {'metric': 'training HR Mpixels/s (RRDB-23 + CEM G fwd+bwd, VGG128_ D + WGAN-GP, Adam)',
            'value': round(value, 4), 'unit': 'HR Mpixels/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(dt / args.steps * 1e3, 2), 'higher_is_better': True,
            'scaling': 'weak', 'dtype': 'f32', 'fwd_dtype': fwd, 'bwd_dtype': bwd, 'd_dtype': dconv.PRECISION, 'data': 'synthetic',
            'generator_steps_in_timed_region': gsteps,
            'config': {'workload': 'BASELINE config %s: batch %d/GPU of %dx%d LR crops (%dx%d HR, D on %dx%d after '
                                   'CEM unpad), nb=%d, latent=%s' % ('4' if world > 1 else '3', args.batch,
                                                                      args.lr_size, args.lr_size, hr, hr, hr - 80,
                                                                      hr - 80, args.nb, args.latent),
                       'global_batch': world * args.batch,
                       'parallelism': 'dp%d (bucketed RCCL all-reduce of G/D grads)' % world},
            'last_losses': {k: v[-1][1] for k, v in model.log_dict.items() if v},
            'step_ms': step_ms,
            'overflow_reruns': {'warmup': reruns1 - reruns0, 'timed': engine.OVERFLOW_RERUNS - reruns1},
            'act_scale': {'before_warmup': a0, 'before_timed': a1, 'after_timed': engine.act_scale(rrdb)},
            'timed_region': dict(obs, gc_policy=GC_POLICY),
            'dist': {'world_size': dist.get_world_size() if world > 1 else 1,
                     'backend': dist.get_backend() if world > 1 else None,
                     'per_step': comm,
                     'note': 'G + D gradient buckets: RCCL all-reduces, bytes and the compute-stream time left waiting '
                             'for them (exposed_ms), averaged over the timed steps'}}


def comm_stats(model):
    """Summed GradBuckets counters of G and D (SRRaGAN_model.GradBuckets.comm_stats)."""
    tot = {'allreduces': 0, 'allreduce_bytes': 0, 'exposed_ms': 0.0}
    for b in (model._g_buckets, model._d_buckets):
        if b is not None:
            for k, v in b.comm_stats().items():
                tot[k] += v
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None, help='ranks (one per GPU); default: WORLD_SIZE, else 1')
    ap.add_argument('--launcher-check', action='store_true', help='bring the ranks up on the CPU (gloo) and stop')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=6)
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--lr-size', type=int, default=96)
    ap.add_argument('--nb', type=int, default=23)
    ap.add_argument('--no-latent', dest='latent', action='store_false')
    args = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import bench_launch
    world = bench_launch.ranks(args.gpus, os.path.abspath(__file__), sys.argv[1:],
                               check_devices=not args.launcher_check)
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.launcher_check:
        bench_launch.launcher_check(world, rank)
        return
    local = bench_launch.local_device_index()
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    world = bench_launch.init(dev, world)
    rec = run(args, dev, world, rank)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
