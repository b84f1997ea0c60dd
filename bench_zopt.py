#!/usr/bin/env python3
"""Z-optimisation benchmark (BASELINE.json config 5): CEM-wrapped latent RRDB-23 with a learned (non-bicubic) blur
kernel — by default the ×4 kernel of the reference's KernelGAN post-processing, --kernel learned13 the 13×13
one of the CEM fixtures — batch 8 of 128×128 LR, eval mode (CEM pre-pad), Z_optimizer('max_STD') iterations — each one a
generator forward with retained activations + the HIP input-gradient sweep to Z + Adam on Z.

    python bench_zopt.py [--gpus N --steps K --warmup W]      (N>1 via torch.distributed.run: images sharded)

value = HR Mpixels/s of delivered (cropped) images per Z iteration summed over ranks; step = one Z iteration.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def kernelgan_kernel():
    """SURVEY §8's config-5 kernel: the ×4 kernel of the reference's KernelGAN post-processing (KernelGAN/util.py:
    123-182, post_process_k + analytic_kernel of a 13×13 ×2 estimate; tests/golden/kernelgan_x4.npz, made by
    tests/golden/make_golden.py with the reference's own functions).  33×33: CEM's margins are 22 LR / 88 HR pixels, so
    the generator runs at 172² per image."""
    with np.load(os.path.join(REPO, 'tests', 'golden', 'kernelgan_x4.npz')) as f:
        return np.asarray(f['kernel_x4'], dtype=np.float64)


KERNELS = {'kgan': 'kernelgan_kernel', 'learned13': 'learned_kernel'}


def learned_kernel():
    """The learned (non-bicubic) 13×13 kernel of the reference-made CEM fixture (tests/golden/cem_learned13.npz,
    `input_kernel`: the kernel tests/golden/make_golden.py fed the reference's CEM filter design; no KernelGAN run
    or dataset here).  With it CEM's margins are 13 LR / 52 HR pixels, so the generator runs at 154² per image."""
    with np.load(os.path.join(REPO, 'tests', 'golden', 'cem_learned13.npz')) as f:
        return np.asarray(f['input_kernel'], dtype=np.float64)


def leg_args(**kw):
    """Default arguments of this benchmark (BASELINE config 5 per GPU), for callers such as bench.py."""
    # warmup 6: the graph captures (2nd call per shape) and the caching allocator's release and regrowth (calls 3-6)
    # stay out of the timed region, as in bench_train.leg_args
    d = dict(gpus=1, steps=10, warmup=6, batch=8, lr_size=128, nb=23, objective='max_STD', kernel='kgan')
    d.update(kw)
    return argparse.Namespace(**d)


def run(args, dev, world, rank):
    """Build the latent CEM model with the learned kernel, run args.warmup then args.steps Z iterations (timed,
    barrier + synchronize bracketed, max over ranks), return the JSON record."""
    from esr_amd import engine
    from esr_amd.SRRaGAN_model import SRRaGANModel
    from esr_amd.Z_optimization import Z_optimizer
    from esr_amd import networks
    opt = {'is_train': False, 'scale': 4, 'gpu_ids': [0], 'range': [0, 1],
           'network_G': {'which_model_G': 'RRDB_net', 'CEM_arch': 1, 'latent_input': 'all_layers',
                         'latent_input_domain': 'HR_downscaled', 'latent_channels': 'SVDinNormedOut_structure_tensor',
                         'norm_type': None, 'mode': 'CNA', 'nf': 64, 'nb': args.nb, 'in_nc': 3, 'out_nc': 3,
                         'gc': 32}}
    torch.manual_seed(1234)  # same generator weights on every rank
    model = SRRaGANModel(opt, kernel=globals()[KERNELS[args.kernel]](), device=dev)
    networks.init_weights(model.netG.module, scale=0.1)
    g = torch.Generator().manual_seed(99 + rank)
    B, h = args.batch, args.lr_size
    data = {'LR': torch.rand(B, 3, h, h, generator=g).to(dev),
            'Z': (torch.rand(B, 3, 4 * h, 4 * h, generator=g) * 2 - 1).to(dev)}
    model.feed_data(data, need_HR=False)
    model.test()
    model.netG.eval()
    cem = model.netG.module
    zo = Z_optimizer(args.objective, [4 * h, 4 * h], model, 1.0, args.warmup, data=data, initial_LR=0.01,
                     batch_size=B)
    rrdb = cem.generated_image_model
    reruns0 = engine.OVERFLOW_RERUNS
    a0 = engine.act_scale(rrdb)
    zo.optimize()  # warmup iterations (workspace allocation, weight packing, graph captures)
    reruns1 = engine.OVERFLOW_RERUNS
    a1 = engine.act_scale(rrdb)
    zo.max_iters = args.steps
    from bench_train import GC_POLICY, observe, observed, settle, unsettle
    settle()
    obs0 = observe()
    stamps = []
    # host stamps after each iteration is enqueued (the overflow flags are read one iteration later, so the host runs
    # about one iteration ahead of the GPU; the timed region ends with a synchronize)
    zo.on_iteration = lambda _: stamps.append(time.perf_counter())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    zo.optimize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    zo.on_iteration = None
    iter_ms = [round((b - a) * 1e3, 2) for a, b in zip([t0] + stamps[:-1], stamps)]
    obs = observed(obs0, observe())
    unsettle()
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    m = int(cem.margins_LR)
    flop_iter = 2 * 2 * 18316944 * (h + 2 * m) ** 2 * B  # fwd + input dgrad, SURVEY.md §8(d) latent MAC/LR-px
    fwd = getattr(cem.generated_image_model, 'esr_precision', engine.DEFAULT_PRECISION)
    from esr_amd import train_engine
    bwd = 'x3' if fwd == 'x3' and train_engine.DGRAD_X3 else 'f32'
    return {'metric': 'Z-optimisation HR Mpixels/s per iteration (latent RRDB-23 + learned-kernel CEM, fwd + dZ + '
                      'Adam)',
            'value': round(world * B * (4 * h) ** 2 * args.steps / dt / 1e6, 4), 'unit': 'HR Mpixels/s',
            'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(dt / args.steps * 1e3, 2), 'higher_is_better': True, 'scaling': 'weak',
            'dtype': 'f32', 'fwd_dtype': fwd, 'bwd_dtype': bwd, 'data': 'synthetic',
            'achieved_TFLOPs': round(flop_iter * args.steps / dt / 1e12, 2),
            'config': {'workload': 'BASELINE config 5: batch %d/GPU of %dx%d LR, %s kernel (CEM margins %d/%d, G at '
                                   '%dx%d), objective %s, nb=%d' % (
                                       B, h, h, {'kgan': 'KernelGAN-recipe x4 33x33',
                                                 'learned13': 'learned 13x13'}[args.kernel], m, 4 * m, h + 2 * m,
                                       h + 2 * m, args.objective, args.nb),
                       'global_batch': world * B, 'parallelism': 'images sharded, no collective'},
            'final_loss': zo.loss_values[-1],
            'iter_ms': iter_ms,
            'overflow_reruns': {'warmup': reruns1 - reruns0, 'timed': engine.OVERFLOW_RERUNS - reruns1},
            'act_scale': {'before_warmup': a0, 'before_timed': a1, 'after_timed': engine.act_scale(rrdb)},
            'timed_region': dict(obs, gc_policy=GC_POLICY)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None, help='ranks (one per GPU); default: WORLD_SIZE, else 1')
    ap.add_argument('--launcher-check', action='store_true', help='bring the ranks up on the CPU (gloo) and stop')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=6)
    ap.add_argument('--batch', type=int, default=8)
    ap.add_argument('--lr-size', type=int, default=128)
    ap.add_argument('--nb', type=int, default=23)
    ap.add_argument('--objective', default='max_STD')
    ap.add_argument('--kernel', choices=sorted(KERNELS), default='kgan')
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
