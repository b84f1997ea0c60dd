#!/usr/bin/env python3
"""Benchmark of the RRDB-23 + CEM ×4 super-resolution hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]        (N>1: N ranks, one per GPU — started by this script through
                                                           torch.distributed.run, or by an external one: bench_launch.py)

A step = one forward of CEM_PyTorch(RRDBNet-23) in eval mode (CEM pre-pad, the reference's test path
SRRaGANModel.test(), SRRaGAN_model.py:577-584) over one batch of B synthetic 128×128 LR images already resident in
HBM, producing B 512×512 HR images.  Multi-GPU: images are independent, so each rank runs its own batch (weak scaling,
no collective in the data path); timing is barrier + synchronize bracketed and the max over ranks is reported.

One JSON line on rank 0: value = HR Mpixels/s over all ranks; `roofline` = the dominant kernel (the 3×3 conv
instantiation that takes the most time) from HIP events around every launch in the timed region (recorded natively by
the op-list executor esr_run_ops, so the timing adds no host round trips); `cpu_baseline` =
the CPU oracle restatement (oracle/esr_oracle.py, PyTorch-CPU oneDNN convs) on a bounded sample, rank 0 only.
Extra keys, each timed separately after the headline (--no-legs skips them): `fp32_c2` (the same step in exact fp32),
`train_c3` / `train_c4` (one SRRaGANModel.optimize_parameters step, bench_train.py), `zopt_c5` (one Z-optimisation
iteration, bench_zopt.py, with SURVEY §8's KernelGAN-recipe kernel; `zopt_c5_learned13` with the 13×13 learned one).
"""
import argparse
import collections
import contextlib
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

METRIC = json.load(open(os.path.join(REPO, 'BASELINE.json')))['metric']
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 matrix = vector peak (f32-input MFMA)
F16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense (spec)
PEAKS = {  # fp32-equivalent peak of each precision mode, in reference (fp32) FLOPs
    'f32': (FP32_PEAK_TFLOPS, 'f32-input MFMA = f32 vector peak'),
    'x3': (F16_DENSE_PEAK_TFLOPS / 3, '2.5 PFLOP/s dense f16 MFMA / 3 f16 products per fp32 product'),
}
DTYPES = {'f32': 'f32', 'x3': 'f32 (x3: f16 hi/lo split operands, 3 f16 MFMA products, fp32 accumulate)'}
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=None, help='ranks (one per GPU); default: WORLD_SIZE, else 1')
    ap.add_argument('--launcher-check', action='store_true', help='bring the ranks up on the CPU (gloo), agree on the '
                    'world size, print it and stop (no GPU)')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=32, help='images per GPU (BASELINE config 2: 32)')
    ap.add_argument('--lr-size', type=int, default=128)
    ap.add_argument('--nb', type=int, default=23)
    ap.add_argument('--variant', choices=['plain', 'latent'], default='plain')
    ap.add_argument('--no-cem', action='store_true', help='bare RRDBNet (no CEM, no pre-pad)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--precision', choices=['x3', 'f32'], default='x3')
    ap.add_argument('--cpu-images', type=int, default=8, help='images in the bounded CPU-baseline sample')
    ap.add_argument('--no-cpu-variants', action='store_true', help='skip the latent Z=0 / Z~U[-1,1] CPU baselines')
    ap.add_argument('--no-legs', action='store_true', help='skip the extra legs (exact-fp32 C2, C3/C4 training step, '
                    'C5 Z-optimisation iteration)')
    ap.add_argument('--leg-steps', type=int, default=10)
    ap.add_argument('--host-io-steps', type=int, default=3, help='steps of the PCIe-inclusive variant (host_io; 0: skip)')
    ap.add_argument('--x3-kernel', type=int, default=None, help='esr_x3_set_kernel variant (A/B: needs the ablation '
                    'library, ESR_AMD_LIB=exp_lib/libesr_exp.so; default automatic)')
    ap.add_argument('--profile-steps', type=int, default=2, help='timed steps (the last ones) that carry per-launch HIP '
                    'events for the roofline')
    ap.add_argument('--eager-overflow-check', action='store_true',
                    help='every timed forward reads its own x3 overflow flag before returning (default: one forward '
                         'late, engine.lagged_overflow_checks, as a serving loop runs)')
    ap.add_argument('--no-op-timers', action='store_true', help='time the steps without the per-launch HIP events '
                    '(no roofline; measures what the events themselves cost)')
    return ap.parse_args()


def build_model(args, dev):
    import esr_amd
    from esr_amd import CEMnet as C
    latent = args.variant == 'latent'
    torch.manual_seed(1234)
    net = esr_amd.RRDBNet(3, 3, 64, args.nb, latent_input='all_layers_HR_downscaled' if latent else None,
                          num_latent_channels=3 if latent else 0)
    model = net if args.no_cem else C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net)
    esr_amd.init_weights(model, 'kaiming', scale=0.1)  # define_G's training-time init (networks.py:97-98)
    with torch.no_grad():  # nonzero biases so the epilogue is exercised
        for n, p in model.named_parameters():
            if n.endswith('bias'):
                p.uniform_(-0.01, 0.01)
    model.eval()
    from esr_amd import engine
    engine.set_precision(model, args.precision)
    return model.to(dev)


def make_gt(args, dev, rank):
    """Seeded synthetic ground-truth HR images (B, 3, 4h, 4w) in [0, 1]: smooth structure (bicubic 16x up of a 32² /
    8x up of a 64² noise field) plus fine detail, so that an SR result has a meaningful PSNR against them."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(100 + rank)
    B, h = args.batch, args.lr_size
    H = 4 * h
    coarse = torch.rand(B, 3, h // 4, h // 4, generator=g)
    mid = torch.rand(B, 3, h // 2, h // 2, generator=g)
    fine = torch.rand(B, 3, H, H, generator=g)
    gt = (0.6 * F.interpolate(coarse, size=(H, H), mode='bicubic', align_corners=False)
          + 0.3 * F.interpolate(mid, size=(H, H), mode='bicubic', align_corners=False) + 0.1 * fine)
    return gt.clamp_(0, 1).to(dev)


def make_input(args, dev, rank, model=None):
    """The LR batch: the CEM's own DownscaleOP (the reference's degradation, CEMnet.py:152,157-162; the build's device
    stencil) of the seeded ground truth make_gt(), so the SR outputs can be scored against it (PSNR-Δ);
    without a CEM (--no-cem) seeded U[0, 1) LR images.  Latent variant: per-image constant Z, raw HR view."""
    g = torch.Generator().manual_seed(200 + rank)
    B, h = args.batch, args.lr_size
    if model is not None and hasattr(model, 'DownscaleOP'):
        with torch.no_grad():
            x = model.DownscaleOP(make_gt(args, dev, rank)).contiguous()
    else:
        x = torch.rand(B, 3, h, h, generator=g).to(dev)
    if args.variant == 'latent':  # per-image constant Z (training-time feed_data), raw HR view (ConcatLatent)
        z = (2 * torch.rand(B, 3, 1, 1, generator=g) - 1).expand(B, 3, 4 * h, 4 * h).contiguous().to(dev)
        x = torch.cat([z.view(B, 48, h, h), x], 1)
    return x


def cpu_baseline(args, model, x_gpu, out_gpu, gt=None):
    """The CPU oracle on a bounded sample of the same workload (same weights, same images), rank 0 only.  With the
    ground truth the LR batch was made from (make_gt), also the PSNR-Δ of SURVEY §8(d): |PSNR(build, GT) −
    PSNR(ref, GT)| with the reference's validation PSNR (0-255 images clamped as tensor2img does, utils/util.py:80-104,
    168-175; SRRaGAN_model.py:627-634)."""
    from oracle import esr_oracle as O
    threads = min(os.cpu_count() or 1, 16)  # the GPU box gives one GPU a 16-CPU share
    torch.set_num_threads(threads)
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    P = O.strip_prefix({k: v for k, v in sd.items() if 'Filter' not in k})
    design = None if args.no_cem else O.cem_design(4)
    n = max(1, min(args.cpu_images, x_gpu.shape[0]))
    xs = x_gpu[:n].cpu()
    latent = args.variant == 'latent'
    with torch.no_grad():
        O.sr_forward(xs[:1], P, args.nb, latent, design, pre_pad=design is not None)  # warm-up
        t0 = time.perf_counter()
        outs = [O.sr_forward(xs[i:i + 1], P, args.nb, latent, design, pre_pad=design is not None) for i in range(n)]
        dt = time.perf_counter() - t0
    ref = torch.cat(outs)
    got = out_gpu[:n].cpu().double()
    err = float((got - ref.double()).abs().max() / ref.double().abs().max())
    mse = float(((got - ref.double()) ** 2).mean())
    hr = 4 * args.lr_size
    par = {'normwise_rel_err_vs_cpu_ref': err, 'psnr_vs_ref_db': (10 * np.log10(1.0 / mse)) if mse > 0 else None,
           'images_compared': n}
    if gt is not None:
        from esr_amd.SRRaGAN_model import _psnr

        def img(t):
            return 255 * t.double().clamp(0, 1).numpy()
        gts = gt[:n].cpu()
        pb = [_psnr(img(got[i].float()), img(gts[i])) for i in range(n)]
        pr = [_psnr(img(ref[i]), img(gts[i])) for i in range(n)]
        par.update({'psnr_build_vs_gt_db': float(np.mean(pb)), 'psnr_ref_vs_gt_db': float(np.mean(pr)),
                    'psnr_delta_db': abs(float(np.mean(pb)) - float(np.mean(pr))),
                    'psnr_delta_max_per_image_db': max(abs(a - b) for a, b in zip(pb, pr)),
                    'gt': 'seeded synthetic HR images (bench.make_gt), LR = the CEM DownscaleOP of them; '
                          'random-init weights, so the absolute PSNRs are low and only the delta is the metric'})
    return ({'value': round(n * hr * hr / dt / 1e6, 4), 'unit': 'HR Mpixels/s', 'cores': threads, 'kind': 'port',
             'sample': '%d image(s) of 128x128 LR -> 512x512, same weights/inputs as the GPU run, PyTorch-CPU '
                       '(oneDNN) restatement oracle/esr_oracle.py, %d threads' % (n, threads)}, par)


def cpu_baseline_variants(args):
    """BASELINE.md's CPU-baseline protocol for the other config-1 variants: latent RRDB-23 (all_layers,
    HR_downscaled, 3 channels) + CEM on one 128² LR image with Z = 0 and with Z ~ U[-1, 1] per HR pixel, 1 warm-up then
    the median of 3 runs, same threads as cpu_baseline.  The oracle with freshly initialised latent weights (the
    plain variant is cpu_baseline itself)."""
    import copy
    from oracle import esr_oracle as O
    a = copy.copy(args)
    a.variant = 'latent'
    model = build_model(a, torch.device('cpu'))
    sd = {k: v.detach().float() for k, v in model.state_dict().items()}
    P = O.strip_prefix({k: v for k, v in sd.items() if 'Filter' not in k})
    design = None if args.no_cem else O.cem_design(4)
    h = args.lr_size
    g = torch.Generator().manual_seed(7)
    lr = torch.rand(1, 3, h, h, generator=g)
    out = {}
    for tag, z in (('latent_z0', torch.zeros(1, 3, 4 * h, 4 * h)),
                   ('latent_zuniform', 2 * torch.rand(1, 3, 4 * h, 4 * h, generator=g) - 1)):
        x = torch.cat([z.reshape(1, 48, h, h), lr], 1)  # raw HR view, SRRaGAN_model.py:252
        ts = []
        with torch.no_grad():
            for r in range(4):
                t0 = time.perf_counter()
                O.sr_forward(x, P, args.nb, True, design, pre_pad=design is not None)
                if r:
                    ts.append(time.perf_counter() - t0)
        t = sorted(ts)[1]
        out[tag] = {'value': round((4 * h) ** 2 / t / 1e6, 4), 'unit': 'HR Mpixels/s', 's_per_image': round(t, 3)}
    out['protocol'] = ('config 1: 1 image %dx%d LR -> %dx%d, RRDB-%d latent%s (eval), 1 warm-up + median of 3, '
                       '%d threads, oracle/esr_oracle.py' % (h, h, 4 * h, 4 * h, args.nb, '' if args.no_cem else ' + CEM',
                                                             torch.get_num_threads()))
    return out


def reference_parity(dev):
    """Production-grid parity of the C3 training step and the C5 Z-gradients against the reference-made fixtures
    (tests/grid_parity.py: the reference's own optimize_parameters at B=16 × 96², its autograd dZ at B=8 × 128² with
    the learned kernel) — a checker like cpu_baseline, run on rank 0 at N=1 after every timed region."""
    tests = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'tests')
    if tests not in sys.path:
        sys.path.insert(0, tests)
    import grid_parity as GP
    out = {}
    for key, fn in (('train_c3', GP.c3_training_step), ('zopt_c5', lambda d: GP.c5_z_gradients(d, kernel='kgan')),
                    ('zopt_c5_learned13', lambda d: GP.c5_z_gradients(d, kernel='learned13'))):
        try:
            r = fn(dev)
            out[key] = {'vs': 'reference float64 run (5x its float32 error + 1e-4 floor; config 3: the largest float32 '
                              'error over the plain and the rounding-perturbed reference runs)', 'ok': r['ok'],
                        'worst_frac_of_bound': r['worst_frac_of_bound'], 'n_fails': len(r['fails'])}
            if 'worst_frac_of_single_run_bound' in r:
                out[key]['worst_frac_of_single_run_bound'] = r['worst_frac_of_single_run_bound']
        except Exception as e:  # noqa: BLE001
            out[key] = {'error': repr(e)}
        torch.cuda.empty_cache()
    return out


HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8 TB/s; 6.3 TB/s measured by a float4 copy)


def pmc_traffic(tags):
    """HBM bytes per launch, launch-weighted over the kernel tags `tags`, from the committed rocprofv3 PMC passes
    (profiles/pmc_latest.json, made by tools/prof_summary.py from separate --pmc FETCH_SIZE / WRITE_SIZE runs of this
    same default bench command, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM), and the per-launch union time of
    the x3 family in that run's kernel trace.  PMC counters cannot be read live from inside the process."""
    path = os.path.join(REPO, 'profiles', 'pmc_latest.json')
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    n = byt = 0.0
    for r in d['kernels']:
        if r['kernel'] in tags and r['hbm_read_bytes_per_launch'] is not None:
            n += r['calls']
            byt += r['calls'] * (r['hbm_read_bytes_per_launch'] + (r['hbm_write_bytes_per_launch'] or 0.0))
    if not n:
        return None
    return byt / n, '%s (%s)' % (os.path.relpath(path, REPO), d['source']), d.get('x3_family_union_us_per_launch')


def _timed(fn, steps, dev, world):
    """Seconds for `steps` calls of fn(), barrier + synchronize bracketed, max over ranks."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt


def host_io(model, x, out, args, dev, world):
    """The headline step with its batch handed over in host memory, as the reference's feed_data / get_current_visuals
    do (SRRaGAN_model.py feed_data .to(device), util.tensor2img .cpu()): pinned LR batch -> device, forward, HR output ->
    pinned host, all on the step's stream, timed like the headline (barrier + synchronize, max over ranks).  The C-ABI
    boundary itself takes device buffers, so this is never `value`."""
    xh = torch.empty(x.shape, dtype=x.dtype, pin_memory=True).copy_(x.cpu())
    oh = torch.empty(out.shape, dtype=out.dtype, pin_memory=True)

    def step():
        xd = xh.to(dev, non_blocking=True)
        oh.copy_(model(xd), non_blocking=True)
    with torch.no_grad():
        step()
        dt = _timed(step, args.host_io_steps, dev, world)
    hr = 4 * args.lr_size
    return {'value': round(world * args.batch * hr * hr * args.host_io_steps / dt / 1e6, 3), 'unit': 'HR Mpixels/s',
            'ms_per_step': round(dt / args.host_io_steps * 1e3, 2), 'steps': args.host_io_steps,
            'h2d_MB_per_step': round(xh.numel() * 4 / 1e6, 2), 'd2h_MB_per_step': round(oh.numel() * 4 / 1e6, 2),
            'note': 'PCIe-inclusive: pinned host LR batch in, HR output back to pinned host memory, per step'}


def per_forward_check(model, x, args, dev, world, dt_headline):
    """The headline step with each forward reading its own x3 overflow flag before it returns (the default outside
    engine.lagged_overflow_checks: one 4-byte device-to-host read per forward, the host waits for the GPU to drain
    between forwards).  Timed like the headline, without per-launch events."""
    with torch.no_grad():
        dt = _timed(lambda: model(x), args.steps, dev, world)
    hr = 4 * args.lr_size
    return {'value': round(world * args.batch * hr * hr * args.steps / dt / 1e6, 3), 'unit': 'HR Mpixels/s',
            'ms_per_step': round(dt / args.steps * 1e3, 3), 'steps': args.steps,
            'headline_ms_per_step': round(dt_headline / args.steps * 1e3, 3),
            'note': 'each forward reads its own overflow flag before returning (no per-launch events); the headline '
                    'reads forward N\'s flag after forward N + 1 is enqueued (engine.lagged_overflow_checks) and '
                    'carries events on its last steps'}


def run_legs(args, dev, world, rank):
    """Extra legs in the same run, each timed on its own after the headline's timed region (HIP work synchronised,
    barrier, max over ranks): the C2 step in exact fp32, one C3 training step (C4 when N>1: DP over RCCL) and one C5
    Z-optimisation iteration.  A failing leg records its error instead of a number."""
    import argparse as ap_
    import bench_train
    import bench_zopt
    legs = {}
    try:
        a = ap_.Namespace(**vars(args))
        a.precision = 'f32'
        model = build_model(a, dev)
        x = make_input(a, dev, rank, model)
        with torch.no_grad():
            model(x)
            dt = _timed(lambda: model(x), args.leg_steps, dev, world)
        hr = 4 * args.lr_size
        legs['fp32_c2'] = {'value': round(world * args.batch * hr * hr * args.leg_steps / dt / 1e6, 3),
                           'unit': 'HR Mpixels/s', 'ms_per_step': round(dt / args.leg_steps * 1e3, 2),
                           'steps': args.leg_steps, 'dtype': 'f32',
                           'note': 'the headline workload with every conv in exact fp32 (f32-input MFMA)'}
        del model, x
    except Exception as e:  # noqa: BLE001
        legs['fp32_c2'] = {'error': repr(e)}
    torch.cuda.empty_cache()
    import gc
    for key, mod, kw in (('train_c4' if world > 1 else 'train_c3', bench_train, {}),
                         ('zopt_c5', bench_zopt, {'kernel': 'kgan'}),
                         ('zopt_c5_learned13', bench_zopt, {'kernel': 'learned13'})):
        try:
            legs[key] = mod.run(mod.leg_args(steps=args.leg_steps, **kw), dev, world, rank)
        except Exception as e:  # noqa: BLE001
            legs[key] = {'error': repr(e)}
        gc.collect()  # the leg's model, even inside reference cycles, before the cache is released
        torch.cuda.empty_cache()
    return legs


def main():
    args = parse()
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
    from esr_amd import engine
    if args.x3_kernel is not None:
        from esr_amd import _lib
        lib = _lib.load()
        if not hasattr(lib, 'esr_x3_set_kernel'):
            raise SystemExit('--x3-kernel needs the ablation library (ESR_AMD_LIB=exp_lib/libesr_exp.so); the product '
                             'library has no kernel-selection state')
        if lib.esr_x3_set_kernel(args.x3_kernel) < 0:
            raise SystemExit('esr_x3_set_kernel(%d) rejected' % args.x3_kernel)
    model = build_model(args, dev)
    x = make_input(args, dev, rank, model)
    with torch.no_grad():
        # the last warmup forward runs profiled to learn the op-list length(s); their timers are then created up front,
        # outside the timed region
        probe = []
        n_prof = min(args.steps, max(1, args.profile_steps))
        for i in range(max(args.warmup, 1)):
            engine._PROFILE = probe if i == max(args.warmup, 1) - 1 else None
            out = model(x)
        torch.cuda.synchronize()
        engine._PROFILE = None
        # one timer set per op list a profiled step runs: the two stream parts record op lists of the same length,
        # so reserve per occurrence (a set of lengths reserved half of them and the rest were created in the timed
        # region)
        for n_ops, c in collections.Counter(e[3] for e in probe if e[0] == 'ops').items():
            engine.reserve_timers(n_ops, c * n_prof)
        list(engine.profile_records(probe))
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        prof = []
        origin = engine.ProfileOrigin(dev)
        origin.record()
        # A serving loop: each forward's x3 overflow flag is read one forward late (engine.lagged_overflow_checks),
        # so forward N + 1 is enqueued before the host waits on N; the block's exit settles the last flag (an
        # overflowed forward is recomputed in exact fp32 into its own output) inside the timed region.
        lag = contextlib.nullcontext() if args.eager_overflow_check or args.precision != 'x3' \
            else engine.lagged_overflow_checks()
        t0 = time.perf_counter()
        ev_prof = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        with lag:
            for i in range(args.steps):  # per-launch events on the last n_prof steps only (~1.5 % of a step)
                engine._PROFILE = prof if (not args.no_op_timers and i >= args.steps - n_prof) else None
                if i == args.steps - n_prof:
                    ev_prof[0].record()  # the profiled steps' own wall time on the device (the busy fraction's base)
                out = model(x)
            ev_prof[1].record()
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        engine._PROFILE = None
        engine.release_timers()
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.barrier()
        dt = float(t.item())
    hr = 4 * args.lr_size
    total_px = world * args.batch * hr * hr * args.steps
    value = total_px / dt / 1e6
    if args.no_op_timers:
        origin.close()
        if rank == 0:
            print(json.dumps({'metric': METRIC, 'value': round(value, 3), 'unit': 'HR Mpixels/s', 'n_gpus': world,
                              'steps': args.steps, 'ms_per_step': round(dt / args.steps * 1e3, 3),
                              'note': 'no per-launch events (timer-overhead check; not the bench line)'}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    # roofline from the per-launch events.  With the batch split over engine.STREAMS HIP streams, launches run
    # concurrently and no single launch's duration is its own: the roofline is that of the x3 MFMA conv family (every
    # profiled launch of the step: the conv_x3c 3x3 convs, the sub-pixel upconvs, the fused HR convs) — their FLOPs
    # over the UNION of their HIP-event intervals, i.e. the MFMA rate the GPU sustained while any of them ran; the
    # per-tag lines beside it give each tag's FLOPs over the union of its own intervals and its mean event duration.
    per = {}
    for tag, flops, t_a, t_b, nbytes in engine.profile_intervals(prof, origin):
        a = per.setdefault(tag, [0, 0.0, 0.0, [], 0.0])
        a[0] += 1
        a[1] += flops
        a[2] += t_b - t_a
        a[3].append((t_a, t_b))
        a[4] += nbytes
    origin.close()
    union = {k: engine.union_ms(v[3]) for k, v in per.items()}
    busy = engine.union_ms([iv for v in per.values() for iv in v[3]])
    n_all, fl_all = sum(v[0] for v in per.values()), sum(v[1] for v in per.values())
    achieved = fl_all / (busy / 1e3) / 1e12
    dom = max(per, key=lambda k: per[k][2])
    peak, peak_note = PEAKS[args.precision]
    # wall time of the profiled steps themselves (device events around them: the event-carrying steps run slower than
    # the average step, so dt * n_prof / steps understated it and the busy fraction could exceed 1)
    prof_ms = ev_prof[0].elapsed_time(ev_prof[1])
    kernels = {k: {'launches_per_step': v[0] // n_prof, 'avg_us': round(v[2] / v[0] * 1e3, 2),
                   'tflops_over_own_union': round(v[1] / (union[k] / 1e3) / 1e12, 2),
                   'share_of_step': round(union[k] / prof_ms, 3)}
               for k, v in per.items()}
    streams = engine.STREAMS if (engine.USE_OP_LISTS and engine.use_streams(x.shape, None if args.no_cem else model)) else 1
    rec = {
        'metric': METRIC, 'value': round(value, 3), 'unit': 'HR Mpixels/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(dt / args.steps * 1e3, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': DTYPES[args.precision], 'data': 'synthetic',
        'config': {'workload': 'RRDB-23 x4 %s%s, batch %d x %dx%d LR -> %dx%d HR per GPU (BASELINE config 2 shape)'
                               % (args.variant, '' if args.no_cem else ' + CEM (eval, LR pre-pad 10)', args.batch,
                                  args.lr_size, args.lr_size, hr, hr),
                   'global_batch': world * args.batch, 'nb': args.nb, 'parallelism': 'dp%d (image sharding, no '
                   'data-path collective)' % world},
        'roofline': {'bound': 'mfma', 'kernel': 'x3 MFMA conv family (%s), all launches of the step' % ', '.join(sorted(per)),
                     'achieved': round(achieved, 2), 'peak': round(peak, 1), 'peak_basis': peak_note,
                     'unit': 'TFLOP/s', 'frac': round(achieved / peak, 4), 'traffic': None,
                     'flops_per_launch': fl_all / n_all, 'launches_per_step': n_all // n_prof,
                     'algorithmic_bytes_per_launch': sum(v[4] for v in per.values()) / n_all,
                     'profiled_steps': n_prof,
                     'union_us_per_launch': round(busy / n_all * 1e3, 2), 'streams': streams,
                     'timing': 'achieved = FLOPs of all launches / union of their HIP-event intervals, events on '
                               'every launch of the last %d of the %d timed steps (%d stream(s); union / launches is '
                               'the effective launch time the rocprof kernel-trace union is checked against)'
                               % (n_prof, args.steps, streams),
                     'dominant_tag': {'tag': dom, 'flops_per_launch': per[dom][1] / per[dom][0],
                                      'avg_launch_us': round(per[dom][2] / per[dom][0] * 1e3, 2)}},
        'kernels': kernels,
        'gpu_busy_frac': round(busy / prof_ms, 3),
        'dist': {'world_size': dist.get_world_size() if world > 1 else 1,
                 'backend': dist.get_backend() if world > 1 else None},
    }
    traffic = pmc_traffic(set(per))
    if traffic is not None:
        rec['roofline']['traffic'] = traffic[0]
        rec['roofline']['traffic_over_algorithmic'] = round(traffic[0] / rec['roofline']['algorithmic_bytes_per_launch'], 3)
    # the same launches against the HBM roofline (north_star's target is stated there): measured HBM bytes per launch
    # (PMC) and the algorithmic minimum, each over the effective launch time (union / launches), vs 8 TB/s
    t_launch = busy / n_all / 1e3  # s
    alg = rec['roofline']['algorithmic_bytes_per_launch']
    rec['roofline']['hbm'] = {
        'peak_GBps': HBM_PEAK_GBPS, 'flop_per_byte_algorithmic': round(fl_all / n_all / alg, 1),
        'ridge_flop_per_byte': round(peak * 1e12 / (HBM_PEAK_GBPS * 1e9), 1),
        'algorithmic_GBps': round(alg / t_launch / 1e9, 1), 'algorithmic_frac': round(alg / t_launch / 1e9 / HBM_PEAK_GBPS, 4)}
    if traffic is not None:
        rec['roofline']['hbm']['measured_GBps'] = round(traffic[0] / t_launch / 1e9, 1)
        rec['roofline']['hbm']['measured_frac'] = round(traffic[0] / t_launch / 1e9 / HBM_PEAK_GBPS, 4)
        rec['roofline']['traffic_source'] = traffic[1]
        rec['roofline']['rocprof_union_us_per_launch'] = traffic[2]
        if traffic[2]:  # the same FLOPs over the rocprofv3 kernel-trace union (the committed trace of this bench)
            rec['roofline']['frac_rocprof_union'] = round(fl_all / n_all / (traffic[2] * 1e-6) / 1e12 / peak, 4)
    if args.host_io_steps > 0:
        rec['host_io'] = host_io(model, x, out, args, dev, world)
    if args.precision == 'x3':
        rec['overflow_check'] = 'per forward' if args.eager_overflow_check else \
            'lagged by one forward (engine.lagged_overflow_checks), last flag settled inside the timed region'
        if not args.eager_overflow_check:
            rec['per_forward_check'] = per_forward_check(model, x, args, dev, world, dt)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb, parity = cpu_baseline(args, model, x, out, None if args.no_cem else make_gt(args, dev, rank))
        if not args.no_cpu_variants:
            cb['variants'] = cpu_baseline_variants(args)
        rec['cpu_baseline'] = cb
        rec['parity'] = parity
    if not args.no_legs:
        rec.update(run_legs(args, dev, world, rank))
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            for key, par in reference_parity(dev).items():
                if isinstance(rec.get(key), dict):
                    rec[key]['parity'] = par
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
