#!/usr/bin/env python3
"""Host-side profile of the config-3 training step (where the GPU waits for the host: the idle gaps of the kernel
trace, e.g. ≈18 ms of a 140 ms step in round 4's r4g trace).  Runs bench_train's leg (warm-up first), then cProfile
over `--steps` optimize_parameters() calls, and prints the top functions by own time and by cumulative time.
    usage: python tools/host_profile.py [--steps 5] [--warmup 4] [--top 45]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

import bench_train as BT  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=4)
    ap.add_argument('--top', type=int, default=45)
    ap.add_argument('--dump', default='gpurun_out/host_profile.pstats')
    ap.add_argument('--callers', nargs='*', default=['named_modules', r'\(parameters\)', 'refresh', 'tolist',
                                                     r'\(clone\)'])
    a = ap.parse_args()
    # the backward's host work on the calling thread, where cProfile sees it (the autograd engine otherwise runs it
    # on a device thread)
    torch.autograd.set_multithreading_enabled(False)
    from esr_amd.SRRaGAN_model import SRRaGANModel
    args = BT.leg_args(steps=a.steps, warmup=a.warmup)
    dev = torch.device('cuda', 0)
    torch.manual_seed(1000)
    model = SRRaGANModel(BT.make_opt(args), device=dev)
    g = torch.Generator(device='cpu').manual_seed(7)
    hr = 4 * args.lr_size
    data = {'LR': torch.rand(args.batch, 3, args.lr_size, args.lr_size, generator=g).to(dev),
            'HR': torch.rand(args.batch, 3, hr, hr, generator=g).to(dev)}
    for _ in range(args.warmup):
        model.feed_data(data)
        model.optimize_parameters()
    BT.settle()
    torch.cuda.synchronize()
    prof = cProfile.Profile()
    t0 = time.perf_counter()
    prof.enable()
    for _ in range(args.steps):
        model.feed_data(data)
        model.optimize_parameters()
    prof.disable()
    torch.cuda.synchronize()
    print('%d steps %.2f ms/step (under cProfile)' % (args.steps, (time.perf_counter() - t0) / args.steps * 1e3))
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats(key).print_stats(a.top)
        print('==== by %s' % key)
        print(s.getvalue())
    os.makedirs(os.path.dirname(a.dump) or '.', exist_ok=True)
    prof.dump_stats(a.dump)
    for pat in a.callers:
        s = io.StringIO()
        pstats.Stats(prof, stream=s).sort_stats('cumulative').print_callers(pat)
        print('==== callers of %s' % pat)
        print(s.getvalue()[-6000:])


if __name__ == '__main__':
    main()
