#!/usr/bin/env python3
"""Host side of the config-3 training step: is the step launch-bound?  Per step: the host time to enqueue one
optimize_parameters() (no sync), the synchronised wall time, Python GC pauses; then a cProfile of the host work of
a few steps (top entries by own time and cumulative time).

    python tools/train_host_probe.py [--steps 6] [--gc-freeze] > gpurun_out/host_probe.txt
"""
import argparse
import cProfile
import gc
import io
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

import bench_train  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--gc-freeze', action='store_true')
    a = ap.parse_args()
    from esr_amd.SRRaGAN_model import SRRaGANModel
    args = bench_train.leg_args()
    dev = torch.device('cuda', 0)
    torch.manual_seed(1000)
    model = SRRaGANModel(bench_train.make_opt(args), device=dev)
    g = torch.Generator(device='cpu').manual_seed(7)
    hr = 4 * args.lr_size
    data = {'LR': torch.rand(args.batch, 3, args.lr_size, args.lr_size, generator=g).to(dev),
            'HR': torch.rand(args.batch, 3, hr, hr, generator=g).to(dev)}
    pauses = []
    t_gc = [0.0]

    def cb(phase, info):
        if phase == 'start':
            t_gc[0] = time.perf_counter()
        else:
            pauses.append((info['generation'], (time.perf_counter() - t_gc[0]) * 1e3))
    gc.callbacks.append(cb)
    for _ in range(2):
        model.feed_data(data)
        model.optimize_parameters()
    torch.cuda.synchronize()
    if a.gc_freeze:
        gc.collect()
        gc.freeze()
    print('gc counts', gc.get_count(), 'thresholds', gc.get_threshold(), 'frozen', gc.get_freeze_count(), flush=True)
    def mem():
        m = torch.cuda.memory_stats(dev)
        return (m.get('num_alloc_retries', 0), m.get('num_device_alloc', 0), m.get('num_device_free', 0),
                round(m.get('reserved_bytes.all.current', 0) / 2**30, 1), round(m.get('allocated_bytes.all.peak', 0) / 2**30, 1))
    print('mem (retries, device allocs, device frees, reserved GiB, peak allocated GiB):', mem(), flush=True)
    for i in range(a.steps):
        pauses.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model.feed_data(data)
        model.optimize_parameters()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print('step %d: host enqueue %.2f ms, wall %.2f ms, gc pauses %s' %
              (i, (t1 - t0) * 1e3, (t2 - t0) * 1e3, [(gen, round(ms, 2)) for gen, ms in pauses]), 'mem', mem(),
              flush=True)
    # back-to-back (as bench_train times them)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        model.feed_data(data)
        model.optimize_parameters()
    torch.cuda.synchronize()
    print('back-to-back: %.2f ms/step' % ((time.perf_counter() - t0) / a.steps * 1e3), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        model.feed_data(data)
        model.optimize_parameters()
    torch.cuda.synchronize()
    pr.disable()
    for key in ('tottime', 'cumulative'):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(35)
        print(s.getvalue(), flush=True)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).print_callers('tensor|item|run_backward|parameters')
    print(s.getvalue(), flush=True)


if __name__ == '__main__':
    main()
