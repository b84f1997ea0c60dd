#!/usr/bin/env python3
"""Which device allocations (hipMalloc: new caching-allocator segments) the config-3 training step still makes after
warm-up, and from where (the bench's timed_region reported device_allocs 11 over 10 steps, device_frees 0).
    usage: python tools/alloc_probe.py [--steps 6] [--warmup 4]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

import bench_train as BT  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--warmup', type=int, default=4)
    a = ap.parse_args()
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
    torch.cuda.synchronize()
    torch.cuda.memory._record_memory_history(enabled='all', context='all', stacks='python', max_entries=200000)
    for s in range(args.steps):
        n0 = torch.cuda.memory_stats().get('num_device_alloc', 0)
        model.feed_data(data)
        model.optimize_parameters()
        torch.cuda.synchronize()
        ms = torch.cuda.memory_stats()
        print('step %d: device allocs %d, reserved %.1f MB, allocated %.1f MB, peak %.1f MB, generator_step %s' % (
            s, ms.get('num_device_alloc', 0) - n0, ms['reserved_bytes.all.current'] / 2**20,
            ms['allocated_bytes.all.current'] / 2**20, ms['allocated_bytes.all.peak'] / 2**20,
            bool(model.generator_step)), flush=True)
    snap = torch.cuda.memory._snapshot()
    torch.cuda.memory._record_memory_history(enabled=None)
    for dev_trace in snap['device_traces']:
        for ev in dev_trace:
            if ev['action'] not in ('segment_alloc', 'segment_free', 'segment_map', 'segment_unmap'):
                continue
            frames = [f for f in ev.get('frames', []) if 'esr_amd' in f['filename'] or 'torch/optim' in f['filename']
                      or 'bench' in f['filename'] or 'torch/autograd' in f['filename']]
            print('%s %.2f MB stream %s' % (ev['action'], ev['size'] / 2**20, ev.get('stream')))
            for f in frames[:8]:
                print('     %s:%d %s' % (f['filename'].split('explorable-super-resolution_old_amd/')[-1], f['line'],
                                         f['name']))


if __name__ == '__main__':
    main()
