"""torch.profiler view of one config-3 training step (after warm-up): the aten ops behind the PyTorch kernels that
remain in the step, with input shapes and the Python line that issued them.

    python tools/torch_prof_train.py [--min-numel N]
"""
import argparse
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
import bench_train  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--min-numel', type=int, default=4_000_000)
    a = ap.parse_args()
    from esr_amd.SRRaGAN_model import SRRaGANModel
    args = bench_train.leg_args()
    dev = torch.device('cuda')
    torch.manual_seed(1000)
    model = SRRaGANModel(bench_train.make_opt(args), device=dev)
    g = torch.Generator().manual_seed(7)
    hr = 4 * args.lr_size
    data = {'LR': torch.rand(args.batch, 3, args.lr_size, args.lr_size, generator=g).to(dev),
            'HR': torch.rand(args.batch, 3, hr, hr, generator=g).to(dev)}
    for _ in range(3):
        model.feed_data(data)
        model.optimize_parameters()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        model.feed_data(data)
        model.optimize_parameters()
        torch.cuda.synchronize()
    for ev in prof.events():
        if ev.name not in ('aten::copy_', 'aten::leaky_relu_backward', 'aten::add', 'aten::add_', 'aten::contiguous',
                           'aten::clone', 'aten::leaky_relu', 'aten::mul', 'aten::sub'):
            continue
        shapes = ev.input_shapes or []
        numel = 0
        for s in shapes:
            if s:
                n = 1
                for d in s:
                    n *= d
                numel = max(numel, n)
        if numel < a.min_numel:
            continue
        stack = [f for f in (ev.stack or []) if 'esr_amd' in f or 'bench' in f or 'torch/autograd' in f][:4]
        print(ev.name, shapes, '|', ' <- '.join(stack), flush=True)


if __name__ == '__main__':
    main()
