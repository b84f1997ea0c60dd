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
    ap.add_argument('--host', action='store_true', help='print the ops by self CPU time instead')
    ap.add_argument('--device', action='store_true', help='print the aten ops by their device (kernel) time, with the '
                    'input shapes and the calling Python frames')
    ap.add_argument('--syncs', action='store_true', help='count the Python call sites of tensor -> host scalar '
                    'conversions (item / float / int / bool / iteration) in one step')
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
    if a.syncs:
        import collections
        import traceback
        cnt = collections.Counter()

        def wrap(name):
            orig = getattr(torch.Tensor, name)

            def f(self, *args, **kw):
                if self.is_cuda:
                    cnt[(name, ''.join(traceback.format_stack(limit=5)[:-1]))] += 1
                return orig(self, *args, **kw)
            setattr(torch.Tensor, name, f)
        for name in ('item', '__float__', '__int__', '__bool__', '__iter__', 'tolist', '__index__'):
            wrap(name)
        model.feed_data(data)
        model.optimize_parameters()
        torch.cuda.synchronize()
        for (name, st), n in cnt.most_common(12):
            print('%5d x %s\n%s' % (n, name, st), flush=True)
        return
    if a.device:
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                     with_stack=True) as prof:
            model.feed_data(data)
            model.optimize_parameters()
            torch.cuda.synchronize()
        print(prof.key_averages(group_by_input_shape=True).table(sort_by='self_cuda_time_total', row_limit=45,
                                                                 max_name_column_width=40, max_shapes_column_width=70),
              flush=True)
        agg = {}
        for ev in prof.events():
            if not ev.name.startswith('aten::') or ev.self_device_time_total <= 0:
                continue
            stack = [f.split('explorable-super-resolution_old_amd/')[-1] for f in (ev.stack or [])
                     if 'esr_amd' in f][:3]
            k = (ev.name, str(ev.input_shapes)[:90], ' <- '.join(stack))
            a = agg.setdefault(k, [0, 0.0])
            a[0] += 1
            a[1] += ev.self_device_time_total
        for (name, shp, st), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
            print('%8.1f us %3d x %-28s %-90s | %s' % (t, n, name, shp, st), flush=True)
        return
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        model.feed_data(data)
        model.optimize_parameters()
        torch.cuda.synchronize()
    if a.host:
        print(prof.key_averages().table(sort_by='self_cpu_time_total', row_limit=40), flush=True)
        print(prof.key_averages(group_by_stack_n=3).table(sort_by='self_cpu_time_total', row_limit=25), flush=True)
        return
    for ev in prof.events():
        if ev.name not in ('aten::copy_', 'aten::leaky_relu_backward', 'aten::add', 'aten::add_', 'aten::contiguous',
                           'aten::clone', 'aten::leaky_relu', 'aten::mul', 'aten::sub', 'aten::cat', 'aten::sum',
                           'aten::mean', 'aten::norm', 'aten::linalg_vector_norm', 'aten::where', 'aten::pow',
                           'aten::div', 'aten::abs', 'aten::lerp_', 'aten::addcmul_', 'aten::index_select',
                           'aten::index', 'aten::mul_', 'aten::zero_', 'aten::fill_', 'aten::sqrt', 'aten::clamp'):
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
