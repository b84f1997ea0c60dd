#!/usr/bin/env python3
"""Attribute the GPU's idle gaps in the config-3 training step to what the host was doing at the time.

torch.profiler (CPU + GPU activities, Python tracer) over `--steps` optimize_parameters() calls after warm-up; every
gap between consecutive GPU kernels / copies of at least `--min-us` is printed with the host's Python call stack
(esr_amd frames, innermost last) and the runtime call in flight at the moment the gap ended (the launch that ended
it), and the gaps are summed per innermost esr_amd frame.
    usage: python tools/gap_attrib.py [--steps 2] [--min-us 40] [--out gpurun_out/gap_attrib.txt]
"""
import argparse
import bisect
import collections
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench_train as BT  # noqa: E402


def _short(name):
    for pre in ('/tmp/', REPO + '/'):
        if pre in name:
            name = name.split('explorable-super-resolution_old_amd/')[-1]
    return name[:110]


def analyse(trace, min_us, out):
    ev = trace['traceEvents']
    gpu = sorted((e for e in ev if e.get('ph') == 'X' and e.get('cat') in ('kernel', 'gpu_memcpy', 'gpu_memset')),
                 key=lambda e: e['ts'])
    py = [e for e in ev if e.get('ph') == 'X' and e.get('cat') == 'python_function']
    rt = sorted((e for e in ev if e.get('ph') == 'X' and e.get('cat') == 'cuda_runtime'), key=lambda e: e['ts'])
    main_tid = collections.Counter(e['tid'] for e in py).most_common(1)[0][0] if py else None
    py = sorted((e for e in py if e['tid'] == main_tid), key=lambda e: e['ts'])
    py_starts = [e['ts'] for e in py]
    rt_starts = [e['ts'] for e in rt]

    def stack_at(t, every=False):
        i = bisect.bisect_right(py_starts, t)
        frames = [e for e in py[max(0, i - 4000):i] if e['ts'] <= t <= e['ts'] + e['dur']]
        frames.sort(key=lambda e: e['ts'])
        return [_short(e['name']) for e in frames if every or 'esr_amd' in e['name'] or 'bench' in e['name']]

    def calls_in(t0, t1):  # the Python calls made on the host thread during [t0, t1] that took >= 5 % of it
        i0, i1 = bisect.bisect_left(py_starts, t0), bisect.bisect_right(py_starts, t1)
        return ['%7.1f us  %s' % (e['dur'], _short(e['name'])) for e in py[i0:i1] if e['dur'] >= 0.05 * (t1 - t0)]

    def rt_at(t):
        i = bisect.bisect_right(rt_starts, t)
        for e in reversed(rt[max(0, i - 50):i]):
            if e['ts'] <= t <= e['ts'] + e['dur']:
                return e['name']
        return rt[i - 1]['name'] if i else '-'

    busy = sum(e['dur'] for e in gpu)
    span = gpu[-1]['ts'] + gpu[-1]['dur'] - gpu[0]['ts']
    lines = ['GPU span %.2f ms, busy %.2f ms (%d ops), idle %.2f ms' % (span / 1e3, busy / 1e3, len(gpu),
                                                                      (span - busy) / 1e3)]
    per_frame = collections.Counter()
    per_frame_n = collections.Counter()
    small = 0.0
    end = gpu[0]['ts'] + gpu[0]['dur']
    prev = gpu[0]
    for e in gpu[1:]:
        gap = e['ts'] - end
        if gap >= min_us:
            st = stack_at(end + gap / 2)
            key = st[-1] if st else '(no esr_amd frame)'
            per_frame[key] += gap
            per_frame_n[key] += 1
            lines.append('%8.1f us  after %-40s before %-40s | rt %s' % (gap, prev['name'][:40], e['name'][:40],
                                                                      rt_at(e['ts'] - 1)))
            lines.extend('      ' + f for f in st[-6:])
            if gap >= 1000:
                lines.extend('    | ' + f for f in stack_at(end + gap / 2, every=True)[-12:])
                lines.extend('    > ' + f for f in calls_in(end, e['ts'])[:30])
        elif gap > 0:
            small += gap
        if e['ts'] + e['dur'] > end:
            end, prev = e['ts'] + e['dur'], e
    lines.append('gaps below %d us: %.2f ms in total' % (min_us, small / 1e3))
    lines.append('==== gaps >= %d us by innermost esr_amd frame (ms, count)' % min_us)
    for k, v in per_frame.most_common(40):
        lines.append('%8.2f %4d  %s' % (v / 1e3, per_frame_n[k], k))
    with open(out, 'w') as f:
        f.write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:1] + lines[-42:]), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--warmup', type=int, default=4)
    ap.add_argument('--min-us', type=float, default=40)
    ap.add_argument('--out', default='gpurun_out/gap_attrib.txt')
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
    BT.settle()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(args.steps):
            model.feed_data(data)
            model.optimize_parameters()
        torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out) or '.', exist_ok=True)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, 'trace.json')
        prof.export_chrome_trace(path)
        with open(path) as f:
            trace = json.load(f)
    analyse(trace, a.min_us, a.out)


if __name__ == '__main__':
    main()
