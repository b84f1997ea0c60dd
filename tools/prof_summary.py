#!/usr/bin/env python3
"""Summarise a rocprofv3 run of bench.py into profiles/<round>_kernels.md and <round>_pmc.json.

    python tools/prof_summary.py gpurun_out/prof_r1 profiles/r1

Inputs (rocprofv3 --output-format csv, -T truncated names):
  <dir>/trace/run_kernel_trace.csv   --kernel-trace --stats pass (durations)
  <dir>/pmc_fetch/run_counter_collection.csv, <dir>/pmc_write/...   separate --pmc FETCH_SIZE / WRITE_SIZE passes
Template instantiations of conv_fwd_kernel share a truncated name; they are told apart by their LDS block size.
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the
bytes of wide (16 B/lane) streaming reads, so it is doubled; WRITE_SIZE is exact for 16 B/lane stores and
uncalibrated for our 4 B/lane epilogue stores (reported as read).
"""
import csv
import json
import os
import sys
from collections import defaultdict

# rocprofv3 reports LDS_Block_Size rounded up to the 512-byte allocation granule
LDS_TAGS = {132096: 'conv3x3_n64', 90624: 'conv3x3_n32', 86016: 'upconv2x_phase', 67584: 'upconv2x_phase_n32'}
LDS_TAGS_X3 = {153600: 'x3_conv3x3_n64', 116736: 'x3_conv3x3_n32', 73728: 'x3_conv3x3_n32', 40960: 'x3_conv3x3_n32', 139264: 'x3_upconv2x_phase',
               96256: 'x3_upconv2x_phase_n32'}
LDS_TAGS_X3C = {76800: 'x3_conv3x3_n64', 67584: 'x3_conv3x3_n64', 58368: 'x3_conv3x3_n32', 49152: 'x3_conv3x3_n32', 56320: 'x3_upconv2x_phase',
                48128: 'x3_upconv2x_phase_n32', 39936: 'x3_conv3x3_regB'}


def tag(name, lds):
    name = name.replace('void (anonymous namespace)::', '')
    if name.startswith('conv_x3_ring_kernel'):
        return 'x3_conv3x3_n32'
    if name.startswith('conv_x3_narrow_kernel'):  # HR_conv1 (cout 3, planar): its own tag, as bench.py's
        return 'x3_conv3x3_n3'
    if name.startswith('conv_fwd_kernel'):
        return LDS_TAGS.get(int(lds), 'conv_fwd_kernel[lds=%s]' % lds)
    if name.startswith('conv_x3_kernel'):
        return LDS_TAGS_X3.get(int(lds), 'conv_x3_kernel[lds=%s]' % lds)
    if name.startswith('conv_x3c_kernel'):  # column-tile kernel (round 2 default for 3x3 convs)
        return LDS_TAGS_X3C.get(int(lds), 'conv_x3c_kernel[lds=%s]' % lds)
    return name


def load_trace(path):
    agg = defaultdict(lambda: [0, 0.0])
    with open(path) as f:
        for r in csv.DictReader(f):
            t = tag(r['Kernel_Name'], r['LDS_Block_Size'])
            agg[t][0] += 1
            agg[t][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    return agg


def x3_family_union(path):
    """(launches, union µs) of the x3 MFMA conv family's kernel intervals in a kernel trace — bench.py's roofline
    divides by the same union (launches of two streams overlap)."""
    iv = []
    with open(path) as f:
        for r in csv.DictReader(f):
            t = tag(r['Kernel_Name'], r['LDS_Block_Size'])
            if t.startswith('x3_') or 'hr1_sum' in t:
                iv.append((int(r['Start_Timestamp']), int(r['End_Timestamp'])))
    tot, hi = 0, None
    for a, b in sorted(iv):
        if hi is None or a > hi:
            tot, hi = tot + b - a, b
        elif b > hi:
            tot, hi = tot + b - hi, b
    return len(iv), tot / 1e3


def load_pmc(path, counter):
    agg = defaultdict(lambda: [0, 0.0])
    if not os.path.exists(path):
        return agg
    with open(path) as f:
        for r in csv.DictReader(f):
            if r['Counter_Name'] != counter:
                continue
            t = tag(r['Kernel_Name'], r['LDS_Block_Size'])
            agg[t][0] += 1
            agg[t][1] += float(r['Counter_Value'])
    return agg


def main(src, dst):
    tr = load_trace(os.path.join(src, 'trace', 'run_kernel_trace.csv'))
    fe = load_pmc(os.path.join(src, 'pmc_fetch', 'run_counter_collection.csv'), 'FETCH_SIZE')
    wr = load_pmc(os.path.join(src, 'pmc_write', 'run_counter_collection.csv'), 'WRITE_SIZE')
    total = sum(v[1] for v in tr.values())
    rows = []
    for k, (n, us) in sorted(tr.items(), key=lambda kv: -kv[1][1]):
        f = fe.get(k)
        w = wr.get(k)
        fetch = 2 * 1024 * f[1] / f[0] if f and f[0] else None   # gfx950: FETCH_SIZE (KiB) reads half
        write = 1024 * w[1] / w[0] if w and w[0] else None
        rows.append(dict(kernel=k, calls=n, avg_us=us / n, total_ms=us / 1e3, share=us / total,
                         hbm_read_bytes_per_launch=fetch, hbm_write_bytes_per_launch=write))
    os.makedirs(os.path.dirname(dst) or '.', exist_ok=True)
    n_x3, u_x3 = x3_family_union(os.path.join(src, 'trace', 'run_kernel_trace.csv'))
    json.dump({'source': src, 'kernels': rows, 'x3_family_launches': n_x3,
               'x3_family_union_us_per_launch': u_x3 / n_x3 if n_x3 else None}, open(dst + '_pmc.json', 'w'), indent=1)
    with open(dst + '_kernels.md', 'w') as f:
        f.write('| kernel | calls | avg µs | total ms | share | HBM read B/launch (FETCH_SIZE×2) | HBM write B/launch |\n')
        f.write('|---|---|---|---|---|---|---|\n')
        for r in rows:
            fmt = lambda v: '—' if v is None else '%.3e' % v  # noqa: E731
            f.write('| %s | %d | %.1f | %.2f | %.4f | %s | %s |\n' % (r['kernel'], r['calls'], r['avg_us'],
                                                                     r['total_ms'], r['share'],
                                                                     fmt(r['hbm_read_bytes_per_launch']),
                                                                     fmt(r['hbm_write_bytes_per_launch'])))
        if n_x3:
            f.write('\nx3 MFMA conv family: %d launches, union of their intervals %.2f ms = %.2f µs per launch '
                    '(bench.py roofline: FLOPs / the same union from HIP events)\n' % (n_x3, u_x3 / 1e3, u_x3 / n_x3))
    print(open(dst + '_kernels.md').read())


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
