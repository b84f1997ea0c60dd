#!/usr/bin/env python3
"""The largest GPU idle gaps inside the last part of a rocprofv3 kernel trace, with the kernels on either side.

    python tools/trace_gaps.py TRACE.csv LAST_MS [N]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
last_ms = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
t_end = max(e[1] for e in ev)
ev = [e for e in ev if e[0] >= t_end - last_ms * 1e6]
t0 = ev[0][0]


def short(k):
    return k.replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:60]


gaps, end, prev = [], ev[0][1], ev[0][2]
for s, e, k in ev[1:]:
    if s > end:
        gaps.append(((s - end) / 1e3, (end - t0) / 1e6, prev, k))
    if e > end:
        end, prev = e, k
tot = sum(g[0] for g in gaps)
print('window %.1f ms, %d kernels, idle %.1f ms in %d gaps (>= 20 us: %.1f ms in %d)' % (
    (t_end - t0) / 1e6, len(ev), tot / 1e3, len(gaps), sum(g[0] for g in gaps if g[0] >= 20) / 1e3,
    sum(1 for g in gaps if g[0] >= 20)))
for us, at, a, b in sorted(gaps, reverse=True)[:n]:
    print('%8.1f us at %8.2f ms  after %-60s before %s' % (us, at, short(a), short(b)))
