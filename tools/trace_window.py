"""Per-kernel time inside the last part of a rocprofv3 kernel trace (the timed steps of a bench run).

    python tools/trace_window.py TRACE.csv START_MS [STEPS]   (START_MS from the trace's first kernel; a negative
                                                              value -X takes the trace's last X ms)
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
start = float(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], r['LDS_Block_Size']) for r in rows)
t0 = ev[0][0]
if start < 0:
    t0 = max(e[1] for e in ev) + start * 1e6
    start = 0.0
ev = [e for e in ev if (e[0] - t0) / 1e6 >= start]
span = (max(e[1] for e in ev) - ev[0][0]) / 1e6
busy, end = 0, 0
for s, e, _, _ in ev:
    s = max(s, end)
    if e > s:
        busy += e - s
        end = e
agg = defaultdict(lambda: [0, 0.0])
for s, e, n, lds in ev:
    n = n.replace('void ', '').replace('(anonymous namespace)::', '')
    k = n.split('(')[0][:60] + (' lds%s' % lds if 'conv' in n else '')
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e6
print('window %.1f ms, busy %.1f ms (%.1f%%), per step: span %.1f busy %.1f' % (span, busy / 1e6, 100 * busy / 1e6 / span,
                                                                             span / steps, busy / 1e6 / steps))
tot = sum(v[1] for v in agg.values())
print('| kernel | calls/step | ms/step | share |\n|---|---|---|---|')
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[4]) if len(sys.argv) > 4 else 30]:
    print('| %s | %d | %.2f | %.3f |' % (k, c // steps, t / steps, t / tot))
