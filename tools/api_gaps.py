"""For each GPU idle gap of a rocprofv3 kernel trace, the HIP API calls the host made from the end of the kernel before
it to the launch that ended it (tools/prof_train_api.sh output).
    python tools/api_gaps.py TRACE_DIR [LAST_MS=420] [MIN_US=300]
"""
import csv
import glob
import os
import sys

_TRIVIAL = {'hipGetDevice', 'hipSetDevice', 'hipGetLastError', 'hipGetDeviceCount', 'hipPeekAtLastError',
            'hipDeviceGetAttribute', 'hipGetDeviceProperties', 'hipStreamGetCaptureInfo', 'hipStreamIsCapturing'}
d = sys.argv[1]
last = float(sys.argv[2]) if len(sys.argv) > 2 else 420.0
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 300.0


def load(pat):
    f = glob.glob(os.path.join(d, '**', pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


k = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in load('*kernel_trace.csv'))
api = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Function'], r.get('Thread_Id', ''))
             for r in load('*hip_api_trace.csv'))
t_end = max(e[1] for e in k)
t0 = t_end - last * 1e6
end, prev = None, None
for s, e, n in k:
    if s < t0:
        end = max(end or 0, e)
        continue
    if end is not None and s - end >= min_us * 1e3:
        print('%8.1f us gap at %8.2f ms  after %s  before %s' % ((s - end) / 1e3, (end - t0) / 1e6, prev[:60], n[:60]))
        for a in api:
            if a[1] >= end - 50e3 and a[0] <= s:
                dur = (a[1] - a[0]) / 1e3
                if a[2] in _TRIVIAL:
                    continue
                if dur >= 20 or a[2] not in ('hipLaunchKernel', 'hipExtModuleLaunchKernel', 'hipModuleLaunchKernel'):
                    print('      %9.3f ms  %8.1f us  %-28s tid %s' % ((a[0] - t0) / 1e6, dur, a[2], a[3]))
    if end is None or e > end:
        end, prev = e, n
