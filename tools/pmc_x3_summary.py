#!/usr/bin/env python3
"""Per-kernel means of the counters of tools/pmc_x3.sh's or tools/pmc_bench_sq.sh's passes (rocprofv3 counter_collection.csv
files)."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(out, 'p*', '**', '*counter_collection.csv'), recursive=True)):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name'][:60]
        if 'conv_x3' not in name:
            continue
        key = (name, r.get('LDS_Block_Size', ''))
        vals[key][r['Counter_Name']].append(float(r['Counter_Value']))
for key, cs in vals.items():
    print('==', key[0], 'lds', key[1])
    for c in sorted(cs):
        v = cs[c]
        print('   %-28s %14.4g  (n=%d)' % (c, sum(v) / len(v), len(v)))
