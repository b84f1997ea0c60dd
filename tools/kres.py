#!/usr/bin/env python3
"""Kernel resource table (VGPRs, AGPRs, spills, LDS, occupancy) of one .hip file for gfx950:
python tools/kres.py <file.hip> [extra hipcc flags]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ['/opt/rocm/bin/hipcc', '-O3', '--offload-arch=gfx950', '-std=c++17', '-fPIC',
       '-I/root/repo/include', '-I/root/repo/explorable-super-resolution_old_amd/csrc', '-c', src, '-o', '/tmp/kres.o',
       '-Rpass-analysis=kernel-resource-usage'] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r'remark: (.*?) \[-Rpass', line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith('Function Name:'):
        cur = {'name': subprocess.run(['c++filt'], input=t.split(':', 1)[1].strip(), capture_output=True,
                                      text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None and ':' in t:
        k, v = t.split(':', 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print('%-4s vgpr %-4s agpr %-4s spillV %-4s spillS %-4s lds %-7s occ %-2s %s' % (
        '', r.get('VGPRs'), r.get('AGPRs'), r.get('VGPRs Spill'), r.get('SGPRs Spill'),
        r.get('LDS Size [bytes/block]'), r.get('Occupancy [waves/SIMD]'), r['name'][:150]))
