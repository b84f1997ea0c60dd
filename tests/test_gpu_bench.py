"""The bench.py driver contract on a small workload (subprocess, one GPU): one JSON line with the required keys,
a roofline object for the dominant kernel and a bounded CPU-baseline leg; the output of that run matched against
the CPU reference (bench.py's own `parity` record)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract():
    cmd = [sys.executable, os.path.join(REPO, 'bench.py'), '--steps', '2', '--warmup', '1', '--batch', '2',
           '--lr-size', '32', '--nb', '1', '--cpu-images', '1', '--no-legs']
    res = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=110)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, res.stdout[-2000:]
    rec = json.loads(lines[0])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config', 'roofline', 'cpu_baseline'):
        assert k in rec, k
    assert rec['n_gpus'] == 1 and rec['steps'] == 2 and rec['warmup'] == 1 and rec['value'] > 0
    assert 'workload' in rec['config']
    rf = rec['roofline']
    assert rf['bound'] in ('hbm', 'mfma') and rf['unit'] in ('GB/s', 'TFLOP/s')
    assert rf['achieved'] > 0 and rf['peak'] > 0 and abs(rf['frac'] - rf['achieved'] / rf['peak']) < 1e-3
    cb = rec['cpu_baseline']
    assert cb['value'] > 0 and cb['cores'] >= 1 and cb['kind'] in ('port', 'reference') and cb['sample']
    assert rec['parity']['normwise_rel_err_vs_cpu_ref'] < 1e-4
