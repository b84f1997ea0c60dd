"""`--gpus N` means N ranks: the bench scripts start N ranks themselves when run directly, and
refuse a launcher whose WORLD_SIZE disagrees.  CPU only: `--launcher-check` brings the ranks up on gloo and stops
before any GPU call; the N-GPU run takes the same path up to that point (bench_launch.ranks)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, *args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR',
                                                               'MASTER_PORT')}
    env.update(env_extra or {})
    env['OMP_NUM_THREADS'] = '1'
    return subprocess.run([sys.executable, os.path.join(REPO, script)] + list(args), cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=240)


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith('{')]


@pytest.mark.parametrize('script', ['bench.py', 'bench_train.py', 'bench_zopt.py'])
def test_gpus_2_starts_two_ranks(script):
    r = _run(script, '--gpus', '2', '--launcher-check')
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    rec = lines[0]
    assert rec['n_gpus'] == 2
    assert sorted(rec['ranks']) == [0, 1]
    assert rec['world_sizes'] == [2, 2]
    assert sorted(rec['local_ranks']) == [0, 1]


def test_gpus_1_is_one_rank():
    r = _run('bench.py', '--launcher-check')
    assert r.returncode == 0, r.stderr[-2000:]
    assert _json_lines(r.stdout)[0]['world_sizes'] == [1]


def test_external_launcher_world_size_must_match():
    r = _run('bench.py', '--gpus', '4', '--launcher-check',
             env_extra={'WORLD_SIZE': '2', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert r.returncode != 0
    assert 'WORLD_SIZE=2' in r.stderr
