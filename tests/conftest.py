import glob
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, 'explorable-super-resolution_old_amd')
GOLDEN = os.path.join(REPO, 'tests', 'golden')
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a ROCm GPU (MI355X) and the built libesr_amd.so')


def golden(name):
    return np.load(os.path.join(GOLDEN, name + '.npz'))


def golden_names(prefix):
    return sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, prefix + '*.npz')))


def fixture_params(d):
    """Regenerate the seeded parameters of an rrdb_* fixture (oracle/recipe.py)."""
    from oracle.recipe import seeded_params
    keys = json.loads(str(d['keys']))
    return keys, seeded_params(keys, int(d['seed']), float(d['w_scale']))


def fixture_input(d):
    """Model input exactly as SRRaGANModel.ConcatLatent builds it (raw view of the HR Z into 48 LR channels)."""
    import torch
    lr = torch.from_numpy(d['lr'])
    if int(d['latent']):
        B, _, h, w = lr.shape
        return torch.cat([torch.from_numpy(d['z']).reshape(B, 48, h, w), lr], 1)
    return lr


def normwise_rel(a, b):
    """max|a-b| / max|b| — the parity metric of SURVEY.md §8(d)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.fixture(scope='session')
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no ROCm device')
    return torch.device('cuda:0')
