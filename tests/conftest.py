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


def fixture_upscale(d):
    """The generator's scale factor of an rrdb_* fixture (×4 unless the fixture records another)."""
    return int(d['upscale']) if 'upscale' in d else 4


def fixture_input(d):
    """Model input exactly as SRRaGANModel.ConcatLatent builds it (raw view of the HR Z into 3·sf² LR channels)."""
    import torch
    lr = torch.from_numpy(d['lr'])
    if int(d['latent']):
        B, _, h, w = lr.shape
        sf = fixture_upscale(d)
        return torch.cat([torch.from_numpy(d['z']).reshape(B, 3 * sf * sf, h, w), lr], 1)
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


@pytest.fixture(scope='session')
def ablation_lib(gpu_device):
    """The ablation library (exp_lib/libesr_exp.so, csrc/esr_ablation.h): the product ABI built from the same sources
    plus the process-wide kernel-selection setters and the non-default kernel variants.  Variant-equality tests run
    the default on the product library and the variants here; the product library has no selection state."""
    from esr_amd import _lib
    try:
        return _lib.load_ablation()
    except _lib.ESRLibraryError as e:
        pytest.skip('ablation library not built: %s' % e)


@pytest.fixture
def via_ablation(ablation_lib):
    """Route the host layer's launches (esr_amd modules call _lib.load()) to the ablation library for one test."""
    from esr_amd import _lib
    prev = _lib._lib
    _lib._lib = ablation_lib
    try:
        yield ablation_lib
    finally:
        _lib._lib = prev


def l2_rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.sqrt(((a - b) ** 2).sum() / max((b ** 2).sum(), 1e-300)))


def grad_parity(a, exact, base, factor=5.0, floor=1e-4):
    """Gradient parity "as accurate as the reference's own fp32": relative L2 error of `a` against the float64
    oracle `exact` must be within `factor`× that of an independent fp32 evaluation `base` (the reference's golden
    values or the oracle in fp32), with an absolute floor (1e-4: either side may be the one that flips a kink).
    The max-norm is not used for gradients: a pre-activation within fp32 rounding of 0 takes LeakyReLU slope 1 in
    one evaluation and 0.2 in another, and each such kink flip
    changes the gradient of its whole receptive field by O(1) locally (tests/test_oracle_golden.py::
    test_fp32_gradients_have_kink_flips: the oracle's own fp32 vs fp64 input gradient differs by 7e-3 max-norm, 1.7e-3
    L2 at 40x40 LR)."""
    e, eb = l2_rel(a, exact), l2_rel(base, exact)
    return e <= max(floor, factor * eb), 'l2 %.2e (fp32 reference %.2e, max-norm %.2e)' % (e, eb, normwise_rel(a, exact))


def oracle_grads(params, lr, z, R, nb, latent, design, pre_pad, dtype, want_params=True, sf=4):
    """Gradients of Σ out·R through the oracle (CEM_PyTorch ∘ RRDBNet) in `dtype`: {'param:<key>', 'dz', 'dlr'}.
    `params` are reference-keyed numpy arrays (prefix stripped here); lr/z numpy NCHW (z = HR latent or None)."""
    import torch
    from oracle import esr_oracle as O
    P = {k: torch.as_tensor(v).to(dtype).requires_grad_(want_params) for k, v in O.strip_prefix(params).items()}
    lr_t = torch.as_tensor(lr).to(dtype).requires_grad_(True)
    B, _, h, w = lr_t.shape
    x = lr_t
    z_t = None
    if latent:
        z_t = torch.as_tensor(z).to(dtype).requires_grad_(True)
        x = torch.cat([z_t.reshape(B, -1, h, w), lr_t], 1)
    out = O.sr_forward(x, P, nb, latent, design, pre_pad=pre_pad, sf=sf)
    (out * torch.as_tensor(R).to(dtype)).sum().backward()
    g = {'dlr': lr_t.grad.double().numpy()}
    if z_t is not None:
        g['dz'] = z_t.grad.double().numpy()
    if want_params:
        for k, v in P.items():
            if v.grad is not None:
                g['param:' + k] = v.grad.double().numpy()
    return g
