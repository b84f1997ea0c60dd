"""GPU parity of the CEM image helpers (esr_amd/cem_ops.py on the csrc/esr_cem.hip stencils) against the reference's
own outputs (tests/golden/cem_np_*.npz, made by tests/golden/make_golden.py from CEMnet.py / imresize_CEM.py):

  imresize ↓4 / ↑4 (edge and zero padding, HWC and HW), DT_Satisfying_Upscale, Project_2_kernel_subspace,
  Enforce_DT_on_Image_Pair (LR-sized and HR-sized sources)                          normwise 1e-5 (fp32 vs float64)
  the batched device-tensor form of the same helpers                                equal to the per-image results
  CEM_PyTorch.Update_Filters (kernel swapped into a built model)                    equal to a freshly built model
"""
import numpy as np
import pytest
import torch

from conftest import normwise_rel

import esr_amd
from esr_amd import CEMnet as C
from esr_amd.imresize_CEM import imresize
from oracle.recipe import seeded_inputs, seeded_params, synthetic_learned_kernel

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _load(name):
    from conftest import golden
    d = golden('cem_np_' + name)
    k = synthetic_learned_kernel() if name == 'learned13' else None
    return d, k, C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=k)


@pytest.mark.parametrize('name', ['bicubic', 'learned13'])
def test_imresize_vs_reference(gpu_device, name):
    d, k, _ = _load(name)
    cases = dict(down=imresize(d['hr'], [1 / 4], kernel=k),
                 down_zp=imresize(d['hr'], [1 / 4], kernel=k, use_zero_padding=True),
                 down_gray=imresize(d['gray'], [1 / 4], kernel=k),
                 up=imresize(d['lr'], [4], kernel=k),
                 up_zp=imresize(d['lr'], [4], kernel=k, use_zero_padding=True),
                 up_shape=imresize(d['lr'], output_shape=[80, 96], kernel=k))
    for key, v in cases.items():
        assert v.shape == d[key].shape, key
        assert normwise_rel(v, d[key]) < TOL, (key, normwise_rel(v, d[key]))


@pytest.mark.parametrize('name', ['bicubic', 'learned13'])
def test_cem_numpy_helpers_vs_reference(gpu_device, name):
    d, _, cem = _load(name)
    cases = dict(dt_up=cem.DT_Satisfying_Upscale(d['lr']), project=cem.Project_2_kernel_subspace(d['hr']),
                 enforce=cem.Enforce_DT_on_Image_Pair(d['lr'], d['hr']),
                 enforce_same=cem.Enforce_DT_on_Image_Pair(d['hr2'], d['hr']))
    for key, v in cases.items():
        assert v.shape == d[key].shape, key
        assert normwise_rel(v, d[key]) < TOL, (key, normwise_rel(v, d[key]))


@pytest.mark.parametrize('name', ['bicubic', 'learned13'])
def test_batched_device_helpers_equal_per_image(gpu_device, name):
    """Device tensors [B, C, H, W] go through the same launches with B*C planes (padded to a multiple of 3)."""
    d, k, cem = _load(name)
    hr = torch.from_numpy(np.stack([d['hr'], d['hr2']]).astype(np.float32)).permute(0, 3, 1, 2).to(gpu_device)
    lr = torch.from_numpy(d['lr'].astype(np.float32)).permute(2, 0, 1)[None].repeat(2, 1, 1, 1).to(gpu_device)
    outs = dict(down=imresize(hr, [1 / 4], kernel=k), project=cem.Project_2_kernel_subspace(hr),
                enforce=cem.Enforce_DT_on_Image_Pair(lr, hr))
    torch.cuda.synchronize()
    for i, im in enumerate((d['hr'], d['hr2'])):
        for key, ref in (('down', imresize(im, [1 / 4], kernel=k)), ('project', cem.Project_2_kernel_subspace(im)),
                         ('enforce', cem.Enforce_DT_on_Image_Pair(d['lr'], im))):
            got = outs[key][i].permute(1, 2, 0).cpu().numpy()
            assert normwise_rel(got, ref) < 1e-7, (key, i)
    # a plane count that is not a multiple of 3 (2 images x 5 channels)
    five = hr[:, 0:1].repeat(1, 5, 1, 1)
    got = imresize(five, [1 / 4], kernel=k).cpu().numpy()
    ref = imresize(np.moveaxis(five[1].cpu().numpy(), 0, -1), [1 / 4], kernel=k)
    assert normwise_rel(np.moveaxis(got[1], 0, -1), ref) < 1e-7


def test_update_filters_equals_fresh_model(gpu_device):
    """A bicubic CEM model re-targeted to a learned kernel (Set_Upscale_Kernel + Update_Filters) computes exactly what
    a model built with that kernel computes, in eval (pre-pad by the new margin) and train mode."""
    k = synthetic_learned_kernel()

    def build(kernel):
        net = esr_amd.RRDBNet(3, 3, 64, 1, num_latent_channels=0)
        cem = C.CEMnet(C.Get_CEM_Config(4), upscale_kernel=kernel)
        return cem, cem.WrapArchitecture_PyTorch(net)

    cem_a, a = build(None)
    _, b = build(k)
    params = seeded_params([(n, tuple(v.shape)) for n, v in a.state_dict().items() if 'Filter' not in n], 31,
                           w_scale=0.5)
    for m in (a, b):
        m.load_state_dict({n: torch.from_numpy(v) for n, v in params.items()}, strict=False)
        m.to(gpu_device)
    lr, _ = seeded_inputs(32, (2, 3, 16, 20))
    x = torch.from_numpy(lr).to(gpu_device)
    with torch.no_grad():
        a.eval()
        before = a(x)
        a.Update_Filters(cem_a.Set_Upscale_Kernel(k))
        for mode in (False, True):
            a.train(mode)
            b.train(mode)
            ya, yb = a(x), b(x)
            assert ya.shape == yb.shape and torch.equal(ya, yb), mode
        assert normwise_rel(before.cpu(), b.eval()(x).cpu()) > 1e-3  # the kernel swap did change the output
