"""CPU tests of the Z-optimisation host logic (Z_optimization.py:271-325): tanh parametrisation, masks, ArcTanH,
and the refusal of the objectives that are broken in the reference (the others: test_zobj_host.py)."""
import numpy as np
import pytest
import torch

from esr_amd.Z_optimization import ArcTanH, Optimizable_Z, TV_Loss, Z_optimizer

CPU = torch.device('cpu')


def test_arctanh_inverts_tanh_parametrisation():
    z = torch.linspace(-0.99, 0.99, 101)
    assert torch.allclose(torch.tanh(ArcTanH(z)), z, atol=1e-6)
    m = Optimizable_Z([1, 3, 4, 4], Z_range=2.0, initial_pre_tanh_Z=ArcTanH(torch.full((1, 3, 4, 4), 0.25)),
                      device=CPU)
    assert torch.allclose(m(), torch.full((1, 3, 4, 4), 0.5), atol=1e-6)


def test_z_mask_keeps_masked_out_region():
    init = torch.zeros(1, 3, 4, 4)
    mask = np.zeros((4, 4), dtype=np.float32)
    mask[:2] = 1
    m = Optimizable_Z([1, 3, 4, 4], Z_range=1.0, initial_pre_tanh_Z=init, Z_mask=mask, device=CPU)
    m.Z.data += 1.0
    z = m()
    assert torch.all(z[..., 2:, :] == 0) and torch.all(z[..., :2, :] > 0.7)


def test_initializer_broadcast_and_shape_check():
    m = Optimizable_Z([3, 3, 4, 4], initial_pre_tanh_Z=torch.ones(1, 3, 4, 4), device=CPU)
    assert torch.all(m.Z.data[0] == 1) and torch.all(m.Z.data[1:] == 0)
    with pytest.raises(AssertionError):
        Optimizable_Z([3, 3, 4, 4], initial_pre_tanh_Z=torch.ones(2, 3, 4, 4), device=CPU)


def test_tv_loss_per_image():
    x = torch.zeros(2, 3, 4, 4)
    x[1, :, :, 2:] = 1
    tv = TV_Loss(x)
    assert tv[0] == 0 and abs(float(tv[1]) - 4 * 3 / (3 * 4 * 3)) < 1e-7


@pytest.mark.parametrize('objective', ['desired_SVD', 'VGG'])
def test_objectives_broken_in_the_reference_are_refused(objective):
    """desired_SVD (FilterLoss reads data keys the Z optimiser never passes: KeyError in the reference) and VGG (its
    feature extractor cannot be built: NameError) raise instead of silently optimising something else."""
    class M:
        device = CPU
    with pytest.raises(NotImplementedError):
        Z_optimizer(objective, [8, 8], M(), 1.0, 3, initial_LR=0.1)


def test_masked_plain_l1_is_refused():
    """'l1' with an image mask: the reference builds a masked-L1 closure over a mask it only defines for 'scribble'
    (NameError at the first iteration); here it raises at construction."""
    class M:
        device = CPU
        fake_H = torch.zeros(1, 3, 8, 8)
    with pytest.raises(NotImplementedError):
        Z_optimizer('l1', [8, 8], M(), 1.0, 3, initial_LR=0.1, image_mask=np.ones((8, 8)), Z_mask=np.ones((8, 8)))
