"""GPU parity of the Z-optimisation loop (Z_optimization.py:326-660): Optimizable_Z (tanh), frozen CEM-wrapped latent
generator on the HIP path (forward + input-gradient sweep), Adam on Z — against the same loop run on the oracle's
autograd on CPU.  Tolerance: normwise 1e-4 on the final Z after a few Adam steps (fp32, observed ~1e-6)."""
import numpy as np
import pytest
import torch

from conftest import grad_parity

from esr_amd.SRRaGAN_model import SRRaGANModel
from esr_amd.Z_optimization import ArcTanH, Z_optimizer
from oracle import esr_oracle as O
from oracle.recipe import seeded_inputs, seeded_params

pytestmark = pytest.mark.gpu


def _opt(nb, cem=1):
    return {'is_train': False, 'scale': 4, 'gpu_ids': [0], 'range': [0, 1],
            'network_G': {'which_model_G': 'RRDB_net', 'CEM_arch': cem, 'latent_input': 'all_layers',
                          'latent_input_domain': 'HR_downscaled', 'latent_channels': 'SVDinNormedOut_structure_tensor',
                          'norm_type': None, 'mode': 'CNA', 'nf': 64, 'nb': nb, 'in_nc': 3, 'out_nc': 3, 'gc': 32}}


@pytest.mark.parametrize('objective', ['l1', 'max_STD'])
def test_z_optimizer_loop_matches_oracle(gpu_device, objective):
    nb, B, h, w, iters, lr_rate = 1, 2, 12, 12, 3, 0.05
    torch.manual_seed(0)
    model = SRRaGANModel(_opt(nb), device=gpu_device)
    sd = model.netG.module.state_dict()
    params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], 71, w_scale=0.5)
    model.netG.module.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    lr, z0 = seeded_inputs(72, (B, 3, h, w), (B, 3, 4 * h, 4 * w), z_mode='pixel')
    hr = np.random.default_rng(73).random((B, 3, 4 * h, 4 * w)).astype(np.float32)
    data = {'LR': torch.from_numpy(lr).to(gpu_device), 'HR': torch.from_numpy(hr).to(gpu_device),
            'Z': torch.from_numpy(0.9 * z0).to(gpu_device)}
    model.feed_data(data, need_HR=False)
    model.test()
    model.netG.eval()  # GUI usage: eval (CEM pre-pad) during Z optimisation
    status = [p.requires_grad for p in model.netG.parameters()]
    zo = Z_optimizer(objective, [4 * h, 4 * w], model, 1.0, iters, data=data, initial_LR=lr_rate, batch_size=B)
    z_gpu = zo.optimize().cpu()
    # the same loop on the oracle (CPU autograd), in float64 (exact) and float32 (the reference's own arithmetic)
    z_start = torch.from_numpy(0.9 * z0).double()

    def oracle_loop(dt):
        P = {k: torch.as_tensor(v).to(dt) for k, v in O.strip_prefix(params).items()}
        eps = torch.finfo(torch.float32).eps
        pre = ArcTanH(torch.clamp(torch.from_numpy(0.9 * z0), -1 + eps, 1 - eps)).to(dt).requires_grad_(True)
        opt = torch.optim.Adam([pre], lr=lr_rate)
        lr_t, hr_t = torch.from_numpy(lr).to(dt), torch.from_numpy(hr).to(dt)
        for _ in range(iters):
            opt.zero_grad()
            out = O.sr_forward(torch.cat([torch.tanh(pre).reshape(B, 48, h, w), lr_t], 1), P, nb, True,
                               O.cem_design(4), pre_pad=True)
            loss = torch.nn.functional.l1_loss(out, hr_t) if objective == 'l1' else \
                -torch.std(out, dim=(1, 2, 3)).mean()
            loss.backward()
            opt.step()
        return torch.tanh(pre).detach().double()
    z64, z32 = oracle_loop(torch.float64), oracle_loop(torch.float32)
    # compared on the Z *update* (much stricter than on Z itself); see conftest.grad_parity for the L2 form
    ok, msg = grad_parity(z_gpu.double() - z_start, z64 - z_start, z32 - z_start, floor=1e-4)
    assert ok, msg
    assert [p.requires_grad for p in model.netG.parameters()] == status  # generator unfrozen again
    assert len(zo.loss_values) == iters


@pytest.mark.parametrize('cem,iters', [(1, 3), (0, 3), (1, -2)])
def test_z_optimizer_overflow_redo_equals_fp32_loop(gpu_device, cem, iters):
    """Z_optimizer.optimize reads the generator's x3 overflow flags once per iteration: with inputs whose activations
    leave the f16 range, every iteration is redone from its snapshot in exact fp32, so the loop ends bitwise where the
    same loop with an exact-fp32 generator does — with the CEM-wrapped generator and with a bare RRDBNet (define_G
    without CEM_arch: no generated_image_model to switch), and with max_iters < 0, where the convergence test
    (Z_optimization.py:567-571) reads the latest loss before the next iteration (the lagged flags are settled first)."""
    from esr_amd import engine
    nb, B, h, w = 1, 2, 12, 12
    lr, z0 = seeded_inputs(72, (B, 3, h, w), (B, 3, 4 * h, 4 * w), z_mode='pixel')
    outs = []
    before = engine.OVERFLOW_RERUNS
    for prec in ('x3', 'f32'):
        torch.manual_seed(0)
        model = SRRaGANModel(_opt(nb, cem), device=gpu_device)
        sd = model.netG.module.state_dict()
        params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], 71, w_scale=0.5)
        model.netG.module.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
        engine.set_precision(model.netG, prec)
        data = {'LR': torch.from_numpy(lr * 3e5).to(gpu_device), 'Z': torch.from_numpy(0.9 * z0).to(gpu_device)}
        model.feed_data(data, need_HR=False)
        model.test()
        model.netG.eval()
        zo = Z_optimizer('max_STD', [4 * h, 4 * w], model, 1.0, iters, data=data, initial_LR=0.05, batch_size=B)
        outs.append((zo.optimize().cpu(), list(zo.loss_values)))
    assert engine.OVERFLOW_RERUNS >= before + len(outs[1][1])
    assert all(np.isfinite(outs[0][1]))
    assert torch.equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]
