"""GPU check of checkpoint compatibility: a plain (no-latent, no-CEM) generator checkpoint written in the reference's
`{step}_G.pth` format, loaded through SRRaGANModel.load_network into the latent CEM model (key prefixing + latent
zero-prepend, base_model.py:100-144), makes that model ignore Z: its output for any Z equals the plain generator's
output under the same CEM.  Both run on the HIP path; tolerance 1e-5 normwise (different K-groupings of the same sums).
"""
import collections

import pytest
import torch

from conftest import normwise_rel

import esr_amd
from esr_amd import CEMnet as C
from esr_amd import SRRaGAN_model as M
from esr_amd import engine
from oracle.recipe import seeded_inputs, seeded_params

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('precision', ['f32', 'x3'])
def test_plain_checkpoint_drives_latent_cem_model(gpu_device, tmp_path, precision):
    plain = esr_amd.RRDBNet(3, 3, 64, 2, num_latent_channels=0)
    params = seeded_params([(k, tuple(v.shape)) for k, v in plain.state_dict().items()], 41, w_scale=0.5)
    plain.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()})
    opt = torch.optim.Adam(plain.parameters(), lr=1e-4)

    cem = C.CEMnet(C.Get_CEM_Config(4))
    latent_model = cem.WrapArchitecture_PyTorch(
        esr_amd.RRDBNet(3, 3, 64, 2, latent_input='all_layers_HR_downscaled', num_latent_channels=3))
    m = M.SRRaGANModel.__new__(M.SRRaGANModel)
    m.opt, m.is_train, m.CEM_arch, m.CEM_net = {'scale': 4}, False, True, cem
    m.latent_input, m.num_latent_channels = 'all_layers', 3
    path = m.save_network(str(tmp_path), plain, 'G', 7, opt)
    m.load_network(path, latent_model)

    plain_cem = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(plain)
    for net in (latent_model, plain_cem):
        net.to(gpu_device).eval()
        engine.set_precision(net, precision)
    lr, z = seeded_inputs(42, (2, 3, 12, 16), (2, 3, 48, 64))
    x = torch.from_numpy(lr).to(gpu_device)
    xz = torch.cat([torch.from_numpy(z).reshape(2, 48, 12, 16).to(gpu_device), x], 1)
    with torch.no_grad():
        ref = plain_cem(x)
        out = latent_model(xz)
        out0 = latent_model(torch.cat([torch.zeros_like(xz[:, :48]), x], 1))
    assert normwise_rel(out.cpu(), ref.cpu()) < 1e-5
    assert normwise_rel(out0.cpu(), ref.cpu()) < 1e-5
    sd = collections.OrderedDict(latent_model.state_dict())
    w = sd['generated_image_model.model.0.weight']
    assert w.shape[1] == 6 and float(w[:, :3].abs().max()) == 0.0  # conv_first sees the 3 bilinear-downscaled Z channels
