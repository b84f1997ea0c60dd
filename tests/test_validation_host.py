"""perform_validation's host side against the reference's own method (tests/golden/validation.npz, made by
tests/golden/make_golden_train.py val): the SR images the reference returned are the CPU oracle's CEM_PyTorch(RRDBNet)
forward on the same seeded weights and images, converted by SRRaGAN_model._tensor2img (utils/util.py:80-104), and the
PSNR sums print_rlt['psnr'] are SRRaGAN_model._psnr (utils/util.py:168-175) of those images.  CPU only: this pins the
oracle on the validation shapes and the port's image conversion / PSNR; tests/test_gpu_validation.py runs the method
itself on the HIP path against the same fixture."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'golden'))
from train_recipe import VAL_CFG, VAL_ZS, val_items  # noqa: E402

from esr_amd.SRRaGAN_model import _psnr, _tensor2img  # noqa: E402
from oracle import esr_oracle as O  # noqa: E402
from oracle.recipe import seeded_params  # noqa: E402


def _keys():
    """The generator's state_dict keys and shapes (the port keeps the reference's order), built on the CPU."""
    import esr_amd
    from esr_amd import CEMnet as C
    net = esr_amd.RRDBNet(3, 3, 64, VAL_CFG['nb'], latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net)
    return [(k, tuple(v.shape)) for k, v in model.state_dict().items()]


def test_validation_images_and_psnr_vs_reference():
    d = np.load(os.path.join(HERE, 'golden', 'validation.npz'))
    params = seeded_params(_keys(), VAL_CFG['seed'], w_scale=VAL_CFG.get('w_scale_G', 1.0))
    P = O.strip_prefix({k: torch.from_numpy(v) for k, v in params.items() if 'Filter' not in k})
    design = O.cem_design(4)
    total = 0.0
    for z in VAL_ZS:
        ps = []
        for i, it in enumerate(val_items()):
            lr = torch.from_numpy(it['LR'])[None]
            h, w = lr.shape[2:]
            zhr = torch.full((1, 3, 4 * h, 4 * w), float(z))
            x = torch.cat([zhr.reshape(1, 48, h, w), lr], 1)  # the raw HR latent view (SRRaGAN_model.py:252)
            with torch.no_grad():
                out = O.sr_forward(x, P, VAL_CFG['nb'], True, design, pre_pad=True)
            sr = 255 * _tensor2img(out[0])
            ref = d['sr:%g:%d' % (z, i)]
            assert sr.shape == ref.shape
            assert float(np.abs(sr.astype(np.float64) - ref).max() / np.abs(ref).max()) < 1e-5
            ps.append(_psnr(ref, 255 * _tensor2img(torch.from_numpy(it['HR']))))
        total += float(np.mean(ps))
        assert abs(total - float(d['psnr_after:%g' % z])) < 1e-9, (z, total)
