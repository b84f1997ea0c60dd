"""SRRaGANModel.perform_validation (SRRaGAN_model.py:586-635) as codes/train.py:163-173 calls it: batch-1 test() per
validation image for each latent value, the PSNR of the 0-255 images (utils/util.py:80-104, 168-175) added into
print_rlt['psnr'], and the collage PNGs."""
import os
import sys
import zlib

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'golden'))
from train_recipe import CKPT_CFG, train_opt  # noqa: E402

pytestmark = pytest.mark.gpu


class _Loader:
    """What train.py's val_loader provides: iteration over batch-1 dicts and .dataset (CHW images)."""
    def __init__(self, items):
        self.dataset = items

    def __iter__(self):
        for it in self.dataset:
            yield {'LR': it['LR'][None], 'HR': it['HR'][None], 'HR_path': [it['HR_path']]}


def _read_png(path):
    data = open(path, 'rb').read()
    assert data[:8] == b'\x89PNG\r\n\x1a\n'
    pos, idat, hdr = 8, b'', None
    while pos < len(data):
        n = int.from_bytes(data[pos:pos + 4], 'big')
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        if tag == b'IHDR':
            hdr = body
        elif tag == b'IDAT':
            idat += body
        pos += 12 + n
    w, h = int.from_bytes(hdr[:4], 'big'), int.from_bytes(hdr[4:8], 'big')
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 3)


def test_perform_validation(gpu_device, tmp_path):
    from esr_amd.SRRaGAN_model import SRRaGANModel
    opt = train_opt(CKPT_CFG)
    opt['path'] = dict(opt['path'], log=str(tmp_path), models=str(tmp_path), val_images=str(tmp_path))
    torch.manual_seed(0)
    model = SRRaGANModel(opt, device=gpu_device)
    rng = np.random.default_rng(5)
    items = []
    for i, (h, w) in enumerate([(20, 24), (24, 20), (22, 22), (20, 20)]):
        items.append({'LR': torch.from_numpy(rng.random((3, h, w), dtype=np.float32)),
                      'HR': torch.from_numpy(rng.random((3, 4 * h, 4 * w), dtype=np.float32)),
                      'HR_path': 'val/img%d.png' % i})
    rlt = {'psnr': 0}
    expected, outs = [], {}
    for z in (0, -1, 1):
        before = rlt['psnr']
        srs = model.perform_validation(_Loader(items), z, rlt, save_GT_HR=True, save_images=True)
        assert len(srs) == 4
        ps = []
        for it, sr in zip(items, srs):
            # the reference's image conversion and PSNR, restated here on the model's own test() output
            model.feed_data({'LR': it['LR'][None], 'HR': it['HR'][None], 'Z': z})
            model.test()
            mine = model.fake_H[0].clamp(0, 1).cpu().numpy().transpose(1, 2, 0)[..., ::-1] * 255
            assert np.array_equal(sr, mine.astype(np.float32))
            gt = it['HR'].clamp(0, 1).numpy().transpose(1, 2, 0)[..., ::-1] * 255
            ps.append(20 * np.log10(255 / np.sqrt(np.mean((sr.astype(np.float64) - gt.astype(np.float64)) ** 2))))
        assert abs((rlt['psnr'] - before) - np.mean(ps)) < 1e-9
        expected.append(np.mean(ps))
        outs[z] = srs
        png = os.path.join(str(tmp_path), '0_Z%sPSNR%.3f.png' % (z, np.mean(ps)))
        img = _read_png(png)
        # 2 collage rows (4 images), each crop the smallest HR side - 2 = 78 pixels, stacked as the reference does
        assert img.shape == (2 * 78, 2 * 78, 3)
        m = ((np.array(srs[0].shape[:2]) - 78) / 2).astype(np.int32)
        crop = np.clip(srs[0][m[0]:-m[0], m[1]:-m[1]], 0, 255).astype(np.uint8)
        assert np.array_equal(img[:78, :78], crop[..., ::-1])  # RGB in the file, BGR in memory (cv2.imwrite)
    assert os.path.isfile(os.path.join(str(tmp_path), 'GT_HR.png'))
    assert not np.array_equal(outs[-1][0], outs[1][0])  # the latent value reaches the generator
    assert model.netG.training  # test() leaves the model in train mode


@pytest.mark.parametrize('precision', ['x3', 'f32'])
def test_perform_validation_vs_reference(gpu_device, precision):
    """perform_validation against the reference's own method (tests/golden/validation.npz, made by
    make_golden_train.py val: the reference's SRRaGANModel with the VAL_CFG seeded weights on the same four images, for
    Z = 0, -1, 1): the returned SR images (HWC BGR float32 0-255) within 1e-4 normwise of the reference's float32 CPU
    run, and print_rlt['psnr'] after each call within 1e-4 dB per image."""
    from esr_amd import engine
    from esr_amd.SRRaGAN_model import SRRaGANModel
    from oracle.recipe import seeded_params
    from train_recipe import VAL_CFG, VAL_ZS, val_items
    d = np.load(os.path.join(HERE, 'golden', 'validation.npz'))
    torch.manual_seed(0)
    model = SRRaGANModel(train_opt(VAL_CFG), device=gpu_device)
    gsd = model.netG.state_dict()
    gp = seeded_params([(k, tuple(v.shape)) for k, v in gsd.items()], VAL_CFG['seed'],
                       w_scale=VAL_CFG.get('w_scale_G', 1.0))
    model.netG.load_state_dict({k: torch.from_numpy(v) for k, v in gp.items()}, strict=False)
    engine.set_precision(model.netG, precision)
    items = [{'LR': torch.from_numpy(it['LR']), 'HR': torch.from_numpy(it['HR']), 'HR_path': it['HR_path']}
             for it in val_items()]
    rlt = {'psnr': 0}
    for z in VAL_ZS:
        srs = model.perform_validation(_Loader(items), z, rlt, save_GT_HR=False, save_images=False)
        for i, sr in enumerate(srs):
            ref = d['sr:%g:%d' % (z, i)]
            assert sr.shape == ref.shape and sr.dtype == np.float32
            err = float(np.abs(sr.astype(np.float64) - ref).max() / np.abs(ref).max())
            assert err < 1e-4, (z, i, err)  # the generator fixtures' bar (observed ~1e-5 x3, ~1e-6 f32)
        assert abs(rlt['psnr'] - float(d['psnr_after:%g' % z])) < 1e-4 * len(items), (z, rlt['psnr'])
