"""SRRaGANModel.update_learning_rate / get_current_log (SRRaGAN_model.py:637-693) against the REFERENCE's own method,
driven the way codes/train.py:187-189 drives it (tests/golden/train_recipe.drive_lr_schedule; fixture made by
tests/golden/make_golden_train.py lr).  CPU only: the model is built on the CPU and no generator forward runs."""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, 'golden'))
from train_recipe import drive_lr_schedule, train_opt  # noqa: E402

from esr_amd.SRRaGAN_model import SRRaGANModel  # noqa: E402


def _model(cfg, tmp_path):
    opt = train_opt(cfg)
    opt['path'] = dict(opt['path'], log=str(tmp_path / 'log'), models=str(tmp_path / 'models'))
    os.makedirs(opt['path']['log'])
    os.makedirs(opt['path']['models'])
    torch.manual_seed(0)
    return SRRaGANModel(opt, accumulation_steps_per_batch=cfg['acc'], device=torch.device('cpu'))


def test_update_learning_rate_matches_reference(tmp_path):
    d = np.load(os.path.join(HERE, 'golden', 'lr_schedule.npz'))
    cfg = json.loads(str(d['cfg']))
    model = _model(cfg, tmp_path)
    records, dec = drive_lr_schedule(model, cfg)
    ref = d['records']
    assert records.shape == ref.shape, (records.shape, ref.shape)
    # cur_step, lr_too_low, model.step (rollbacks), D_loss_STD count, LR_decrease count: exact
    for col in (0, 1, 4, 5, 7):
        assert np.array_equal(records[:, col], ref[:, col]), (col, records[:, col], ref[:, col])
    np.testing.assert_allclose(records[:, 2:4], ref[:, 2:4], rtol=1e-12)  # learning rates
    np.testing.assert_allclose(records[:, 6], ref[:, 6], rtol=1e-12, equal_nan=True)  # D_loss_STD
    # probe parameter change (float32 adds on each side's own initial values): back to the checkpoint on a rollback
    np.testing.assert_allclose(records[:, 8], ref[:, 8], rtol=1e-5, atol=1e-6)
    assert np.array_equal(dec, d['lr_decrease'])
    with np.load(str(tmp_path / 'log' / 'lr.npz')) as f:
        mine = np.array([f['step_num'], f['lr_G'], f['lr_D']], dtype=np.float64)
    np.testing.assert_allclose(mine, d['lr_file'], rtol=1e-12)
    # the schedule covers every branch: too few entries, std below the threshold, rollbacks, lr_too_low
    assert ref[:, 1].sum() == 1 and len(set(ref[:, 4] - ref[:, 0])) > 1 and np.isnan(ref[0, 6])


def test_lr_untouched_without_drops_and_schedulers_not_stepped(tmp_path):
    """No drop below std_4_lr_drop: the learning rates stay, whatever MultiStepLR's milestones say."""
    d = np.load(os.path.join(HERE, 'golden', 'lr_schedule.npz'))
    cfg = dict(json.loads(str(d['cfg'])), std_4_lr_drop=None, n_calls=25)
    cfg['lr_steps'] = [1]
    model = _model(cfg, tmp_path)
    records, dec = drive_lr_schedule(model, cfg)
    assert (records[:, 2] == cfg['lr']).all() and (records[:, 1] == 0).all() and len(dec) == 0
    assert records[-1, 5] > 0  # D_loss_STD is still logged


def test_get_current_log_latest_values(tmp_path):
    d = np.load(os.path.join(HERE, 'golden', 'lr_schedule.npz'))
    cfg = json.loads(str(d['cfg']))
    model = _model(cfg, tmp_path)
    assert model.get_current_log() == {}
    model.log_dict['l_d_real'].extend([(0, 1.5), (1, 2.5)])
    model.log_dict['D_loss_STD'].append([1, 0.25])
    model.log_dict['LR_decrease'].append([3, {'lr_G': 1e-5, 'lr_D': 1e-5}])
    out = model.get_current_log()
    # the reference's key order (SRRaGAN_model.py:72-75) and the value of the latest (step, value) pair
    assert list(out) == ['l_d_real', 'D_loss_STD', 'LR_decrease']
    assert out['l_d_real'] == 2.5 and out['D_loss_STD'] == 0.25 and out['LR_decrease'] == {'lr_G': 1e-5, 'lr_D': 1e-5}
    assert model.get_current_learning_rate() == cfg['lr']
    assert model.generator_changed  # :243
