"""Checkpoint / log compatibility of SRRaGANModel (base_model.py:86-144; SRRaGAN_model.py:695-719, 766-813), CPU only:
the positional key-remapping loader, latent-channel zero-prepend, CEM-filter skipping, `{step}_G.pth` selection,
save/load round trips with optimizer state, logs.npz / lr.npz."""
import collections
import os

import numpy as np
import pytest
import torch

import esr_amd
from esr_amd import CEMnet as C
from esr_amd import SRRaGAN_model as M


def _latent_cem_net():
    net = esr_amd.RRDBNet(3, 3, 64, 2, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    cem = C.CEMnet(C.Get_CEM_Config(4))
    return cem, cem.WrapArchitecture_PyTorch(net)


def _bare_model(cem, latent, is_train=False, path=None):
    """An SRRaGANModel shell (the constructor needs a GPU): just the attributes the checkpoint methods read."""
    m = M.SRRaGANModel.__new__(M.SRRaGANModel)
    m.opt = {'scale': 4, 'is_train': is_train, 'path': path or {}, 'train': {'resume': 0}}
    m.is_train = is_train
    m.CEM_arch = True
    m.CEM_net = cem
    m.latent_input = 'all_layers' if latent else None
    m.num_latent_channels = 3 if latent else 0
    m.save_dir = (path or {}).get('models')
    m.log_path = (path or {}).get('log')
    m.log_dict = collections.OrderedDict((k, []) for k in ('l_d_real', 'D_logits_diff'))
    m.step = 0
    return m


def test_plain_checkpoint_into_latent_cem_model_zero_prepends_latent_weights():
    """A pretrained plain ESRGAN state dict (no CEM prefix, no latent inputs) loads into the latent CEM model: keys get
    the generated_image_model. prefix, every latent-widened weight gets zero columns in front, the CEM filters keep
    the current design, and the widened channels are recorded for gradient amplification."""
    torch.manual_seed(0)
    plain = esr_amd.RRDBNet(3, 3, 64, 2, num_latent_channels=0).state_dict()
    cem, model = _latent_cem_net()
    m = _bare_model(cem, latent=True)
    m.channels_idx_4_grad_amplification = [[] for _ in model.parameters()]
    cur = model.state_dict()
    adj = C.Adjust_State_Dict_Keys(plain, cur)
    out = m.process_loaded_state_dict(adj, cur)
    assert not any('Filter' in k for k in out)
    widened = 0
    for k, v in out.items():
        assert v.shape == cur[k].shape, k
        src = plain[k[len('generated_image_model.'):]]
        if src.shape != v.shape:
            extra = v.shape[1] - src.shape[1]
            assert extra == 3, (k, extra)  # Z_LR (bilinear-downscaled) or Z_HR: 3 channels each
            assert torch.equal(v[:, :extra], torch.zeros_like(v[:, :extra])) and torch.equal(v[:, extra:], src)
            widened += 1
        else:
            assert torch.equal(v, src)
    assert widened == 2 * 3 * 5 + 1 + 1 + 2  # every RDB conv, LR_conv, conv_first, HR_conv0/1
    amplified = [i for i, c in enumerate(m.channels_idx_4_grad_amplification) if c]
    assert len(amplified) == widened
    missing, unexpected = model.load_state_dict(out, strict=False)
    assert not unexpected and all('Filter' in k for k in missing)


def test_positional_remap_of_renamed_keys_and_shape_guard():
    cem, model = _latent_cem_net()
    m = _bare_model(cem, latent=False)
    cur = model.state_dict()
    renamed = collections.OrderedDict(('old_%d' % i, v.clone()) for i, v in enumerate(cur.values()))
    with pytest.warns(UserWarning, match='Modified'):
        out = m.process_loaded_state_dict(renamed, cur)
    # the reference skips CEM filters by the LOADED key name (base_model.py:138), so renamed filters map positionally
    assert list(out) == list(cur)
    bad = collections.OrderedDict(renamed)
    first = next(iter(bad))
    bad[first] = torch.zeros(7, *cur[next(iter(cur))].shape[1:])
    with pytest.raises(AssertionError, match='Unmatching'):
        m.process_loaded_state_dict(bad, cur)
    short = collections.OrderedDict(list(renamed.items())[:-1])
    with pytest.raises(AssertionError, match='same number'):
        m.process_loaded_state_dict(short, cur)


def test_save_load_roundtrip_selects_step_and_restores_optimizer(tmp_path):
    models, logs = tmp_path / 'models', tmp_path / 'log'
    models.mkdir()
    logs.mkdir()
    cem, model = _latent_cem_net()
    m = _bare_model(cem, latent=True, path={'models': str(models), 'log': str(logs)})
    m.netG = model
    gparams = [p for n, p in model.named_parameters() if 'Filter' not in n]
    opt = torch.optim.Adam(gparams, lr=1e-4)
    saved = {}
    for step in (5, 12, 100):
        with torch.no_grad():
            for p in gparams:
                p.add_(0.01 * step)
        model.zero_grad()
        sum(p.sum() for p in gparams).backward()
        opt.step()
        saved[step] = {k: v.clone() for k, v in model.state_dict().items()}
        path = m.save_network(str(models), model, 'G', step, opt)
        assert os.path.basename(path) == '%d_G.pth' % step
    blob = torch.load(str(models / '12_G.pth'), weights_only=True)
    assert set(blob) == {'model_state_dict', 'optimizer_state_dict'}
    # test mode: load(max_step=50) picks 12_G.pth, never 100
    with torch.no_grad():
        for p in gparams:
            p.zero_()
    m.load(max_step=50)
    assert m.gradient_step_num == 12
    for k, v in model.state_dict().items():  # filters included: never loaded, never changed
        assert torch.equal(v, saved[12][k]), k
    # resume (train) mode restores the optimizer state and the step counter
    m.is_train, m.opt['is_train'] = True, True
    m.max_accumulation_steps, m.D_exists = 1, False
    m.optimizer_G = torch.optim.Adam(gparams, lr=1e-4)
    m.load(resume_train=True)
    assert m.step == 101
    assert int(m.optimizer_G.state_dict()['state'][0]['step']) == 3
    for k, v in model.state_dict().items():
        assert torch.equal(v, saved[100][k]), k


def test_logs_and_lr_npz_roundtrip(tmp_path):
    cem, _ = _latent_cem_net()
    m = _bare_model(cem, latent=False, path={'log': str(tmp_path)})
    m.log_dict['l_d_real'] = [(1, 0.5), (2, 0.25), (9, -1.0)]
    m.log_dict['D_logits_diff'] = [(1, 2.0)]
    m.save_log()
    with np.load(tmp_path / 'logs.npz') as f:
        assert f['l_d_real'].shape == (3, 2)
    m.log_dict = collections.OrderedDict((k, []) for k in m.log_dict)
    m.load_log(max_step=2)
    assert m.log_dict['l_d_real'] == [(1.0, 0.5), (2.0, 0.25)] and m.log_dict['D_logits_diff'] == [(1.0, 2.0)]
    p = torch.nn.Parameter(torch.zeros(1))
    m.optimizer_G = torch.optim.Adam([p], lr=3e-5)
    m.optimizer_D = torch.optim.Adam([p], lr=7e-5)
    m.save_lr(40)
    with np.load(tmp_path / 'lr.npz') as f:
        assert float(f['lr_G']) == 3e-5 and float(f['lr_D']) == 7e-5 and int(f['step_num']) == 40


# ---- pinned by the reference itself (tests/golden/make_golden_train.py: the reference's base_model.py ran here) ----
GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def _sha(t):
    import hashlib
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()


def _latent_cem_nb1(seed):
    """The latent CEM generator (nb=1) holding the seeded parameters the reference model held (make_golden_train
    build_reference: seeded_params over its state_dict keys, w_scale 1)."""
    import json
    from oracle.recipe import seeded_params
    net = esr_amd.RRDBNet(3, 3, 64, 1, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    cem = C.CEMnet(C.Get_CEM_Config(4))
    model = cem.WrapArchitecture_PyTorch(net)
    sd = model.state_dict()
    params = seeded_params([(k, tuple(v.shape)) for k, v in sd.items()], seed, w_scale=1.0)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    return cem, model, params


def test_load_network_matches_reference_remap(tmp_path):
    """base_model.load_network + process_loaded_state_dict (base_model.py:100-144) of a plain pretrained RRDBNet
    state dict into the latent CEM generator, as the reference computed it: same key order, bitwise equal tensors
    (the prepended latent weights are the reference's signed zeros), same gradient-amplified channel lists."""
    import json
    from oracle.recipe import seeded_params
    d = np.load(os.path.join(GOLDEN, 'ckpt_remap.npz'))
    cfg = json.loads(str(d['cfg']))
    cem, model, _ = _latent_cem_nb1(cfg['seed'])
    plain = esr_amd.RRDBNet(3, 3, 64, 1, num_latent_channels=0).state_dict()
    psd = seeded_params([(k, tuple(v.shape)) for k, v in plain.items()], int(d['plain_seed']), w_scale=1.0)
    path = str(tmp_path / 'plain_G.pth')
    torch.save({k: torch.from_numpy(v) for k, v in psd.items()}, path)
    m = _bare_model(cem, latent=True)
    m.channels_idx_4_grad_amplification = [[] for _ in model.parameters()]
    m.load_network(path, model)
    sd = model.state_dict()
    assert list(sd) == json.loads(str(d['keys']))
    ref_sha = json.loads(str(d['sha']))
    bad = [k for k, v in sd.items() if _sha(v) != ref_sha[k]]
    assert not bad, bad
    assert m.channels_idx_4_grad_amplification == json.loads(str(d['amplified']))


def test_reference_saved_checkpoint_loads(tmp_path):
    """A {step}_G.pth written by the reference's save_network (base_model.py:86-97) after one Adam step on three
    parameters: load_network restores every parameter and the Adam state bit for bit; a checkpoint the port writes has
    the same structure (keys, dtypes, shapes, optimizer param_groups keys)."""
    import json
    d = np.load(os.path.join(GOLDEN, 'ckpt_save.npz'))
    cfg = json.loads(str(d['cfg']))
    names = json.loads(str(d['names']))
    cem, model, params = _latent_cem_nb1(cfg['seed'] + 1)  # different weights: the load must overwrite them all
    gparams = [p for n, p in model.named_parameters() if 'Filter' not in n]
    opt = torch.optim.Adam(gparams, lr=cfg['lr'], betas=(0.9, 0.999))
    m = _bare_model(cem, latent=True)
    m.channels_idx_4_grad_amplification = [[] for _ in model.parameters()]
    ref_file = os.path.join(GOLDEN, 'ckpt', '7_G.pth')
    m.load_network(ref_file, model, optimizer=opt)
    _, _, expect = _latent_cem_nb1(cfg['seed'])
    for k, v in model.named_parameters():
        if 'Filter' in k:
            continue
        ref = d['after:' + k] if k in names else expect[k]
        assert np.array_equal(v.detach().numpy(), ref), k
    st = opt.state_dict()['state']
    assert sorted(st) == sorted(int(f.split(':')[1]) for f in d.files if f.startswith('exp_avg:'))
    for i, s in st.items():
        assert np.array_equal(s['exp_avg'].numpy(), d['exp_avg:%d' % i])
        assert np.array_equal(s['exp_avg_sq'].numpy(), d['exp_avg_sq:%d' % i])
    mine = torch.load(m.save_network(str(tmp_path), model, 'G', 7, opt), weights_only=True)
    ref = torch.load(ref_file, weights_only=True)
    assert set(mine) == set(ref) == {'model_state_dict', 'optimizer_state_dict'}
    assert list(mine['model_state_dict']) == list(ref['model_state_dict'])
    for k, v in ref['model_state_dict'].items():
        w = mine['model_state_dict'][k]
        assert w.dtype == v.dtype and w.shape == v.shape and w.device == v.device, k
        assert torch.equal(w, v), k
    assert set(mine['optimizer_state_dict']) == set(ref['optimizer_state_dict'])
    assert set(mine['optimizer_state_dict']['param_groups'][0]) >= {'lr', 'betas', 'eps', 'weight_decay', 'params'}
    assert mine['optimizer_state_dict']['param_groups'][0]['params'] == ref['optimizer_state_dict']['param_groups'][0]['params']
