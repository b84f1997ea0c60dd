"""Configurations and per-step data of the training-loop fixtures (tests/golden/make_golden_train.py runs the
reference on them; tests/test_gpu_train_loop.py runs esr_amd on them).  Pure NumPy: no reference code.

TEST INFRASTRUCTURE ONLY."""
import numpy as np

from oracle.recipe import seeded_inputs


def train_opt(cfg):
    """The shipped train_esrgan_CEM.json at fixture size (nb, batch, patch), with the loop knobs of `cfg`."""
    patch = 4 * cfg['lr_size']
    return {
        'model': 'srragan', 'is_train': True, 'scale': 4, 'gpu_ids': None, 'range': [0, 1], 'test': None,
        'path': {'log': '/tmp/esr_golden_train_log', 'models': '/tmp/esr_golden_train_models',
                 'pretrain_model_G': None, 'pretrain_model_D': None},
        'datasets': {'train': {'patch_size': patch, 'batch_size': cfg['batch']}},
        'network_G': {'which_model_G': 'RRDB_net', 'CEM_arch': cfg.get('cem_arch', 1), 'latent_input': 'all_layers',
                      'latent_input_domain': 'HR_downscaled', 'latent_channels': 'SVDinNormedOut_structure_tensor',
                      'norm_type': None, 'mode': 'CNA', 'nf': 64, 'nb': cfg['nb'], 'in_nc': 3, 'out_nc': 3, 'gc': 32,
                      'group': 1, 'scale': 4},
        'network_D': {'which_model_D': 'discriminator_vgg_128', 'relativistic': cfg['relativistic'],
                      'decomposed_input': 0, 'pre_clipping': 0, 'add_quantization_noise': 0, 'norm_type': 'batch',
                      'act_type': 'leakyrelu', 'mode': 'CNA', 'n_layers': 6, 'nf': 64, 'in_nc': 3},
        'train': {'resume': 0, 'lr_G': cfg['lr'], 'weight_decay_G': 0, 'beta1_G': 0.9, 'lr_D': cfg.get('lr_D', cfg['lr']),
                  'lr_E': 1e-4, 'lr_latent': cfg['lr'], 'weight_decay_D': 0, 'beta1_D': 0.9,
                  'lr_scheme': 'MultiStepLR', 'lr_steps': [50000], 'lr_gamma': cfg.get('lr_gamma', 0.5),
                  'steps_4_loss_std': cfg.get('steps_4_loss_std'), 'std_4_lr_drop': cfg.get('std_4_lr_drop'),
                  'pixel_domain': cfg.get('pixel_domain', 'HR'),
                  'pixel_criterion': cfg.get('pixel_criterion', 'l1'), 'feature_domain': 'HR', 'feature_criterion': 'l1', 'gan_type': 'wgan-gp',
                  'optimalZ_loss_type': None, 'D_verification': cfg['D_verification'],
                  'min_D_prob_ratio_4_G': cfg['min_D_prob_ratio_4_G'], 'min_mean_D_correct': cfg['min_mean_D_correct'],
                  'D_update_ratio': cfg['D_update_ratio'], 'D_valid_Steps_4_G_update': cfg['D_valid_steps'],
                  'CEM_exp': 1, 'pixel_weight': cfg.get('pixel_weight', 0), 'feature_weight': 0, 'gan_weight': 1, 'latent_weight': 0,
                  'optimalZ_loss_weight': 0, 'range_weight': 5000, 'highpass_weight': 0, 'shift_invariant_weight': 0,
                  'D_init_iters': 0, 'E_init_iters': 40000, 'gp_weigth': 10,
                  'grad_accumulation_steps_G': cfg['acc'], 'grad_accumulation_steps_D': cfg['acc']},
    }


def step_data(cfg, k):
    """Micro-step k's batch: LR ~ U[0,1), HR ~ U[0,1) (patch size), per-image constant Z ~ U[-1,1) at HR size."""
    B, h = cfg['batch'], cfg['lr_size']
    lr, z = seeded_inputs(cfg['seed'] + 100 + k, (B, 3, h, h), (B, 3, 4 * h, 4 * h), z_mode='image')
    hr = np.random.default_rng(cfg['seed'] + 200 + k).random((B, 3, 4 * h, 4 * h)).astype(np.float32)
    return lr, hr, z


def random_points(cfg):
    rng = np.random.default_rng(cfg['seed'] + 300)
    while True:
        yield rng.random((cfg['batch'], 1, 1, 1)).astype(np.float32)


# the shipped loop at fixture size: non-relativistic WGAN-GP, fixed D_update_ratio, D_verification 'past', gradient
# accumulation 2; and the other branches: relativistic D, adaptive ratio (D_update_ratio 0), no verification
TRAIN_CFGS = {
    'past_ratio2_acc2': dict(nb=1, batch=2, lr_size=40, lr=1e-4, relativistic=0, D_update_ratio=2,
                             D_verification='past', D_valid_steps=1, min_D_prob_ratio_4_G=float(np.exp(0.02)),
                             min_mean_D_correct=-1.0, acc=2, steps=12, seed=500),
    'adaptive_rel': dict(nb=1, batch=2, lr_size=40, lr=1e-4, relativistic=1, D_update_ratio=0,
                         D_verification=None, D_valid_steps=2, min_D_prob_ratio_4_G=1.0,
                         min_mean_D_correct=0.0, acc=1, steps=8, seed=600),
    # the G pixel loss (SRRaGAN_model.py:108-120, 477-483) at the JSON's commented default weight 1e-2
    # (train_esrgan_CEM.json:100): L1 in the HR domain with the CEM generator; L2 in the LR domain ('pixel_domain':
    # 'LR', bilinear Convert_2_LR) with the plain latent generator (the reference asserts HR with CEM_arch, :61)
    'pixel_l1_hr': dict(nb=1, batch=2, lr_size=40, lr=1e-4, relativistic=1, D_update_ratio=1,
                        D_verification=None, D_valid_steps=1, min_D_prob_ratio_4_G=1.0, min_mean_D_correct=0.0,
                        acc=1, steps=6, seed=650, pixel_weight=1e-2, pixel_criterion='l1', pixel_domain='HR'),
    'pixel_l2_lr': dict(nb=1, batch=2, lr_size=40, lr=1e-4, relativistic=0, D_update_ratio=1,
                        D_verification=None, D_valid_steps=1, min_D_prob_ratio_4_G=1.0, min_mean_D_correct=0.0,
                        acc=1, steps=6, seed=660, pixel_weight=1e-2, pixel_criterion='l2', pixel_domain='LR',
                        cem_arch=0),
}
CKPT_CFG = dict(nb=1, batch=2, lr_size=40, lr=1e-4, relativistic=0, D_update_ratio=1, D_verification=None,
                D_valid_steps=1, min_D_prob_ratio_4_G=1.0, min_mean_D_correct=0.0, acc=1, steps=0, seed=700)



# perform_validation (SRRaGAN_model.py:586-635) as train.py:163-173 calls it: the CKPT_CFG model (nb=1 latent CEM, its
# own seeded weights) on four batch-1 validation images of different sizes, for latent values 0, -1 and 1
VAL_CFG = dict(CKPT_CFG, seed=720)
VAL_SIZES = [(20, 24), (24, 20), (22, 22), (20, 20)]
VAL_ZS = (0, -1, 1)


def val_items():
    """The validation set: CHW float32 LR / HR pairs (HR 4× the LR) and their paths."""
    rng = np.random.default_rng(5)
    items = []
    for i, (h, w) in enumerate(VAL_SIZES):
        items.append({'LR': rng.random((3, h, w), dtype=np.float32),
                      'HR': rng.random((3, 4 * h, 4 * w), dtype=np.float32), 'HR_path': 'val/img%d.png' % i})
    return items


# update_learning_rate (SRRaGAN_model.py:637-683) as train.py:187-189 drives it: one call per gradient step, D losses
# whose spread jumps at step 10 (std over a 4-step window: ~0.01 before, ~0.5 after, threshold 0.05), checkpoints at
# gradient steps 2 and 5 (saved only before the first LR drop), lr_gamma 0.05 so that the fourth drop takes the LR
# below 1e-8 (the `lr_too_low` return)
LR_CFG = dict(CKPT_CFG, seed=710, steps_4_loss_std=4, std_4_lr_drop=0.05, lr_gamma=0.05, ckpt_steps=[2, 5],
              n_calls=60, probe='generated_image_model.model.0.bias')


def lr_log_rows(cfg, g):
    """(l_d_real, l_d_fake, D_logits_diff) logged at gradient step g."""
    amp = 0.01 if g < 10 else 0.5
    return 1.0 + amp * np.random.default_rng(cfg['seed'] * 1000 + g).standard_normal(3)


def drive_lr_schedule(model, cfg):
    """train.py's per-step sequence around update_learning_rate, with the D logs and a parameter change ("training")
    made up: returns one record per call: [cur_step, returned lr_too_low, lr_G, lr_D, model.step after the call,
    len(D_loss_STD), last D_loss_STD (nan if none), len(LR_decrease), summed change of the probe parameter] and the
    LR_decrease entries as [step, lr_G, lr_D].  Works on the reference's model and on esr_amd's (same methods)."""
    import torch
    acc = cfg['acc']
    probe = dict(model.netG.named_parameters())[cfg['probe']]
    start = probe.detach().double().clone()
    records = []
    for _ in range(cfg['n_calls']):
        g = model.step // acc
        model.gradient_step_num = g  # optimize_parameters' first statement (SRRaGAN_model.py:308)
        for k, v in zip(('l_d_real', 'l_d_fake', 'D_logits_diff'), lr_log_rows(cfg, g)):
            model.log_dict[k].append((g, float(v)))
        with torch.no_grad():
            probe.add_(1e-3 * (g + 1))
        model.step += acc
        if g in cfg['ckpt_steps'] and not model.log_dict['LR_decrease']:
            model.save(g)
            model.save_log()
        ret = model.update_learning_rate(g)
        std = model.log_dict['D_loss_STD']
        records.append([g, float(bool(ret)), model.optimizer_G.param_groups[0]['lr'],
                        model.optimizer_D.param_groups[0]['lr'], model.step, len(std),
                        float(std[-1][1]) if std else float('nan'), len(model.log_dict['LR_decrease']),
                        float((probe.detach().double() - start).sum())])
        if ret:
            break
    dec = [[e[0], e[1]['lr_G'], e[1]['lr_D']] for e in model.log_dict['LR_decrease']]
    return np.array(records, dtype=np.float64), np.array(dec, dtype=np.float64).reshape(-1, 3)


# config 3 at its production grid: B=16 × 96² LR crops, RRDB-23, latent, CEM train mode (the D sees
# the unpadded 304² HR), WGAN-GP non-relativistic as shipped; 2 micro-steps: step 0 = D step only (generator_step needs
# gradient_step_num > D_init_iters), step 1 = D step + G step.  define_G's training-time init scale (kaiming × 0.1)
# for the generator.  The fixture holds digests of the step-1 gradients of every G and D parameter (K seeded random
# projections + the norm), the logs and the D BatchNorm buffers, from the reference in float32 and float64.
C3_GRID_CFG = dict(nb=23, batch=16, lr_size=96, lr=1e-4, relativistic=0, D_update_ratio=1, D_verification=None,
                   D_valid_steps=1, min_D_prob_ratio_4_G=1.0, min_mean_D_correct=0.0, acc=1, steps=2, seed=800,
                   w_scale_G=0.1, proj=8)


def grad_projections(grad, seed, index, k):
    """k projections of a gradient (any shape, float64 numpy) on seeded standard-normal directions."""
    g = np.asarray(grad, dtype=np.float64).ravel()
    P = np.random.default_rng([seed, index]).standard_normal((k, g.size))
    return P @ g
