"""Diagnostic (GPU): how many times does each discriminator parameter's post-accumulate-grad hook fire in one D step
(the C4 test's half-0 model, one process)?  A DDP bucket launched on a parameter's first accumulation misses the
later ones."""
import collections
import sys

import numpy as np
import torch

sys.path.insert(0, 'tests')
sys.path.insert(0, 'tests/golden')
sys.path.insert(0, '.')
sys.path.insert(0, 'explorable-super-resolution_old_amd')


def main():
    from train_recipe import step_data, train_opt
    from oracle.recipe import seeded_params
    from esr_amd.SRRaGAN_model import SRRaGANModel
    import test_gpu_ddp_c4 as T
    cfg = T._cfg()
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    model = SRRaGANModel(train_opt(cfg), accumulation_steps_per_batch=1, device=dev)
    gsd, dsd = model.netG.state_dict(), model.netD.state_dict()
    gp = seeded_params([(k, tuple(v.shape)) for k, v in gsd.items()], cfg['seed'], w_scale=cfg['w_scale_G'])
    dp = seeded_params([(k, tuple(v.shape)) for k, v in dsd.items() if 'running' not in k and 'num_batches' not in k],
                       cfg['seed'] + 1, w_scale=1.0)
    model.netG.load_state_dict({k: torch.from_numpy(v) for k, v in gp.items()}, strict=False)
    model.netD.load_state_dict({k: torch.from_numpy(v) for k, v in dp.items()}, strict=False)
    rng = np.random.default_rng(cfg['seed'] + 300)
    model._interp_points = lambda n: torch.from_numpy(rng.random((n, 1, 1, 1)).astype(np.float32)).to(dev)
    calls = collections.Counter()
    names = {id(p): k for k, p in model.netD.named_parameters()}
    for p in model.netD.parameters():
        p.register_post_accumulate_grad_hook(lambda t: calls.update([names[id(t)]]))
    lr, hr, z = step_data(dict(cfg, batch=32), 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a[:16])).to(dev)  # noqa: E731
    model.feed_data({'LR': t(lr), 'HR': t(hr), 'Z': t(z)})
    model.optimize_parameters()
    multi = {k: v for k, v in calls.items() if v != 1}
    print('D parameters: %d, hooks fired: %d, parameters whose hook fired != 1 time: %s' % (
        len(names), sum(calls.values()), multi or 'none'), flush=True)


if __name__ == '__main__':
    main()
