"""Bitwise determinism of the discriminator step pieces (a round-3 loop probe found ~1e-8 run-to-run differences
in D conv / BN weight gradients): runs each variant 3 times on the same inputs and lists the parameters whose
gradients differ.  Usage (GPU): python tools/d_determinism.py [H]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

from esr_amd import dconv, loss as L  # noqa: E402
from esr_amd.discriminator import Discriminator_VGG_128_  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 120
dev = torch.device('cuda:0')
dconv.set_precision('f32')
torch.manual_seed(0)
D = Discriminator_VGG_128_(3, 64, input_patch_size=H, nb=6).to(dev).train()
g = torch.Generator(device=dev).manual_seed(1)
real = torch.rand(2, 3, H, H, device=dev, generator=g)
fake = torch.rand(2, 3, H, H, device=dev, generator=g)
rp = torch.rand(2, 1, 1, 1, device=dev, generator=g)
gan, gp = L.GANLoss('wgan-gp', 1.0, 0.0), L.GradientPenaltyLoss(device=dev)
sd0 = {k: v.clone() for k, v in D.state_dict().items()}


def step(variant):
    D.load_state_dict(sd0)
    D.zero_grad(set_to_none=True)
    loss = 0
    if variant in ('real', 'all', 'nogp'):
        loss = loss + gan(D(real), True)
    if variant in ('all', 'nogp'):
        loss = loss + gan(D(fake), False)
    if variant in ('gp', 'all'):
        it = (rp * fake + (1 - rp) * real).requires_grad_(True)
        loss = loss + 10 * gp(it, D(it))
    loss.backward()
    return {k: p.grad.clone() for k, p in D.named_parameters() if p.grad is not None}


for variant in ('real', 'nogp', 'gp', 'all'):
    runs = [step(variant) for _ in range(3)]
    diff = sorted({k for r in runs[1:] for k in r if not torch.equal(r[k], runs[0][k])})
    print('%-5s differing grads: %s' % (variant, diff), flush=True)
