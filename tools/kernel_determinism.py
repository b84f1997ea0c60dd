"""Bitwise run-to-run determinism of the discriminator's HIP ops on one input: each conv op (forward, data gradient,
weight gradient) at the config-3 layer shapes and the fused BatchNorm + LeakyReLU (forward, backward, double
backward), 5 runs each.  Usage (GPU): python tools/kernel_determinism.py [precision]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

from esr_amd import bn, dconv  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else 'f32'
dconv.set_precision(prec)
dev = torch.device('cuda:0')
g = torch.Generator(device=dev).manual_seed(3)
B = 4
for name, ci, co, k, s, p, H in [('conv0_1', 64, 64, 4, 2, 1, 120), ('conv1_0', 64, 128, 3, 1, 1, 60),
                                  ('conv1_1', 128, 128, 4, 2, 1, 60), ('fc8', 256, 100, 8, 1, 0, 15)]:
    x = torch.randn(B, H, H, ci, device=dev, generator=g)
    w = torch.randn(co, ci, k, k, device=dev, generator=g) / (ci * k * k) ** 0.5
    Ho = dconv.out_size(H, k, s, p)
    gy = torch.randn(B, Ho, Ho, co, device=dev, generator=g)
    outs = {'fwd': [], 'dgrad': [], 'wgrad': []}
    for _ in range(5):
        outs['fwd'].append(dconv.conv_forward(x, w, None, k, s, p))
        outs['dgrad'].append(dconv.conv_dgrad(gy, w, k, s, p, H, H))
        outs['wgrad'].append(dconv.conv_wgrad(x, gy, k, s, p))
    torch.cuda.synchronize()
    print(name, {op: all(torch.equal(v[0], t) for t in v[1:]) for op, v in outs.items()}, flush=True)
# fused BN + LeakyReLU and its two backwards
bnm = torch.nn.BatchNorm2d(128).to(dev).train()
x = torch.randn(B, 128, 60, 60, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
res = []
for _ in range(5):
    xx = x.clone().requires_grad_(True)
    y = bn.bn_lrelu(xx, bnm, 0.2)
    gx, = torch.autograd.grad((y * y).sum(), xx, create_graph=True)
    (gg,) = torch.autograd.grad((gx * gx).sum(), xx)
    res.append((y.detach(), gx.detach(), gg))
torch.cuda.synchronize()
print('bn_lrelu', [all(torch.equal(a[i], b[i]) for b in res[1:]) for i, a in enumerate([res[0]] * 3)], flush=True)
