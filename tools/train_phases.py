"""Where a config-3 training step spends its time: G forward+backward alone, the D step (WGAN-GP) alone, the full
optimize_parameters step; wall time per part (synchronised) and host-side enqueue time (no sync)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'explorable-super-resolution_old_amd'))
import bench_train as bt  # noqa: E402


def timed(fn, n=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    th = time.perf_counter() - t0
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, th / n * 1e3


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    from esr_amd.SRRaGAN_model import SRRaGANModel
    import argparse
    args = argparse.Namespace(batch=16, lr_size=96, nb=23, latent=True, gpus=1)
    torch.manual_seed(1000)
    model = SRRaGANModel(bt.make_opt(args), device=dev)
    g = torch.Generator(device='cpu').manual_seed(7)
    data = {'LR': torch.rand(16, 3, 96, 96, generator=g).to(dev), 'HR': torch.rand(16, 3, 384, 384, generator=g).to(dev)}

    def step():
        model.feed_data(data)
        model.optimize_parameters()
    for _ in range(3):
        step()
    print('full step      wall %.1f ms  host %.1f ms' % timed(step))
    model.feed_data(data)
    x = model.model_input

    def gfb():
        out = model.netG(x)
        out.sum().backward()
    print('G fwd+bwd      wall %.1f ms  host %.1f ms' % timed(gfb))

    def gf():
        with torch.no_grad():
            model.netG.train()
            for p in model.netG.parameters():
                pass
            model.netG(x)
    fake = model.netG(x).detach()[:, :, 40:-40, 40:-40].contiguous()
    real = data['HR'][:, :, 40:-40, 40:-40].contiguous()
    D = model.netD

    def dstep():
        pr, pf = D(real), D(fake)
        rp = torch.rand(16, 1, 1, 1, device=dev)
        it = (rp * fake + (1 - rp) * real).requires_grad_(True)
        loss = -pr.mean() + pf.mean() + 10 * model.cri_gp(it, D(it))
        loss.backward()
    print('D step         wall %.1f ms  host %.1f ms' % timed(dstep))

    def dfwd():
        with torch.no_grad():
            D(real)
    print('D fwd (nograd) wall %.1f ms  host %.1f ms' % timed(dfwd))


if __name__ == '__main__':
    main()
