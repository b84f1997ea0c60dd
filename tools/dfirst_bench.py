#!/usr/bin/env python3
"""Time the discriminator's first conv block at the config-3 shape (B=16, 304x304, 3 -> 64): the fused kernels
(dconv.dfirst_lrelu: esr_dfirst_fwd / esr_dfirst_bwd + reduce) against the general path (ESR_DFIRST=0: im2col, the
1x1 conv at the D precision, LeakyReLU), forward and forward + backward (input, weight and bias gradients).
    usage: python tools/dfirst_bench.py [B H W]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))
import torch  # noqa: E402
from esr_amd import dconv  # noqa: E402
from esr_amd.discriminator import _run  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


def main():
    B, H, W = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (16, 304, 304)
    dev = torch.device('cuda')
    torch.manual_seed(0)
    seq = torch.nn.Sequential(dconv.HipConv2d(3, 64, 3, 1, 1), torch.nn.LeakyReLU(0.2, True)).to(dev)
    x = torch.randn(B, 3, H, W, device=dev, requires_grad=True)
    g = torch.randn(B, H, W, 64, device=dev).permute(0, 3, 1, 2)
    out_b = B * H * W * 64 * 4
    for fused in (True, False):
        dconv.FUSED_FIRST = fused

        def fwd():
            with torch.no_grad():
                _run(seq, x)

        def fwd_bwd():
            y = _run(seq, x)
            torch.autograd.backward(y, g)
        tf, tb = timed(fwd), timed(fwd_bwd)
        print('%-8s forward %8.1f us (%5.2f TB/s of the 64-channel output)   forward + backward %8.1f us'
              % ('fused' if fused else 'general', tf, out_b / tf / 1e6, tb), flush=True)
    dconv.FUSED_FIRST = True


if __name__ == '__main__':
    main()
