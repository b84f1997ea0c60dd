"""BatchNorm2d (training mode) + LeakyReLU of the discriminator's conv_block(CNA) (block.py:129-156), fused on HIP
(csrc/esr_bn.hip): forward, backward and the backward's own backward, which the WGAN-GP penalty needs
(loss.py:244-263: autograd.grad(create_graph=True) through the discriminator, then .backward()).

Same semantics as nn.BatchNorm2d(affine, track_running_stats) followed by nn.LeakyReLU(slope) in training mode: batch
statistics over (N, H, W) with the biased variance, running buffers updated with the unbiased one (momentum, or the
cumulative average when momentum is None), num_batches_tracked incremented.  The activations are the channels-last
tensors the discriminator convolutions produce ([P][C] rows).  Without this, PyTorch runs the penalty's double
backward through BatchNorm as ~10 elementwise / reduction kernels per layer on channels-last views."""
import ctypes

import torch

from . import _lib


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _ws(lib, P, C, dev):
    return torch.empty(int(lib.esr_bn_workspace_floats(P, C)), device=dev, dtype=torch.float32)


class _BNLReLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, gamma, beta, eps, slope, run=None):
        """run = (running_mean, running_var, num_batches_tracked, momentum): updated by the same launch, or None."""
        lib = _lib.load()
        P, C = x2.shape
        y = torch.empty_like(x2)
        mu, rs, var = (torch.empty(C, device=x2.device) for _ in range(3))
        rm, rv, nbt, m = run if run is not None else (None, None, None, 0.0)
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        _lib.check(lib.esr_bn_lrelu_fwd(x2.data_ptr(), P, C, gamma.data_ptr(), beta.data_ptr(), eps, slope,
                                        y.data_ptr(), mu.data_ptr(), rs.data_ptr(), var.data_ptr(),
                                        _ws(lib, P, C, x2.device).data_ptr(), ptr(rm), ptr(rv), ptr(nbt), m,
                                        _stream(x2)), 'esr_bn_lrelu_fwd')
        ctx.save_for_backward(x2, gamma, beta, mu, rs)
        ctx.slope = slope
        ctx.mark_non_differentiable(mu, var)
        return y, mu, var

    @staticmethod
    def backward(ctx, gy, _gmu, _gvar):
        x2, gamma, beta, mu, rs = ctx.saved_tensors
        gx, gg, gb = _BNLReLUBwdFn.apply(x2, gamma, beta, gy.contiguous(), mu, rs, ctx.slope)
        return gx, gg, gb, None, None, None


class _BNLReLUBwdFn(torch.autograd.Function):
    """(x, γ, gy) -> (gx, dγ, dβ) of the fused layer, differentiable once more (esr_bn_lrelu_bwd2)."""

    @staticmethod
    def forward(ctx, x2, gamma, beta, gy, mu, rs, slope):
        lib = _lib.load()
        P, C = x2.shape
        gx = torch.empty_like(x2)
        sums2 = torch.empty(2, C, device=x2.device)
        _lib.check(lib.esr_bn_lrelu_bwd(x2.data_ptr(), gy.data_ptr(), P, C, gamma.data_ptr(), beta.data_ptr(),
                                        mu.data_ptr(), rs.data_ptr(), slope, gx.data_ptr(), sums2.data_ptr(),
                                        _ws(lib, P, C, x2.device).data_ptr(), _stream(x2)), 'esr_bn_lrelu_bwd')
        ctx.save_for_backward(x2, gamma, beta, gy, mu, rs, sums2)
        ctx.slope = slope
        return gx, sums2[1].clone(), sums2[0].clone()

    @staticmethod
    def backward(ctx, ggx, ggg, ggb):
        x2, gamma, beta, gy, mu, rs, sums2 = ctx.saved_tensors
        lib = _lib.load()
        P, C = x2.shape
        g_x, g_gy = torch.empty_like(x2), torch.empty_like(x2)
        g_gamma = torch.empty(C, device=x2.device)
        ggx = ggx.contiguous() if ggx is not None else None
        ptr = lambda t: None if t is None else t.contiguous().data_ptr()  # noqa: E731
        _lib.check(lib.esr_bn_lrelu_bwd2(x2.data_ptr(), gy.data_ptr(), ptr(ggx), ptr(ggg), ptr(ggb), P, C,
                                         gamma.data_ptr(), beta.data_ptr(), mu.data_ptr(), rs.data_ptr(), ctx.slope,
                                         sums2.data_ptr(), g_x.data_ptr(), g_gy.data_ptr(), g_gamma.data_ptr(),
                                         _ws(lib, P, C, x2.device).data_ptr(), _stream(x2)), 'esr_bn_lrelu_bwd2')
        return g_x, g_gamma, None, g_gy, None, None, None


def bn_lrelu(x, bn, slope):
    """lrelu(bn(x)) for a training-mode nn.BatchNorm2d `bn` on an NCHW tensor with channels-last storage; updates
    bn's running buffers like nn.BatchNorm2d.forward does.  Returns an NCHW tensor with channels-last storage."""
    B, C, H, W = x.shape
    xh = x.permute(0, 2, 3, 1)
    if not xh.is_contiguous():
        xh = xh.contiguous()
    # running buffers updated by the forward launch itself (momentum; the cumulative average of momentum=None needs
    # the count on the host and keeps the PyTorch ops)
    inplace = bn.track_running_stats and bn.momentum is not None and bn.running_mean is not None and \
        bn.num_batches_tracked is not None and bn.num_batches_tracked.dtype == torch.int64
    run = (bn.running_mean, bn.running_var, bn.num_batches_tracked, float(bn.momentum)) if inplace else None
    y, mu, var = _BNLReLUFn.apply(xh.view(B * H * W, C), bn.weight, bn.bias, float(bn.eps), float(slope), run)
    if bn.track_running_stats and not inplace:
        with torch.no_grad():
            bn.num_batches_tracked.add_(1)
            m = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
            n = B * H * W
            bn.running_mean.mul_(1 - m).add_(mu, alpha=m)
            bn.running_var.mul_(1 - m).add_(var, alpha=m * n / max(n - 1, 1))
    return y.view(B, H, W, C).permute(0, 3, 1, 2)


class _LReLUFn(torch.autograd.Function):
    """LeakyReLU on a contiguous channels-last tensor, out of place (y saved; its sign is the mask)."""

    @staticmethod
    def forward(ctx, x, slope):
        y = torch.nn.functional.leaky_relu(x, slope)  # one pass (x > 0 ? x : x·slope); where() took three
        ctx.save_for_backward(y)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        return _LReLUBwdFn.apply(g.contiguous(), y, ctx.slope), None


class _LReLUBwdFn(torch.autograd.Function):
    """g -> g·lrelu'(y): linear in g (its own backward applies the same mask); the mask has zero derivative."""

    @staticmethod
    def forward(ctx, g, y, slope):
        ctx.save_for_backward(y)
        ctx.slope = slope
        return torch.ops.aten.leaky_relu_backward(g, y, slope, True)  # y > 0 ? g : g·slope, one pass

    @staticmethod
    def backward(ctx, gg):
        (y,) = ctx.saved_tensors
        return _LReLUBwdFn.apply(gg.contiguous(), y, ctx.slope), None, None


def lrelu_nhwc(x, slope):
    """nn.LeakyReLU(slope) (in-place or not: same values) on an NCHW tensor with channels-last storage, computed out of
    place on the contiguous NHWC storage.  The discriminator's in-place LeakyReLU on such a view made autograd clone and
    re-copy the 64-channel 304² activation of its first conv about 30 times per training step."""
    y = _LReLUFn.apply(x.permute(0, 2, 3, 1), slope)
    return y.permute(0, 3, 1, 2)
