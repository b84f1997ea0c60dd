"""CEM resampling — counterpart of reference codes/CEM/imresize_CEM.py.

Host side (NumPy float64, filter design only): the upscale kernel of a given scale factor (bicubic default, blurred
bicubic, or a custom/learned kernel re-centred with Center_Mass) and the zero-padded integer downscale used to measure
the ds_kernel's invalid margin.  `imresize` itself runs on the device (esr_amd/cem_ops.py stencils).

Behavioural difference by design: the reference caches the kernel in a process-global dict
(`imresize.kernels`, imresize_CEM.py:9,23-42) so the first kernel of a scale factor silently wins; here the kernel is an
explicit argument of every call.  The reference's string sentinels ('cubic', 'reset_2_default', 'blurry_cubic_<σ>')
are accepted with their documented meaning.
"""
import numpy as np
from scipy.signal import convolve2d
from scipy.signal.windows import gaussian
from scipy.stats import norm

_CUBIC_A = -0.75  # OpenCV INTER_CUBIC coefficient (cv2.resize used by imresize_CEM.py:91)


def calc_strides(array, factor, align_center=False):
    """imresize_CEM.py:73-86: split of the (sf-1) zero samples around each LR sample."""
    integer_factor = int(np.maximum(factor, 1 / factor))
    if align_center:
        half = np.ceil(np.array(array.shape[:2]) / 2 * (factor if factor > 1 else 1))
        pre = np.mod(half, integer_factor)
        pre[pre == 0] = integer_factor
        pre = (pre - 1).astype(np.int32)
        post = integer_factor - pre - 1
    else:
        post = (np.floor(integer_factor / 2) * np.ones(2)).astype(np.int32)
        pre = (integer_factor - post - 1).astype(np.int32)
    return pre, post


def cubic_taps(sf):
    """1-D taps of cv2.resize(delta, ×sf, INTER_CUBIC) around the delta (imresize_CEM.py:88-94).

    Output x samples source coordinate (x+0.5)/sf - 0.5; the response to a unit delta at source c is the Keys cubic
    (A = -0.75) of the distance.  Nonzero support only, exactly as Cubic_Kernel crops it.
    """
    def keys(t):
        t = abs(t)
        if t <= 1:
            return ((_CUBIC_A + 2) * t - (_CUBIC_A + 3)) * t * t + 1
        if t < 2:
            return ((_CUBIC_A * t - 5 * _CUBIC_A) * t + 8 * _CUBIC_A) * t - 4 * _CUBIC_A
        return 0.0
    size = 11
    c = int(np.ceil(size / 2)) - 1
    v = np.array([keys((x + 0.5) / sf - 0.5 - c) for x in range(sf * size)])
    nz = np.nonzero(v)[0]
    return v[nz[0]:nz[-1] + 1]


def Cubic_Kernel(sf):
    t = cubic_taps(sf)
    return np.outer(t, t)


def Gaussian_2D(sigma, size=None):
    """imresize_CEM.py:101-108."""
    if size is None:
        size = int(1 + 2 * np.ceil(-1 * norm.ppf(0.005, scale=sigma)))
    g = gaussian(size, sigma).reshape([1, size]) * gaussian(size, sigma).reshape([size, 1])
    return g / np.sum(g)


def Return_Filter_Energy_Distribution(filt):
    e = [np.sqrt(np.sum(filt ** 2))] + [np.sqrt(np.sum(filt[f:-f, f:-f] ** 2))
                                         for f in range(1, int(np.ceil(filt.shape[0] / 2)))]
    return np.array(e) / e[0]


def Center_Mass(kernel, ds_factor):
    """imresize_CEM.py:113-159: pad a custom kernel around its centre of mass, trim to 99 % energy with the kernel
    size constrained so that (size - 1 + (sf+1)%2) is a multiple of sf, renormalise."""
    assert kernel.shape[0] == kernel.shape[1], 'Currently supporting only square kernels'
    n = kernel.shape[0]
    gx, gy = np.meshgrid(np.arange(n), np.arange(n))
    cx = float(convolve2d(gx, kernel, mode='valid')[0, 0]) + 1
    cy = float(convolve2d(gy, kernel, mode='valid')[0, 0]) + 1
    x_pad, y_pad = 2 * (n / 2 - cx), 2 * (n / 2 - cy)
    padding_diff = np.round(np.abs(y_pad)) - np.round(np.abs(x_pad))
    pre_x, post_x = np.maximum(0, -x_pad), np.maximum(0, x_pad)
    pre_y, post_y = np.maximum(0, -y_pad), np.maximum(0, y_pad)

    def rnd(v):
        return int(np.round(v))

    def distribute(pre, post, extra):
        to_right = np.round(post) - post - (np.round(pre) - pre)
        pre, post = rnd(pre), rnd(post)
        if to_right > 0:
            return pre + int(np.floor(extra / 2)), post + int(np.ceil(extra / 2))
        return pre + int(np.ceil(extra / 2)), post + int(np.floor(extra / 2))

    if padding_diff > 0:
        pre_y, post_y = rnd(pre_y), rnd(post_y)
        pre_x, post_x = distribute(pre_x, post_x, padding_diff)
    elif padding_diff < 0:
        pre_x, post_x = rnd(pre_x), rnd(post_x)
        pre_y, post_y = distribute(pre_y, post_y, -padding_diff)
    kernel = np.pad(kernel, ((rnd(pre_y), rnd(post_y)), (rnd(pre_x), rnd(post_x))), mode='constant')
    assert kernel.shape[0] == kernel.shape[1], 'I caused the kernel to stop being a square...'
    margins = np.argwhere(Return_Filter_Energy_Distribution(kernel) < 0.99)[0][0] * np.ones(2, dtype=np.int32)
    side = 0
    while np.mod(kernel.shape[0] - np.sum(margins) - 1 + np.mod(ds_factor + 1, 2), ds_factor) != 0:
        margins[side] -= 1
        side = (side + 1) % 2
    kernel = kernel[margins[0]:-margins[1], margins[0]:-margins[1]]
    return kernel / np.sum(kernel)


def upscale_kernel(sf, kernel=None):
    """The anti-aliasing UPSCALE kernel of imresize(..., return_upscale_kernel=True) (imresize_CEM.py:18-47):
    base kernel (cubic / blurred cubic / custom downscale kernel rotated + Center_Mass'ed ×sf²) zero-padded by the
    even-factor stride imbalance."""
    sf = int(sf)
    pre, post = calc_strides(None, sf)
    kpost = np.maximum(0, pre - post)
    kpre = np.maximum(0, post - pre)
    if isinstance(kernel, np.ndarray):
        assert np.abs(1 - np.sum(kernel)) < np.finfo(np.float32).eps, 'Supplied non-default kernel does not sum to 1'
        k = Center_Mass(np.rot90(kernel, 2), ds_factor=sf) * sf ** 2
        assert k.shape[0] == k.shape[1], 'Only square kernels supported for now'
        assert np.all(np.mod(k.shape + kpost + kpre - 1, sf) == 0)
    else:
        assert kernel is None or any(w in kernel for w in ('cubic', 'blurry_cubic', 'reset_2_default'))
        k = Cubic_Kernel(sf)
        if kernel is not None and 'blurry_cubic' in kernel:
            k = convolve2d(k, Gaussian_2D(sigma=float(kernel[len('blurry_cubic_'):])))
    return np.pad(k, ((kpre[0], kpost[0]), (kpre[1], kpost[1])), mode='constant')


def downscale_zero_padded(im, sf, up_kernel):
    """imresize(im, [1/sf], use_zero_padding=True) for a 2-D image (imresize_CEM.py:44-45, 65-66, 70)."""
    pre, _ = calc_strides(im, 1 / sf)
    aa = np.rot90(up_kernel * (1 / sf) ** 2, 2)
    return convolve2d(im, aa, mode='same')[pre[0]::sf, pre[1]::sf]


def _to_device(im, device):
    """NumPy HW / HWC image -> float32 device tensor [C, H, W] (C = 1 for HW) and a function mapping results back."""
    import torch
    if isinstance(im, torch.Tensor):
        return im, lambda t: t
    if device is None:
        if not torch.cuda.is_available():
            raise RuntimeError('esr_amd.imresize: needs a ROCm device (this build has no CPU path)')
        device = torch.device('cuda', torch.cuda.current_device())
    a = np.asarray(im)
    hw = a.ndim < 3
    t = torch.from_numpy(np.ascontiguousarray(a[None] if hw else np.moveaxis(a, -1, 0), dtype=np.float32)).to(device)

    def back(y):
        y = y.cpu().numpy()
        return y[0] if hw else np.squeeze(np.moveaxis(y, 0, -1))
    return t, back


def imresize(im, scale_factor=None, output_shape=None, kernel=None, align_center=False, return_upscale_kernel=False,
             use_zero_padding=False, antialiasing=True, kernel_shift_flag=False, device=None):
    """imresize_CEM.py:7-71 on the device: integer down- or up-scaling of an image with the CEM anti-aliasing kernel.

    `im`: NumPy HW or HWC array (returned as a float32 NumPy array of the reference's shape — np.squeeze'd, :71) or a
    float32 ROCm tensor [..., H, W] (batched; returned on the device, e.g. on-the-fly LR for LRHR_dataset.py:87).
    `kernel`: None / 'cubic' / 'reset_2_default' (bicubic), 'blurry_cubic_<sigma>', or a custom DOWNSCALE kernel
    ndarray; unlike the reference it is not cached between calls (Appendix B of SURVEY.md), so pass the same kernel to
    every call that should use it.  `antialiasing` and `kernel_shift_flag` are accepted and unused, as in the
    reference.  align_center=True is the reference's hTh alias-sampling convention, not used with images: rejected.
    """
    if scale_factor is None:
        scale_factor = [output_shape[0] / im.shape[0]]
    elif not isinstance(scale_factor, (list, tuple)):
        scale_factor = [scale_factor]
    assert len(scale_factor) == 1 or scale_factor[0] == scale_factor[1]
    s = scale_factor[0]
    assert np.round(s) == s or np.round(1 / s) == 1 / s, 'Only supporting integer downsampling or upsampling rates'
    sf = int(np.maximum(s, 1 / s))
    k_up = upscale_kernel(sf, kernel)
    aa = k_up if s >= 1 else np.rot90(k_up * s ** 2, 2)
    if return_upscale_kernel:
        return aa
    if align_center:
        raise NotImplementedError('imresize: align_center=True is not supported for images')
    import torch
    from . import cem_ops
    x, back = _to_device(im, device)
    if output_shape is not None:
        assert np.all(s * np.array(x.shape[-2:]) == np.asarray(output_shape)[:2])
    if s >= 1:
        w = torch.from_numpy(np.ascontiguousarray(np.rot90(k_up, 2), dtype=np.float32)).to(x.device)
        y = cem_ops.upscale(x, w, sf, zero_pad=use_zero_padding)
    else:
        w = torch.from_numpy(np.ascontiguousarray(k_up / sf ** 2, dtype=np.float32)).to(x.device)
        y = cem_ops.downscale(x, w, sf, zero_pad=use_zero_padding)
    return back(y)
