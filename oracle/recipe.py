"""Deterministic synthetic-weight and input recipe shared by the golden generator, the oracle and the tests.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

No pretrained RRDB/ESRGAN weights exist offline, so parity is established on seeded synthetic
weights.  The recipe follows the reference's own training-time initialisation, `init_weights(netG, 'kaiming',
scale=0.1)` (reference codes/models/networks.py:28-44, 62-74, 97-98): kaiming-normal, fan_in, a=0 → std sqrt(2/fan_in),
multiplied by `scale`.  The reference zeroes the biases; we draw small uniform biases instead so that the bias path of
every kernel is exercised.  Everything is drawn from NumPy PCG64 so the fixtures can be regenerated anywhere without the
reference.
"""
import numpy as np


def seeded_params(named_shapes, seed, w_scale=0.1, b_range=0.01):
    """named_shapes: iterable of (name, shape) in state_dict order. Returns {name: float32 ndarray}.

    Parameters whose name contains 'Filter' (the frozen CEM filters, CEMnet.py:130-135) are skipped: they come from the
    CEM filter design, not from the initialiser (networks.py:29-30 skips them too).
    """
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in named_shapes:
        if 'Filter' in name:
            continue
        shape = tuple(int(s) for s in shape)
        if name.endswith('weight') and len(shape) == 4:
            fan_in = shape[1] * shape[2] * shape[3]
            w = rng.standard_normal(shape) * np.sqrt(2.0 / fan_in) * w_scale
            out[name] = w.astype(np.float32)
        elif name.endswith('bias'):
            out[name] = rng.uniform(-b_range, b_range, size=shape).astype(np.float32)
        elif name.endswith('weight'):  # BatchNorm affine weight (discriminator)
            out[name] = (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
        else:
            raise ValueError('unexpected parameter %s' % name)
    return out


def seeded_inputs(seed, lr_shape, z_hr_shape=None, z_mode='pixel'):
    """LR ~ U[0,1) float32 NCHW; optional HR latent Z ~ U[-1,1) ('pixel') or per-image constant ('image').

    The per-image constant Z mirrors training-time feed_data (reference SRRaGAN_model.py:279-290).
    """
    rng = np.random.default_rng(seed)
    lr = rng.random(lr_shape, dtype=np.float64).astype(np.float32)
    z = None
    if z_hr_shape is not None:
        if z_mode == 'pixel':
            z = (2.0 * rng.random(z_hr_shape) - 1.0).astype(np.float32)
        else:
            b, c = z_hr_shape[:2]
            z = np.broadcast_to((2.0 * rng.random((b, c, 1, 1)) - 1.0), z_hr_shape).astype(np.float32).copy()
    return lr, z


def synthetic_learned_kernel(size=13, sigma=(1.6, 2.6), theta_deg=30.0, shift=(0.3, -0.2)):
    """A deterministic anisotropic, slightly off-centre blur kernel standing in for a KernelGAN estimate.

    KernelGAN (reference codes/KernelGAN/) cannot run offline (CUDA-only); its output is a k×k float64 ndarray summing
    to 1 that is handed to `CEMnet(config, upscale_kernel=k)` (GUI.py:1195-1214, CEMnet.py:17-22).  This stands in for
    such an estimate.
    """
    c = (size - 1) / 2.0
    y, x = np.mgrid[0:size, 0:size].astype(np.float64)
    x = x - c - shift[0]
    y = y - c - shift[1]
    t = np.deg2rad(theta_deg)
    xr = np.cos(t) * x + np.sin(t) * y
    yr = -np.sin(t) * x + np.cos(t) * y
    k = np.exp(-0.5 * ((xr / sigma[0]) ** 2 + (yr / sigma[1]) ** 2))
    return k / k.sum()
