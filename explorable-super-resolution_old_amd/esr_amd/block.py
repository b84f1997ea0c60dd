"""Parameter-holding building blocks with the reference's module hierarchy — counterpart of codes/models/modules/block.py.

These classes exist so that `state_dict()` keys, shapes and ORDER are exactly the reference's (checkpoint loading maps
keys by position, base_model.py:117-141).  They hold nn.Conv2d parameters; their forward is not used on the hot path:
RRDBNet.forward hands the whole generator to the HIP executor (esr_amd/engine.py), which reads these parameters.
Calling a sub-block directly raises, because there is no per-block CPU/PyTorch fallback in this build.
"""
import torch.nn as nn

LRELU_SLOPE = 0.2  # block.py:10 act(neg_slope=0.2)


class _ContainerOnly(nn.Module):
    def forward(self, *args, **kwargs):
        raise RuntimeError('%s is a parameter container; run the whole generator through RRDBNet / CEM_PyTorch '
                           '(HIP executor)' % type(self).__name__)


def conv_block(in_nc, out_nc, kernel_size=3, act=True, return_module_list=False):
    """conv_block(mode='CNA', norm None) of block.py:129-156: Conv2d(k, padding=k//2, bias) [+ LeakyReLU(0.2)].
    Returns nn.Sequential(conv[, act]) or, with return_module_list, the bare module list (block.py:106-126)."""
    mods = [nn.Conv2d(in_nc, out_nc, kernel_size=kernel_size, padding=kernel_size // 2, bias=True)]
    if act:
        mods.append(nn.LeakyReLU(LRELU_SLOPE, True))
    if return_module_list:
        return mods
    return nn.Sequential(*mods)


class ResidualDenseBlock_5C(_ContainerOnly):
    """block.py:196-242 (ModuleList mode): convs[i] = Conv(nc + i*gc + nl -> gc | nc), LReLU for i < 4."""

    def __init__(self, nc, gc=32, latent_input_channels=0):
        super().__init__()
        self.convs = nn.ModuleList([conv_block(nc + i * gc + latent_input_channels, gc if i < 4 else nc, act=i < 4)
                                    for i in range(5)])


class RRDB(_ContainerOnly):
    """block.py:245-270."""

    def __init__(self, nc, gc=32, latent_input_channels=0):
        super().__init__()
        self.num_latent_channels = latent_input_channels
        self.RDB1 = ResidualDenseBlock_5C(nc, gc, latent_input_channels)
        self.RDB2 = ResidualDenseBlock_5C(nc, gc, latent_input_channels)
        self.RDB3 = ResidualDenseBlock_5C(nc, gc, latent_input_channels)


class ShortcutBlock(_ContainerOnly):
    """block.py:76-103 with use_module_list=True: sub = ModuleList(nb RRDBs + LR_conv)."""

    def __init__(self, submodules, latent_input_channels=0):
        super().__init__()
        self.sub = nn.ModuleList(submodules)
        self.num_latent_channels = latent_input_channels


def upconv_blcok(in_nc, out_nc, upscale_factor=2):
    """block.py:294-301: Sequential(Upsample(nearest), Conv2d, LeakyReLU) — keys '<i>.1.weight/bias'."""
    return nn.Sequential(nn.Upsample(scale_factor=upscale_factor, mode='nearest'),
                         *conv_block(in_nc, out_nc, act=True, return_module_list=True))
