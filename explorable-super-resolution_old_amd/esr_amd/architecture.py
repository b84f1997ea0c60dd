"""RRDBNet generator — counterpart of codes/models/modules/architecture.py:102-175 (RRDBNet).

Same constructor signature, attributes (`latent_input`, `num_latent_channels`, `upscale`, `Z`) and state_dict layout
as the reference; forward runs on the HIP executor (esr_amd/engine.py).
"""
import math

import torch.nn as nn

from . import block as B
from . import engine


class RRDBNet(nn.Module):
    def __init__(self, in_nc, out_nc, nf, nb, gc=32, upscale=4, norm_type=None, act_type='leakyrelu', mode='CNA',
                 upsample_mode='upconv', latent_input=None, num_latent_channels=None):
        super().__init__()
        if norm_type is not None or act_type != 'leakyrelu' or mode != 'CNA' or upsample_mode != 'upconv':
            # define_G (networks.py:89-92) only ever builds this configuration
            raise NotImplementedError('esr_amd RRDBNet supports norm None, leakyrelu, CNA, upconv (the define_G path)')
        if upscale == 3:
            # the reference cannot build ×3 either: its nearest-×3 upconv_blcok is an nn.Sequential concatenated to a
            # list (architecture.py:132-133, 144: TypeError: can only concatenate list (not "Sequential") to list)
            raise NotImplementedError('RRDBNet ×3: the reference raises TypeError at architecture.py:144')
        if upscale not in (2, 4):
            raise NotImplementedError('esr_amd RRDBNet implements ×2 (one nearest-×2 upconv) and ×4 (two)')
        self.latent_input = latent_input
        if num_latent_channels is not None and num_latent_channels > 0:
            num_latent_channels_HR = 1 * num_latent_channels
            if 'HR_rearranged' in latent_input:
                num_latent_channels *= upscale ** 2
        self.num_latent_channels = 1 * num_latent_channels  # TypeError on None, as architecture.py:111
        self.upscale = upscale
        n_upscale = int(math.log(upscale, 2))
        self.n_up, self.up_factor = n_upscale, 2
        if latent_input is not None:
            in_nc += num_latent_channels
        if latent_input is None or 'all_layers' not in latent_input:
            num_latent_channels, num_latent_channels_HR = 0, 0
        if latent_input is not None and latent_input != 'all_layers_HR_downscaled':
            raise NotImplementedError('esr_amd implements latent_input None or all_layers + HR_downscaled (the '
                                      'shipped configs, train_esrgan_CEM.json / GUI_esrgan.json)')
        self.nb, self.nf, self.gc, self.in_nc, self.out_nc = nb, nf, gc, in_nc, out_nc
        if nf != 64 or gc != 32:
            raise NotImplementedError('esr_amd RRDBNet kernels are specialised for nf=64, gc=32 (RRDB-23 ESRGAN)')
        self.nl = num_latent_channels  # latent channels concatenated into every trunk/HR conv
        fea_conv = B.conv_block(in_nc, nf, act=False, return_module_list=True)
        rb_blocks = [B.RRDB(nf, gc=gc, latent_input_channels=num_latent_channels) for _ in range(nb)]
        LR_conv = B.conv_block(nf + num_latent_channels, nf, act=False, return_module_list=True)
        upsampler = [B.upconv_blcok(nf, nf, self.up_factor) for _ in range(n_upscale)]
        HR_conv0 = B.conv_block(nf + num_latent_channels_HR, nf, act=True, return_module_list=True)
        HR_conv1 = B.conv_block(nf + num_latent_channels_HR, out_nc, act=False, return_module_list=True)
        self.model = nn.ModuleList(fea_conv + [B.ShortcutBlock(rb_blocks + LR_conv, num_latent_channels)] +
                                   upsampler + HR_conv0 + HR_conv1)
        self.Z = None
        self._esr_cache = {}

    def forward(self, x):
        """architecture.py:151-175 (bare generator, no CEM)."""
        return engine.generator_forward(self, x, cem=None)
