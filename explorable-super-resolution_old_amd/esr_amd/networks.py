"""Generator factory — counterpart of reference codes/models/networks.py (define_G, init_weights).

`define_G(opt, CEM=None, num_latent_channels=None)` reads the same option keys (network_G.*, scale, gpu_ids,
is_train, datasets.train.patch_size) and returns the same object shape: CEM_PyTorch(RRDBNet) when network_G.CEM_arch,
initialised with kaiming×0.1 when training (networks.py:95-98), wrapped so that `.module` reaches it when gpu_ids is
set (networks.py:99-101).  Multi-GPU in this build is one process per GPU (torch.distributed over RCCL), so the
wrapper is a single-device nn.DataParallel on the process's current device, never a multi-device replicate/scatter.
"""
import functools

import torch
import torch.nn as nn
from torch.nn import init

from . import architecture as arch
from . import engine as E


_PLAIN = (int, float, bool, str, type(None))


class DeviceParallel(nn.DataParallel):
    """The single-device nn.DataParallel of define_G / define_D (networks.py:99-101, 125-126): the same `.module`,
    state_dict keys, isinstance and device check, without DataParallel.forward's per-call walk of the module tree.

    DataParallel.forward walks every submodule for the parameters and again for the buffers to check their device
    (RRDB-23: ~1000 modules, 1.5–3 ms of host time per call, at the start of a training step while the GPU waited), then
    scatters the inputs to its one device.  Here the check reads the cached parameter list (engine.param_list,
    revalidated per call) and a buffer list cached with it, and inputs already on the device are passed through (the
    single-device scatter of a tensor on its device is an identity); anything else takes DataParallel.forward."""

    def _tensors(self):
        plist = E.param_list(self.module)
        c = self.__dict__.get('_esr_tensors')
        if c is None or c[0] is not plist:
            c = (plist, plist + [b for b in self.module.buffers()])
            self.__dict__['_esr_tensors'] = c
        return c[1]

    def forward(self, *inputs, **kwargs):
        if len(self.device_ids) != 1:
            return super().forward(*inputs, **kwargs)
        idx = self.src_device_obj.index
        for t in self._tensors():
            if t.get_device() != idx:
                raise RuntimeError('module must have its parameters and buffers on device %s (device_ids[0]) but found '
                                   'one of them on device: %s' % (self.src_device_obj, t.device))
        local = lambda x: x.get_device() == idx if torch.is_tensor(x) else isinstance(x, _PLAIN)  # noqa: E731
        if all(local(x) for x in inputs) and all(local(x) for x in kwargs.values()):
            return self.module(*inputs, **kwargs)
        return super().forward(*inputs, **kwargs)


def weights_init_kaiming(m, scale=1):
    """networks.py:28-44 (CEM filter layers are skipped)."""
    if getattr(m, 'filter_layer', False):
        return
    classname = m.__class__.__name__
    if classname.find('Conv') != -1 or classname.find('Linear') != -1:
        init.kaiming_normal_(m.weight.data, a=0, mode='fan_in')
        m.weight.data *= scale
        if m.bias is not None:
            m.bias.data.zero_()
    elif classname.find('BatchNorm2d') != -1:
        init.constant_(m.weight.data, 1.0)
        init.constant_(m.bias.data, 0.0)


def init_weights(net, init_type='kaiming', scale=1, std=0.02):
    if init_type != 'kaiming':
        raise NotImplementedError('only the kaiming initialisation used by define_G/define_D is provided')
    net.apply(functools.partial(weights_init_kaiming, scale=scale))


def define_D(opt, CEM=None):
    """networks.py:105-127.  The shipped `discriminator_vgg_128` + `n_layers` combination builds
    Discriminator_VGG_128_(nb=n_layers) (the reference's define_G passes nb= to the class without it: TypeError)."""
    from .discriminator import Discriminator_VGG_128_
    gpu_ids = opt['gpu_ids']
    opt_net = opt['network_D']
    if opt_net['which_model_D'] != 'discriminator_vgg_128':
        raise NotImplementedError('Discriminator model [{:s}] not recognized'.format(opt_net['which_model_D']))
    patch = opt['datasets']['train']['patch_size']
    if CEM is not None:
        patch -= 2 * int(CEM.invalidity_margins_HR)
    kwargs = {'num_2_strides': opt_net['num_2_strides']} if 'num_2_strides' in opt_net else {}
    netD = Discriminator_VGG_128_(in_nc=opt_net['in_nc'], base_nf=opt_net['nf'], norm_type=opt_net['norm_type'],
                                  act_type=opt_net['act_type'], mode=opt_net['mode'], input_patch_size=patch,
                                  nb=opt_net['n_layers'], **kwargs)
    init_weights(netD, init_type='kaiming', scale=1)
    if gpu_ids:
        dev = torch.cuda.current_device()
        netD = DeviceParallel(netD.to(dev), device_ids=[dev])
    return netD


def define_G(opt, CEM=None, num_latent_channels=None):
    gpu_ids = opt['gpu_ids']
    opt_net = opt['network_G']
    which_model = opt_net['which_model_G']
    latent = opt_net.get('latent_input')
    latent = latent if latent not in (None, 'None') else None
    opt_net['latent_input'] = latent
    if which_model != 'RRDB_net':
        raise NotImplementedError('Generator model [{:s}] not recognized'.format(which_model))
    netG = arch.RRDBNet(in_nc=opt_net['in_nc'], out_nc=opt_net['out_nc'], nf=opt_net['nf'], nb=opt_net['nb'],
                        gc=opt_net['gc'], upscale=opt_net['scale'] if 'scale' in opt_net else opt['scale'],
                        norm_type=opt_net.get('norm_type'), act_type='leakyrelu', mode=opt_net.get('mode', 'CNA'),
                        upsample_mode='upconv',
                        latent_input=(latent + '_' + opt_net['latent_input_domain']) if latent is not None else None,
                        num_latent_channels=num_latent_channels)
    if opt_net.get('CEM_arch'):
        netG = CEM.WrapArchitecture_PyTorch(netG, opt['datasets']['train']['patch_size'] if opt['is_train'] else None)
    if opt['is_train']:
        init_weights(netG, init_type='kaiming', scale=0.1)
    if gpu_ids:
        assert torch.cuda.is_available()
        dev = torch.cuda.current_device()
        netG = DeviceParallel(netG.to(dev), device_ids=[dev])
    return netG
