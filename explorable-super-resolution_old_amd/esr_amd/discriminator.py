"""Discriminator_VGG_128_ — counterpart of reference codes/models/modules/architecture.py:222-284.

The patch ("pseudo-FC") VGG discriminator the shipped training config uses (network_D: n_layers 6, nf 64, batch norm,
leakyrelu, CNA; train_esrgan_CEM.json).  As shipped, `define_D` builds `Discriminator_VGG_128` and passes `nb=`, which
that class does not accept (TypeError, networks.py:115-120 vs architecture.py:183-184); the class that takes `nb` is
this one — `define_D` here builds it (SURVEY.md §7 "training path is broken as shipped").  Same module tree, hence the
same state_dict keys and order as the reference (tests/golden/disc_*.npz).

Every convolution (3×3 s1, 4×4 s2, the 8×8 "pseudo-FC" and the 1×1 head) is a HipConv2d: forward, data gradient
and weight gradient on the MFMA kernels of csrc/esr_dconv.hip, differentiable to any order, so the D step and the
WGAN-GP double backward (loss.py:244-263) run every convolution on HIP.  Their precision is the process-wide
esr_amd.dconv.PRECISION (default 'x3': split-f16 operands with per-K-step power-of-two scaling on f16 MFMA; 'x6' and
exact 'f32' via dconv.set_precision or ESR_DCONV_PRECISION) — except the first conv block (3 -> 64, 3x3, + LeakyReLU),
which runs fused in exact fp32 on the VALU at every precision (dconv.dfirst_lrelu, csrc/esr_dfirst.hip: 27 MACs per
output feed no MFMA; the layer's cost is its 64-channel output, now moved once per pass).  BatchNorm and LeakyReLU
run fused on HIP in training mode (esr_amd/bn.py: forward, backward, double backward); in eval mode they are
PyTorch ops on the channels-last activations the convolutions produce.
"""
import os

import torch.nn as nn

from .bn import bn_lrelu, lrelu_nhwc
from .dconv import HipConv2d, dfirst_lrelu, dfirst_ok

# BatchNorm + LeakyReLU pairs fused on HIP in training mode (esr_amd/bn.py); ESR_FUSED_BN=0 keeps PyTorch's ops
FUSED_BN = os.environ.get('ESR_FUSED_BN', '1') != '0'

LRELU = 0.2


def _conv_block(in_nc, out_nc, k, stride=1, norm=True, act=True, zero_pad=True):
    """conv_block(mode='CNA') of block.py:129-156 flattened the way `sequential` does (block.py:106-126)."""
    pad = (k - 1) // 2 if zero_pad else 0  # get_valid_padding; pad_type=None means no padding at all
    mods = [HipConv2d(in_nc, out_nc, kernel_size=k, stride=stride, padding=pad, bias=True)]
    if norm:
        mods.append(nn.BatchNorm2d(out_nc, affine=True))
    if act:
        mods.append(nn.LeakyReLU(LRELU, True))
    return mods


class Discriminator_VGG_128_(nn.Module):
    def __init__(self, in_nc, base_nf, norm_type='batch', act_type='leakyrelu', mode='CNA', input_patch_size=128,
                 num_2_strides=5, nb=10):
        super().__init__()
        if norm_type != 'batch' or act_type != 'leakyrelu' or mode != 'CNA':
            raise NotImplementedError('Discriminator_VGG_128_ is built for the shipped batch/leakyrelu/CNA config')
        assert num_2_strides <= 5
        self.num_2_strides = num_2_strides
        nf = base_nf
        plan = [(in_nc, nf, 3, 1, False), (nf, nf, 4, 2, True), (nf, 2 * nf, 3, 1, True), (2 * nf, 2 * nf, 4, 2, True),
                (2 * nf, 4 * nf, 3, 1, True), (4 * nf, 4 * nf, 4, 2, True), (4 * nf, 8 * nf, 3, 1, True),
                (8 * nf, 8 * nf, 4, 2, True), (8 * nf, 8 * nf, 3, 1, True), (8 * nf, 8 * nf, 4, 2, True)]
        strides_left = num_2_strides
        mods = []
        for i, (ci, co, k, s, norm) in enumerate(plan[:nb]):
            if s == 2:
                s = 2 if strides_left > 0 else 1
                strides_left -= 1
            mods += _conv_block(ci, co, k, s, norm=norm)
        self.features = nn.Sequential(*mods)
        self.last_FC_layers = False
        nfeat = [m for m in self.features.children()][-2].num_features
        self.classifier = nn.Sequential(nn.Sequential(*_conv_block(nfeat, min(100, nfeat), 8, zero_pad=False)),
                                        nn.LeakyReLU(LRELU, False),
                                        nn.Sequential(*_conv_block(min(100, nfeat), 1, 1)))

        head = os.environ.get('ESR_D_HEAD_PRECISION')  # (experiment) the classifier's convs in their own precision
        if head:
            for m in self.classifier.modules():
                if isinstance(m, HipConv2d):
                    m.esr_precision = head

    def forward(self, x):
        return _run(self.classifier, _run(self.features, x))


def _run(seq, x):
    """seq(x), with every training-mode BatchNorm2d -> LeakyReLU pair (conv_block's norm + act) run as the fused HIP
    layer of bn.py (forward, backward and double backward), the first conv block (3 -> 64 3x3 conv + LeakyReLU) on the
    fused exact-fp32 kernels of dconv.dfirst_lrelu, and the other LeakyReLUs out of place on the channels-last storage
    (bn.lrelu_nhwc); nested Sequentials are walked the same way."""
    mods = list(seq.children())
    i = 0
    while i < len(mods):
        m = mods[i]
        nxt = mods[i + 1] if i + 1 < len(mods) else None
        if isinstance(m, nn.Sequential):
            x = _run(m, x)
        elif isinstance(m, HipConv2d) and isinstance(nxt, nn.LeakyReLU) and x.is_cuda and dfirst_ok(m):
            x = dfirst_lrelu(x, m, nxt.negative_slope)  # conv0 + its LeakyReLU, one fused pass (esr_dfirst_*)
            i += 1
        elif FUSED_BN and isinstance(m, nn.BatchNorm2d) and m.training and isinstance(nxt, nn.LeakyReLU) and x.is_cuda:
            x = bn_lrelu(x, m, nxt.negative_slope)
            i += 1
        elif FUSED_BN and isinstance(m, nn.LeakyReLU) and x.is_cuda and \
                x.permute(0, 2, 3, 1).is_contiguous():  # a LeakyReLU without norm in front (conv0, classifier)
            x = lrelu_nhwc(x, m.negative_slope)
        else:
            x = m(x)
        i += 1
    return x
