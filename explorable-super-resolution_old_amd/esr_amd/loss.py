"""Training losses of the hot path's training step — counterpart of reference codes/models/modules/loss.py.

GANLoss (202-234), GradientPenaltyLoss (244-263) and CreateRangeLoss (236-242) with the reference semantics.
CreateRangeLoss does not hard-wire torch.cuda.FloatTensor (the reference does, which fails without CUDA); the range
lives on the input's device.
"""
import torch
import torch.nn as nn


class GANLoss(nn.Module):
    def __init__(self, gan_type, real_label_val=1.0, fake_label_val=0.0):
        super().__init__()
        self.gan_type = gan_type.lower()
        self.real_label_val = real_label_val
        self.fake_label_val = fake_label_val
        if self.gan_type == 'vanilla':
            self.loss = nn.BCEWithLogitsLoss()
        elif self.gan_type == 'lsgan':
            self.loss = nn.MSELoss()
        elif self.gan_type == 'wgan-gp':
            self.loss = lambda x, target: -1 * x.mean() if target else x.mean()
        else:
            raise NotImplementedError('GAN type [{:s}] is not found'.format(self.gan_type))

    def get_target_label(self, x, target_is_real):
        if self.gan_type == 'wgan-gp':
            return target_is_real
        return torch.empty_like(x).fill_(self.real_label_val if target_is_real else self.fake_label_val)

    def forward(self, x, target_is_real):
        return self.loss(x, self.get_target_label(x, target_is_real))


def CreateRangeLoss(legit_range):
    lo, hi = float(legit_range[0]), float(legit_range[1])

    def RangeLoss(x):
        # mean deviation from the legitimate range over all channels and pixels
        zero = torch.zeros(1, device=x.device, dtype=x.dtype)
        return torch.max(torch.max(x - hi, other=zero), other=torch.max(lo - x, other=zero)).mean()
    return RangeLoss


class GradientPenaltyLoss(nn.Module):
    """WGAN-GP: ((‖∂D(interp)/∂interp‖₂ − 1)²).mean() with create_graph (double backward through D)."""

    def __init__(self, device=torch.device('cpu')):
        super().__init__()
        self.register_buffer('grad_outputs', torch.Tensor())
        self.grad_outputs = self.grad_outputs.to(device)

    def get_grad_outputs(self, x):
        if self.grad_outputs.size() != x.size() or self.grad_outputs.device != x.device:
            self.grad_outputs = torch.ones_like(x)
        return self.grad_outputs

    def forward(self, interp, interp_crit):
        g = torch.autograd.grad(outputs=interp_crit, inputs=interp, grad_outputs=self.get_grad_outputs(interp_crit),
                                create_graph=True, retain_graph=True, only_inputs=True)[0]
        return ((g.view(g.size(0), -1).norm(2, dim=1) - 1) ** 2).mean()
