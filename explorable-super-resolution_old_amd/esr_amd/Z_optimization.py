"""Latent-space (Z) optimisation on the HIP generator — counterpart of reference codes/Z_optimization.py.

The hot part of every iteration is the generator forward with retained activations and the HIP data-gradient sweep
back to the model input (train_engine.generator_backward with need_params=False): CEM adjoint → every conv's data
gradient → the Z slots of all LR/HR convs → bilinear ↓4 adjoint → replicate pre-pad adjoint (esr_input_adjoint).  The
generator is frozen exactly as the reference freezes it (Manage_Model_Grad_Requirements, Z_optimization.py:545-553),
so no weight gradients are computed.  Z is parametrised as Z_range·tanh(Z_pre) and stepped with Adam
(Z_optimization.py:292-300, 451).

Objectives carried over (Z_optimization.py:574-640): 'l1' (to data['HR']), 'max_STD' / 'min_STD' /
'STD_increase' / 'STD_decrease' (global masked STD), 'TV' (STD-preserving TV), 'Adversarial' (WGAN generator loss on
netD) and 'random_l1' (batch diversity).  The GUI-editing objectives (scribble, hist / dict, periodicity, local STD,
desired_SVD, Mag, VGG) are image-editing losses of the GUI, outside this hot path; they raise NotImplementedError.
"""
import numpy as np
import torch

from . import engine as E
from . import train_engine as TE
from .loss import GANLoss

_UNSUPPORTED = ('scribble', 'hist', 'dict', 'periodicity', 'local', 'desired_SVD', 'Mag', 'VGG')


class Optimizable_Z(torch.nn.Module):
    """Z_optimization.py:271-308: Z = Z_range·tanh(Z_pre) (identity without Z_range), optional Z mask that keeps the
    masked-out region at its initial value."""

    def __init__(self, Z_shape, Z_range=None, initial_pre_tanh_Z=None, Z_mask=None, random_perturbations=False,
                 device=None):
        super().__init__()
        device = device if device is not None else torch.device('cuda', torch.cuda.current_device())
        self.Z = torch.nn.Parameter(torch.zeros(Z_shape, dtype=torch.float32, device=device))
        if Z_mask is not None and not np.all(Z_mask):
            self.mask = torch.as_tensor(np.asarray(Z_mask), dtype=torch.float32, device=device)
            self.initial_pre_tanh_Z = 1 * initial_pre_tanh_Z.float().to(device)
        else:
            self.mask = None
        if initial_pre_tanh_Z is not None:
            assert tuple(initial_pre_tanh_Z.shape[1:]) == tuple(self.Z.shape[1:]) and \
                initial_pre_tanh_Z.size(0) in (1, self.Z.size(0)), 'Initilizer size does not match desired Z size'
            init = initial_pre_tanh_Z.float().to(device)
            if random_perturbations:
                init = init + 0.001 * torch.randn_like(init)
            self.Z.data[:init.size(0)] = init
        self.Z_range = Z_range

    def forward(self):
        if self.Z_range is not None:
            fmax = torch.finfo(self.Z.dtype).max
            self.Z.data.clamp_(-fmax, fmax)
        if self.mask is not None:
            self.Z.data = self.mask * self.Z.data + (1 - self.mask) * self.initial_pre_tanh_Z
        if self.Z_range is not None:
            return self.Z_range * torch.tanh(self.Z)
        return self.Z

    def PreTanhZ(self):
        if self.mask is not None:
            return self.mask * self.Z.data + (1 - self.mask) * self.initial_pre_tanh_Z
        return self.Z.data

    def Randomize_Z(self, what_2_shuffle):
        assert what_2_shuffle in ['all', 'allButFirst']
        if what_2_shuffle == 'all':
            torch.nn.init.xavier_uniform_(self.Z.data, gain=100)
        else:
            torch.nn.init.xavier_uniform_(self.Z.data[1:], gain=100)

    def Return_Detached_Z(self):
        return self.forward().detach()


def ArcTanH(x):
    eps = torch.finfo(x.dtype).eps
    return 0.5 * torch.log((1 + x + eps) / (1 - x + eps))


def TV_Loss(image):
    return (image[:, :, :, :-1] - image[:, :, :, 1:]).abs().mean(dim=(1, 2, 3)) + \
        (image[:, :, :-1, :] - image[:, :, 1:, :]).abs().mean(dim=(1, 2, 3))


class Z_optimizer:
    """Z_optimization.py:326-660 (same constructor arguments; see the module docstring for the objectives)."""
    MIN_LR = 1e-5

    def __init__(self, objective, Z_size, model, Z_range, max_iters, data=None, loggers=None, image_mask=None,
                 Z_mask=None, initial_Z=None, initial_LR=None, existing_optimizer=None, batch_size=1,
                 HR_unpadder=None, auto_set_hist_temperature=False, random_Z_inits=False):
        bad = [t for t in _UNSUPPORTED if t in objective]
        if bad or (image_mask is not None and 'l1' in objective):
            raise NotImplementedError('Z objective %r uses GUI image-editing losses (%s) outside the built path'
                                      % (objective, ', '.join(bad) or 'masked l1 = scribble loss'))
        self.device = model.device
        if initial_Z is not None or hasattr(model, 'model_input'):
            if initial_Z is None:
                initial_Z = 1 * model.GetLatent()
            pre = initial_Z / Z_range
            eps = torch.finfo(pre.dtype).eps
            initial_pre_tanh_Z = ArcTanH(torch.clamp(pre, min=-1 + eps, max=1. - eps))
        else:
            initial_pre_tanh_Z = None
        self.Z_model = Optimizable_Z([batch_size, model.num_latent_channels] + list(Z_size), Z_range=Z_range,
                                     initial_pre_tanh_Z=initial_pre_tanh_Z, Z_mask=Z_mask,
                                     random_perturbations=(random_Z_inits and 'random' not in objective) or
                                     ('random' in objective and 'limited' in objective), device=self.device)
        assert initial_LR is not None or existing_optimizer is not None, \
            'Should either supply optimizer from previous iterations or initial LR for new optimizer'
        self.objective = objective
        self.data = data
        self.model = model
        self.model_training = HR_unpadder is not None
        if image_mask is None:
            self.image_mask = torch.ones(list(model.fake_H.shape[2:]), device=self.device) \
                if getattr(model, 'fake_H', None) is not None else None
            self.Z_mask = None
        else:
            self.image_mask = torch.as_tensor(np.asarray(image_mask), dtype=torch.float32, device=self.device)
            self.Z_mask = torch.as_tensor(np.asarray(Z_mask), dtype=torch.float32, device=self.device)
        if not self.model_training and self.image_mask is not None:
            self.initial_STD = self.Masked_STD(first_image_only=True)
        if existing_optimizer is None:
            if 'l1' in objective and 'random' not in objective:
                if data is not None and 'HR' in data:
                    self.GT_HR = data['HR']
                self.loss = torch.nn.L1Loss()
            elif 'STD' in objective and 'TV' not in objective:
                assert objective in ['max_STD', 'min_STD', 'STD_increase', 'STD_decrease']
                if 'increase' in objective or 'decrease' in objective:
                    inc = data.get('STD_increment') if data is not None else None
                    self.desired_STD = self.initial_STD
                    if inc is None:
                        self.desired_STD = self.desired_STD * (1.05 if 'increase' in objective else 1 / 1.05)
                    else:
                        self.desired_STD = self.desired_STD + (inc if 'increase' in objective else -inc)
            elif 'TV' in objective:
                self.STD_PRESERVING_WEIGHT = 100
            elif 'Adversarial' in objective:
                self.netD = model.netD
                self.loss = GANLoss('wgan-gp', 1.0, 0.0)
            elif 'limited' in objective:
                self.initial_image = 1 * model.fake_H.detach()
                self.rmse_weight = data['rmse_weight']
            self.optimizer = torch.optim.Adam(self.Z_model.parameters(), lr=initial_LR)
        else:
            self.optimizer = existing_optimizer
        self.LR = initial_LR
        self.loggers = loggers
        self.cur_iter = 0
        self.max_iters = max_iters
        self.random_Z_inits = 'all' if (random_Z_inits or self.model_training) else \
            'allButFirst' if (initial_pre_tanh_Z is not None and initial_pre_tanh_Z.size(0) < batch_size) else False
        self.HR_unpadder = HR_unpadder

    def Masked_STD(self, first_image_only=False):
        fake = self.model.fake_H[:1] if first_image_only else self.model.fake_H
        return torch.std(fake * self.image_mask, dim=(1, 2, 3)).view(1, -1)

    def feed_data(self, data):
        self.data = data
        self.cur_iter = 0
        if 'l1' in self.objective:
            self.GT_HR = data['HR'].to(self.device)

    def Manage_Model_Grad_Requirements(self, disable):
        if disable:
            self.original_requires_grad_status = [p.requires_grad for p in self.model.netG.parameters()]
            for p in self.model.netG.parameters():
                p.requires_grad = False
        else:
            for p, s in zip(self.model.netG.parameters(), self.original_requires_grad_status):
                p.requires_grad = s

    def _loss(self, z_iter):
        fake = self.model.fake_H
        o = self.objective
        if 'random' in o:
            eye = torch.eye(fake.size(0), device=fake.device).view(fake.size(0), fake.size(0), 1, 1, 1)
            Z_loss = torch.min((fake.unsqueeze(0) - fake.unsqueeze(1)).abs() + eye, dim=0)[0]
            if 'limited' in o:
                Z_loss = Z_loss - self.rmse_weight * (fake - self.initial_image).abs()
            if self.Z_mask is not None:
                Z_loss = Z_loss * self.Z_mask
            Z_loss = -1 * Z_loss.mean(dim=(1, 2, 3))
        elif 'l1' in o:
            Z_loss = self.loss(fake, self.GT_HR.to(self.device))
        elif 'Adversarial' in o:
            Z_loss = self.loss(self.netD(self.model.CEM_net.HR_unpadder(fake)), True)
        elif 'STD' in o and 'TV' not in o:
            Z_loss = self.Masked_STD(first_image_only=False)
            if 'increase' in o or 'decrease' in o:
                Z_loss = (Z_loss - self.desired_STD) ** 2
            Z_loss = Z_loss.mean(0)
        elif 'TV' in o:
            Z_loss = (self.STD_PRESERVING_WEIGHT * (self.Masked_STD(first_image_only=False) - self.initial_STD) ** 2
                      ).mean(0) + TV_Loss(fake * self.image_mask)
        else:
            raise NotImplementedError(o)
        if 'max' in o:
            Z_loss = -1 * Z_loss
        return Z_loss

    def optimize(self):
        """Z_optimization.py:555-655."""
        if 'Adversarial' in self.objective:
            self.model.netG.train(True)
        self.Manage_Model_Grad_Requirements(disable=True)
        self.loss_values = []
        if self.random_Z_inits and self.cur_iter == 0:
            self.Z_model.Randomize_Z(what_2_shuffle=self.random_Z_inits)
        z_iter = self.cur_iter
        while True:
            if self.max_iters > 0:
                if z_iter == self.cur_iter + self.max_iters:
                    break
            elif len(self.loss_values) >= -self.max_iters:
                if z_iter == self.cur_iter - 5 * self.max_iters:
                    break
                first, last = float(self.loss_values[self.max_iters]), float(self.loss_values[-1])
                if (first - last) / np.abs(first) < 1e-2 * self.LR:
                    break
            # one Z iteration with the generator's x3 overflow checks read once at its end (not after the forward
            # and again after the backward, each a stream drain): from a snapshot of Z and its Adam state the
            # iteration is redone with the generator in exact fp32 if a flag was set
            snap = self._snapshot()
            with TE.deferred_overflow_checks() as chk:
                Z_loss = self._iteration(z_iter)
            if chk.overflowed():
                E.OVERFLOW_RERUNS += 1
                self._restore(snap)
                g = self.model.netG.module.generated_image_model if hasattr(self.model.netG, 'module') else None
                prev = getattr(g, 'esr_precision', None)
                if g is not None:
                    g.esr_precision = 'f32'
                try:
                    Z_loss = self._iteration(z_iter)
                finally:
                    if g is not None:
                        g.esr_precision = prev
            self.loss_values.append(Z_loss)
            z_iter += 1
        self.loss_values = [float(v) for v in self.loss_values]
        if not self.model_training:
            self.latest_Z_loss_values = [float(v) for v in self.latest_Z_loss_values]
        if 'Adversarial' in self.objective:
            self.model.netG.train(False)
        if 'random' in self.objective and 'limited' in self.objective and len(self.loss_values) > 1:
            self.loss_values[0] = self.loss_values[1]
        self.cur_iter = z_iter + 1
        Z_2_return = self.Z_model.Return_Detached_Z()
        self.Manage_Model_Grad_Requirements(disable=False)
        if self.model_training:
            self.data['Z'] = Z_2_return
            self.model.feed_data(self.data, need_HR=False)
            self.model.fake_H = self.model.netG(self.model.model_input)
        return Z_2_return

    def _snapshot(self):
        params = [p.detach().clone() for p in self.Z_model.parameters()]
        state = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.optimizer.state[p].items()}
                 for p in self.Z_model.parameters() if p in self.optimizer.state}
        return params, state, self.__dict__.get('latest_Z_loss_values')

    def _restore(self, snap):
        params, state, latest = snap
        with torch.no_grad():
            for p, v in zip(self.Z_model.parameters(), params):
                p.copy_(v)
                if id(p) in state:
                    for k, v2 in state[id(p)].items():
                        if torch.is_tensor(v2):
                            self.optimizer.state[p][k].copy_(v2)
                        else:
                            self.optimizer.state[p][k] = v2
                else:
                    self.optimizer.state.pop(p, None)
        if latest is not None:
            self.latest_Z_loss_values = latest

    def _iteration(self, z_iter):
        """Z_optimization.py:574-630: forward with the current Z, the objective, its backward to Z, one Adam step.
        Returns the (device) mean loss."""
        self.optimizer.zero_grad()
        self.data['Z'] = self.Z_model()
        self.model.feed_data(self.data, need_HR=False)
        self.model.fake_H = self.model.netG(self.model.model_input)
        if self.model_training:
            self.model.fake_H = self.HR_unpadder(self.model.fake_H)
        Z_loss = self._loss(z_iter)
        if self.loggers is not None:
            for n, logger in enumerate(self.loggers):
                v = Z_loss[n].item() if Z_loss.dim() > 0 else Z_loss.item()
                logger.print_format_results('val', {'epoch': 0, 'iters': z_iter, 'time': 0, 'model': '',
                                                    'lr': self.optimizer.param_groups[0]['lr'], 'Z_loss': v},
                                            dont_print=True)
        if not self.model_training:
            self.latest_Z_loss_values = Z_loss.detach().reshape(-1)  # kept on device (no per-iter sync)
        Z_loss = Z_loss.mean()
        Z_loss.backward()
        self.optimizer.step()
        return Z_loss.detach()
