"""Consistency Enforcing Module — counterpart of reference codes/CEM/CEMnet.py.

`CEMnet` designs the three fixed filters on the host (NumPy float64, once per model build: CEMnet.py:17-26,105-126);
`CEM_PyTorch` wraps a generator and runs the CEM back-projection on the GPU through the libesr_amd stencils
(esr_amd/engine.py: cem_apply).  The reference's NumPy image helpers (Pad_LR_Batch, Unpad_HR_Batch,
DT_Satisfying_Upscale, Project_2_kernel_subspace, Enforce_DT_on_Image_Pair; CEMnet.py:44-57,88-100) keep their NumPy
HWC signatures but compute on the device (esr_amd/cem_ops.py); they also take device tensors [..., H, W] for batches.  Module names, the frozen `Filter_OP` parameters and their state_dict order match the
reference (checkpoint loading skips keys containing 'Filter', base_model.py:138-139; CEMnet.py:241-242).
"""
import collections

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from scipy.signal import convolve2d as conv2

from . import cem_ops, engine
from .imresize_CEM import _to_device, calc_strides, downscale_zero_padded, upscale_kernel


class CEMnet:
    NFFT_add = 36

    def __init__(self, config, upscale_kernel=None):
        self.config = config
        self.ds_factor = np.array(config.scale_factor, dtype=np.int32)
        assert np.round(self.ds_factor) == self.ds_factor, 'Currently only supporting integer scale factors'
        assert upscale_kernel is None or isinstance(upscale_kernel, (str, np.ndarray)), \
            'Kernels should be given as ND-arrays, except for some specific possible strings'
        self.Set_Upscale_Kernel(upscale_kernel)

    def Set_Upscale_Kernel(self, upscale_kernel):
        """Redo the filter design for another kernel (CEMnet.py:22-26).  test.py:143-148 re-creates the whole model per
        image to change kernels; here CEM_PyTorch.Update_Filters(self) swaps the new filters into a built model."""
        self.upscale_kernel = upscale_kernel
        self._k_up = upscale_kernel_cached = upscale_kernel_of(int(self.ds_factor), upscale_kernel)
        self.ds_kernel = Return_kernel(self.ds_factor, upscale_kernel_cached)
        self.ds_kernel_invalidity_half_size_LR = self.Return_Invalid_Margin_Size_in_LR(
            'ds_kernel', self.config.filter_pertubation_limit)
        self.compute_inv_hTh()
        self.invalidity_margins_LR = 2 * self.ds_kernel_invalidity_half_size_LR + self.inv_hTh_invalidity_half_size
        self.invalidity_margins_HR = self.ds_factor * self.invalidity_margins_LR
        self._dev_filters = {}
        return self

    def Return_Invalid_Margin_Size_in_LR(self, filter, max_allowed_perturbation):
        """CEMnet.py:28-42: response of the filter to a constant image, normalised at the centre; the margin is one
        past the deepest pixel whose response deviates by more than the allowed perturbation."""
        n = 100
        assert filter in ['ds_kernel', 'inv_hTh']
        if filter == 'ds_kernel':
            resp = downscale_zero_padded(np.ones([int(self.ds_factor) * n] * 2), int(self.ds_factor), self._k_up)
        else:
            resp = conv2(np.ones([n, n]), self.inv_hTh, mode='same')
        resp = resp / resp[n // 2, n // 2]
        resp[resp <= 0] = max_allowed_perturbation / 2
        invalid = np.exp(-np.abs(np.log(resp))) < max_allowed_perturbation
        sizes = [np.argwhere(invalid[:n // 2, n // 2])[-1][0] + 1, np.argwhere(invalid[n // 2, :n // 2])[-1][0] + 1]
        return int(np.max(sizes))

    def compute_inv_hTh(self):
        """CEMnet.py:105-126: regularised inverse of h^T h (aliased to the LR grid), recentred and energy-cropped."""
        sf = int(self.ds_factor)
        hTh = conv2(self.ds_kernel, np.rot90(self.ds_kernel, 2)) * sf ** 2
        pre, _ = calc_strides(hTh, 1 / sf, align_center=True)
        hTh = hTh[pre[0]::sf, pre[1]::sf]
        pad = self.NFFT_add // 2
        H = np.fft.fft2(np.pad(hTh, ((pad, pad), (pad, pad)), mode='constant'))
        H = H * np.maximum(1, self.config.lower_magnitude_bound / np.abs(H))
        inv = np.real(np.fft.ifft2(1 / H))
        max_row, max_col = np.unravel_index(np.argmax(inv), inv.shape)
        if not np.all(np.ceil(np.array(inv.shape) / 2) == np.array([max_row, max_col]) - 1):
            half = min(inv.shape[0] - max_row - 1, inv.shape[0] - max_col - 1, max_row, max_col)
            inv = inv[max_row - half:max_row + half + 1, max_col - half:max_col + half + 1]
        self.inv_hTh = inv
        self.inv_hTh_invalidity_half_size = self.Return_Invalid_Margin_Size_in_LR(
            'inv_hTh', self.config.filter_pertubation_limit)
        drop = inv.shape[0] // 2 - self.Return_Invalid_Margin_Size_in_LR(
            'inv_hTh', self.config.desired_inv_hTh_energy_portion)
        if drop > 0:
            self.inv_hTh = inv[drop:-drop, drop:-drop]

    # ---- NumPy image helpers (CEMnet.py:44-57, 88-100), computed on the device --------------------------------------
    def Pad_LR_Batch(self, batch, num_recursion=1):
        """CEMnet.py:44-47: NHWC batch edge-padded by the LR invalidity margin, num_recursion times (host data
        movement; returns float64 like the reference's 1.0*np.pad)."""
        m = int(self.invalidity_margins_LR)
        for _ in range(num_recursion):
            batch = 1.0 * np.pad(batch, pad_width=((0, 0), (m, m), (m, m), (0, 0)), mode='edge')
        return batch

    def Unpad_HR_Batch(self, batch, num_recursion=1):
        """CEMnet.py:49-51 (Python slice semantics kept: too large a margin gives an empty batch)."""
        r = int(self.ds_factor) ** num_recursion * int(self.invalidity_margins_LR) * num_recursion
        return batch[:, r:-r, r:-r, :]

    def _filters(self, device):
        """Device float32 filters of the helpers: k_up/sf² (downscale), rot180(k_up) (upscale), rot180(inv_hTh)
        (scipy conv2 is a flipped cross-correlation)."""
        key = str(device)
        if key not in self._dev_filters:
            sf = int(self.ds_factor)
            f = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(device)  # noqa: E731
            self._dev_filters[key] = dict(down=f(self._k_up / sf ** 2), up=f(np.rot90(self._k_up, 2)),
                                          inv=f(np.rot90(self.inv_hTh, 2)))
        return self._dev_filters[key]

    def _dt_upscale(self, x):
        sf = int(self.ds_factor)
        m = int(2 * self.inv_hTh_invalidity_half_size + self.ds_kernel_invalidity_half_size_LR)
        f = self._filters(x.device)
        H, W = x.shape[-2:]
        xp = F.pad(x.reshape(-1, 1, H, W), (m, m, m, m), mode='replicate').view(*x.shape[:-2], H + 2 * m, W + 2 * m)
        return cem_ops.upscale(cem_ops.filter_same(xp, f['inv']), f['up'], sf, crop=sf * m)

    def _project(self, x):
        return self._dt_upscale(cem_ops.downscale(x, self._filters(x.device)['down'], int(self.ds_factor)))

    def DT_Satisfying_Upscale(self, LR_image):
        """CEMnet.py:53-57: edge-pad by 2*inv_half + ds_half, 'same' zero-padded convolution with inv_hTh, imresize
        ×sf, unpad — the upscale whose downscale reproduces LR_image (HWC NumPy, or a device tensor [..., h, w])."""
        x, back = _to_device(LR_image, None)
        return back(self._dt_upscale(x))

    def Project_2_kernel_subspace(self, HR_input):
        """CEMnet.py:98-100: downscale (imresize 1/sf, edge padding) then DT_Satisfying_Upscale."""
        x, back = _to_device(HR_input, None)
        return back(self._project(x))

    def Enforce_DT_on_Image_Pair(self, LR_source, HR_input):
        """CEMnet.py:88-96: HR_input - Project(HR_input) + (DT_Satisfying_Upscale(LR_source) if LR_source is LR-sized
        else Project(LR_source)).  Used by GUI.py:951,1105 and test.py:218."""
        sf = int(self.ds_factor)
        same = [a == b for a, b in zip(LR_source.shape, HR_input.shape)]
        lr_scale = [sf * a == b for a, b in zip(LR_source.shape, HR_input.shape)]
        assert np.all(np.logical_or(same, lr_scale))
        lr, _ = _to_device(LR_source, None)
        hr, back = _to_device(HR_input, None)
        lr = lr.to(hr.device)
        src = self._dt_upscale(lr) if np.any(lr_scale) else self._project(lr)
        return back(hr - self._project(hr) + src)

    def WrapArchitecture_PyTorch(self, generated_image=None, training_patch_size=None, only_padders=False):
        """CEMnet.py:59-81."""
        mL = int(self.invalidity_margins_LR)
        mH = int(self.ds_factor) * mL
        self.LR_padder = nn.ReplicationPad2d((mL, mL, mL, mL))
        self.HR_padder = nn.ReplicationPad2d((mH, mH, mH, mH))
        self.HR_unpadder = lambda x: x[:, :, mH:-mH, mH:-mH]
        self.LR_unpadder = lambda x: x[:, :, mL:-mL, mL:-mL]
        self.loss_mask = None
        self.training_patch_size = training_patch_size
        if training_patch_size is not None:
            mask = np.zeros([1, 1, training_patch_size, training_patch_size])
            M = int(self.invalidity_margins_HR)
            mask[:, :, M:-M, M:-M] = 1
            assert np.mean(mask) > 0, 'Loss mask completely nullifies image.'
            self.loss_mask = torch.from_numpy(mask).float()
        if only_padders:
            return
        module = CEM_PyTorch(self, generated_image)
        self.OP_names = [m[0] for m in module.named_modules() if 'Filter_OP' in m[0]]
        return module

    def Mask_Invalid_Regions_PyTorch(self, im1, im2):
        assert self.loss_mask is not None, 'Mask not defined, probably didn''t pass patch size'
        mask = self.loss_mask.to(im1.device)
        return mask * im1, mask * im2


class Filter_Layer(nn.Module):
    """CEMnet.py:130-140: frozen depthwise conv.  Forward runs the matching libesr_amd stencil."""

    def __init__(self, filt, kind, sf=4):
        super().__init__()
        self.sf = int(sf)  # the CEM's scale factor (stride of 'down', zero-stuffing of 'up')
        k = np.asarray(filt)
        self.Filter_OP = nn.Conv2d(in_channels=3, out_channels=3, kernel_size=k.shape, bias=False, groups=3)
        self.Filter_OP.weight = nn.Parameter(
            data=torch.from_numpy(np.tile(k[None, None], reps=[3, 1, 1, 1])).float(), requires_grad=False)
        self.Filter_OP.filter_layer = True
        self.kind = kind  # 'inv' | 'up' | 'down'

    def forward(self, x):
        return engine.cem_filter_op(self, x)


class CEM_PyTorch(nn.Module):
    """CEMnet.py:142-194.  forward = generator on the (pre-padded) input + back-projection onto the LR-consistent
    affine subspace; `train(mode)` toggles pre-padding (eval pads, train does not)."""

    def __init__(self, CEMnet, generated_image):
        super().__init__()
        self.ds_factor = CEMnet.ds_factor
        self.config = CEMnet.config
        self.generated_image_model = generated_image
        self._set_filters(CEMnet)
        self.LR_padder = CEMnet.LR_padder
        self.HR_padder = CEMnet.HR_padder
        self.HR_unpadder = CEMnet.HR_unpadder
        self.LR_unpadder = CEMnet.LR_unpadder
        self.pre_pad = False

    def _set_filters(self, CEMnet):
        sf = int(CEMnet.ds_factor)
        self.Conv_LR_with_Inv_hTh_OP = Filter_Layer(CEMnet.inv_hTh, 'inv', sf)
        self.Upscale_OP = Filter_Layer(CEMnet.ds_kernel * CEMnet.ds_factor ** 2, 'up', sf)
        self.DownscaleOP = Filter_Layer(np.rot90(CEMnet.ds_kernel, 2), 'down', sf)
        self.margins_LR = int(CEMnet.invalidity_margins_LR)
        self.margins_HR = int(CEMnet.invalidity_margins_HR)

    def Update_Filters(self, CEMnet):
        """Swap in the filters and margins of a re-designed CEMnet (CEMnet.Set_Upscale_Kernel) without rebuilding the
        generator: per-image kernels (test.py:143-148) at the cost of the design only.  The padders/unpadders are
        rebuilt for the new margins (and the loss mask for the last training patch size); the plan cache keys on the filter storage, so the next forward replans."""
        dev = self.DownscaleOP.Filter_OP.weight.device
        self._set_filters(CEMnet)
        for m in (self.Conv_LR_with_Inv_hTh_OP, self.Upscale_OP, self.DownscaleOP):
            m.to(dev)
        CEMnet.WrapArchitecture_PyTorch(training_patch_size=getattr(CEMnet, 'training_patch_size', None),
                                        only_padders=True)
        self.LR_padder, self.HR_padder = CEMnet.LR_padder, CEMnet.HR_padder
        self.HR_unpadder, self.LR_unpadder = CEMnet.HR_unpadder, CEMnet.LR_unpadder
        return self

    def forward(self, x):
        return engine.generator_forward(self.generated_image_model, x, cem=self)

    def train(self, mode=True):
        super().train(mode=mode)
        self.pre_pad = not mode
        return self


def upscale_kernel_of(sf, kernel):
    return upscale_kernel(sf, kernel)


def Return_kernel(ds_factor, upscale_kernel):
    """CEMnet.py:218-219: the DOWNSCALE kernel = rot180(upscale kernel) / sf² (float32 cast, then float64 under
    NumPy 2 promotion, exactly as the reference)."""
    return np.rot90(upscale_kernel, 2).astype(np.float32) / (np.asarray(ds_factor, dtype=np.int32) ** 2)


def Get_CEM_Config(sf):
    class config:
        scale_factor = sf
        desired_inv_hTh_energy_portion = 1 - 1e-6
        filter_pertubation_limit = 0.999
        lower_magnitude_bound = 0.01
    return config


def Adjust_State_Dict_Keys(loaded_state_dict, current_state_dict):
    """CEMnet.py:235-245: prefix a non-CEM checkpoint's keys with 'generated_image_model.' and keep the current CEM
    filters."""
    if all(('generated_image_model' in k or 'Filter' in k) for k in current_state_dict.keys()) and \
            not any('generated_image_model' in k for k in loaded_state_dict.keys()):
        out = collections.OrderedDict()
        for k in loaded_state_dict:
            out['generated_image_model.' + k] = loaded_state_dict[k]
        for k in [k for k in current_state_dict.keys() if 'Filter' in k]:
            out[k] = current_state_dict[k]
        return out
    return loaded_state_dict
