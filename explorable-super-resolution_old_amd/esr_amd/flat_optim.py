"""Adam over one flat parameter buffer: the generator's optimiser (SRRaGAN_model.py:196-198 builds
`torch.optim.Adam(optim_params, lr, weight_decay, betas)` over RRDB-23's 702 parameter tensors).

Per element the update is the reference's: torch's Adam applies the same elementwise ops with the same per-tensor
scalars to every tensor (exp_avg.lerp_, exp_avg_sq.mul_().addcmul_(), sqrt / bias-correction / eps, addcdiv_), so
running them once over a buffer that holds all parameters back to back gives bit-identical parameters and moments —
without the host cost of 702-tensor lists (≈5 ms per step at config 3; `Adam(fused=True)` is faster still but
computes the bias corrections on the device in fp32, which is not the reference's update).

The parameters become views of `flat` and their `.grad` views of `flat.grad`, so everything that reads or writes
them per tensor (autograd accumulation, the latent-channel gradient amplification, checkpoints, load_state_dict)
keeps working.  `zero_grad()` zeroes the flat gradient.  torch's Adam skips a parameter whose .grad is None (and
keeps a step count per parameter); here every .grad is a view, so step() raises if a parameter does not require grad
(how a parameter is left out of a backward) instead of updating it with a zero gradient.  In the training step every
generator / discriminator parameter is in every backward.
`state_dict()` / `load_state_dict()` use the per-parameter format of torch.optim.Adam, i.e. the reference's
checkpoint layout (base_model.py:86-111)."""
import torch

_MOMENTS = ('exp_avg', 'exp_avg_sq', 'max_exp_avg_sq')


class FlatAdam(torch.optim.Adam):
    def __init__(self, params, **kw):
        self.flat_params = list(params)
        if not self.flat_params:
            raise ValueError('FlatAdam: no parameters')
        p0 = self.flat_params[0]
        if any(p.dtype != p0.dtype or p.device != p0.device for p in self.flat_params):
            raise ValueError('FlatAdam: parameters of one dtype on one device')
        n = sum(p.numel() for p in self.flat_params)
        data = torch.empty(n, device=p0.device, dtype=p0.dtype)
        o = 0
        for p in self.flat_params:
            data[o:o + p.numel()].copy_(p.detach().reshape(-1))
            o += p.numel()
        self.flat = torch.nn.Parameter(data)
        self.flat.grad = torch.zeros_like(data)
        self._bind()
        super().__init__([self.flat], **kw)

    def _bind(self):
        o = 0
        for p in self.flat_params:
            k = p.numel()
            p.data = self.flat.data[o:o + k].view_as(p)
            p.grad = self.flat.grad[o:o + k].view_as(p)
            p._esr_flat = self.flat  # engine._param_key: an in-place update of `flat` changes every parameter
            o += k
        self._ptrs = [(p.data_ptr(), p.grad.data_ptr()) for p in self.flat_params]

    def _sync_views(self):
        """Re-attach parameters / gradients that were replaced since the last bind (p.data = t, p.grad = None or a
        new tensor), copying their current values into the flat buffers first."""
        o, rebind = 0, False
        with torch.no_grad():
            for p, (dp, gp) in zip(self.flat_params, self._ptrs):
                k = p.numel()
                if p.data_ptr() != dp:
                    self.flat.data[o:o + k].copy_(p.detach().reshape(-1))
                    rebind = True
                g = p.grad
                if g is None:
                    self.flat.grad[o:o + k].zero_()
                    rebind = True
                elif g.data_ptr() != gp:
                    self.flat.grad[o:o + k].copy_(g.reshape(-1))
                    rebind = True
                o += k
        if rebind:
            self._bind()

    def accepts_flat_grad(self, params):
        """True if `params` (in order) are exactly this optimiser's parameters: a backward that produces their
        gradients as one buffer in that layout may add it to `flat.grad` directly (train_engine)."""
        return len(params) == len(self.flat_params) and all(a is b for a, b in zip(params, self.flat_params))

    def zero_grad(self, set_to_none=True):
        self._sync_views()
        self.flat.grad.zero_()

    @torch.no_grad()
    def step(self, closure=None):
        # a .grad set to None from outside (module.zero_grad(set_to_none=True)) and not refilled by a backward: torch's
        # Adam would skip that parameter, a flat update would move it by its moments with a zero gradient
        missing = [i for i, p in enumerate(self.flat_params) if p.grad is None]
        if missing:
            raise RuntimeError('FlatAdam.step: parameters %s have no gradient (torch.optim.Adam would skip them); '
                               'run their backward or use a per-tensor optimiser' % missing[:8])
        self._sync_views()
        frozen = [i for i, p in enumerate(self.flat_params) if not p.requires_grad]
        if frozen:
            # torch's Adam would skip these (grad None) and keep a per-parameter step count; one flat update cannot
            raise RuntimeError('FlatAdam.step: parameters %s do not require grad (they would be skipped by '
                               'torch.optim.Adam); unfreeze them or use a per-tensor optimiser' % frozen[:8])
        return super().step(closure)

    def state_dict(self):
        sd = super().state_dict()
        group = dict(sd['param_groups'][0])
        group['params'] = list(range(len(self.flat_params)))
        st = sd['state'].get(0)
        state = {}
        if st:
            o = 0
            for i, p in enumerate(self.flat_params):
                k = p.numel()
                e = {'step': st['step'].clone()}
                for key in _MOMENTS:
                    if key in st:
                        e[key] = st[key][o:o + k].view_as(p).clone()
                state[i] = e
                o += k
        return {'state': state, 'param_groups': [group]}

    def load_state_dict(self, state_dict):
        groups = state_dict['param_groups']
        if len(groups) != 1 or len(groups[0]['params']) != len(self.flat_params):
            raise ValueError('FlatAdam.load_state_dict: expected one group of %d parameters' % len(self.flat_params))
        ids = list(groups[0]['params'])
        st = state_dict['state']
        flat_sd = {'param_groups': [dict(groups[0], params=[0])], 'state': {}}
        have = [i in st for i in ids]
        if any(have):
            if not all(have):
                raise ValueError('FlatAdam.load_state_dict: state for only some parameters')
            steps = {float(st[i]['step']) for i in ids}
            if len(steps) != 1:
                raise ValueError('FlatAdam.load_state_dict: parameters at different steps')
            e = {'step': torch.as_tensor(st[ids[0]]['step']).clone()}
            for key in _MOMENTS:
                if key in st[ids[0]]:
                    e[key] = torch.cat([st[i][key].reshape(-1) for i in ids])
            flat_sd['state'][0] = e
        super().load_state_dict(flat_sd)
