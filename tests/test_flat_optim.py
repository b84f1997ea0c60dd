"""FlatAdam (esr_amd/flat_optim.py): the generator's Adam over one flat buffer is bit-identical to torch.optim.Adam
over the individual parameter tensors (the reference's optimiser, SRRaGAN_model.py:196-198), and its state_dict is
the per-parameter checkpoint format (base_model.py:86-111)."""
import torch

from esr_amd.flat_optim import FlatAdam


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 3, 3, 3), (64,), (32, 64, 3, 3), (32,), (3, 64, 3, 3), (3,)]
    return [torch.nn.Parameter(torch.randn(s, generator=g) * 0.1) for s in shapes]


def _run(opt_cls, params, steps, foreach, **kw):
    opt = opt_cls(params, lr=1e-3, betas=(0.9, 0.999), foreach=foreach, **kw)
    g = torch.Generator().manual_seed(5)
    for _ in range(steps):
        opt.zero_grad()
        for _acc in range(2):  # gradient accumulation: the second micro-step adds into .grad
            for p in params:
                gr = torch.randn(p.shape, generator=g) * 1e-3
                if p.grad is None:
                    p.grad = gr
                else:
                    p.grad += gr
        opt.step()
    return opt


def test_flat_adam_bitwise_equals_per_tensor_adam():
    for wd in (0.0, 1e-4):
        for foreach in (False, True):
            a, b = _params(1), _params(1)
            oa = _run(torch.optim.Adam, a, 5, foreach, weight_decay=wd)
            ob = _run(FlatAdam, b, 5, foreach, weight_decay=wd)
            for pa, pb in zip(a, b):
                assert torch.equal(pa.detach(), pb.detach())
            sa, sb = oa.state_dict(), ob.state_dict()
            assert set(sa['param_groups'][0]) == set(sb['param_groups'][0])
            assert sa['param_groups'][0]['params'] == sb['param_groups'][0]['params']
            for i in sa['state']:
                assert list(sa['state'][i]) == list(sb['state'][i])
                for k in sa['state'][i]:
                    assert torch.equal(sa['state'][i][k], sb['state'][i][k]), (i, k)


def test_flat_adam_loads_per_tensor_state_and_continues_identically():
    a, b = _params(2), _params(2)
    oa = _run(torch.optim.Adam, a, 3, False)
    ob = FlatAdam(b, lr=1e-3, foreach=False)
    with torch.no_grad():
        for pa, pb in zip(a, b):
            pb.copy_(pa)
    ob.load_state_dict(oa.state_dict())
    g = torch.Generator().manual_seed(9)
    for _ in range(2):
        oa.zero_grad()
        ob.zero_grad()
        for pa, pb in zip(a, b):
            gr = torch.randn(pa.shape, generator=g)
            pa.grad = gr.clone()
            pb.grad.copy_(gr)
        oa.step()
        ob.step()
    for pa, pb in zip(a, b):
        assert torch.equal(pa.detach(), pb.detach())


def test_flat_adam_reattaches_replaced_tensors():
    """A parameter whose storage was replaced (p.data = t) or whose gradient was set to a new tensor is copied back
    into the flat buffers before the step."""
    a, b = _params(3), _params(3)
    oa = torch.optim.Adam(a, lr=1e-2, foreach=False)
    ob = FlatAdam(b, lr=1e-2, foreach=False)
    b[2].data = b[2].detach().clone() * 2
    with torch.no_grad():
        a[2].mul_(2)
    for pa, pb in zip(a, b):
        pa.grad = torch.full_like(pa, 0.5)
        pb.grad = torch.full_like(pb, 0.5)
    oa.step()
    ob.step()
    for pa, pb in zip(a, b):
        assert torch.equal(pa.detach(), pb.detach())
    assert b[2].data_ptr() == ob.flat.data_ptr() + 4 * sum(p.numel() for p in b[:2])


def test_flat_adam_refuses_a_frozen_parameter():
    """torch.optim.Adam skips a parameter that got no gradient; FlatAdam cannot, so it raises instead of moving it."""
    import pytest
    ps = _params(3)
    opt = FlatAdam(ps, lr=1e-3)
    opt.zero_grad()
    ps[1].requires_grad_(False)
    with pytest.raises(RuntimeError, match='do not require grad'):
        opt.step()
    ps[1].requires_grad_(True)
    opt.step()


def test_flat_adam_refuses_a_missing_gradient():
    """A gradient set to None (module.zero_grad(set_to_none=True)) and not refilled: torch's Adam would skip the
    parameter, so FlatAdam raises instead of moving it with a zero gradient; after a backward it steps again."""
    import pytest
    ps = _params(3)
    opt = FlatAdam(ps, lr=1e-3)
    opt.zero_grad()
    ps[2].grad = None
    with pytest.raises(RuntimeError, match='no gradient'):
        opt.step()
    sum((p * p).sum() for p in ps).backward()
    opt.step()
