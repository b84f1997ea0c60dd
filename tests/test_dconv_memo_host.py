"""Host logic of the discriminator's conv0 im2col adjoint and of its packed-weight memo (esr_amd/dconv.py _packed):
a memo hit while the parameter is unchanged, a rebuild after every kind of change a training run makes (optimiser
step, FlatAdam step on the shared buffer, load_state_dict, a .data swap), and no memo for tensors that are not marked
discriminator parameters."""
import torch

from esr_amd import dconv
from esr_amd.flat_optim import FlatAdam


def _counting():
    calls = []

    def make(w):
        def f():
            calls.append(1)
            return (w.detach().clone(), 1, 64)
        return f
    return calls, make


def test_memo_hits_until_the_parameter_changes():
    calls, make = _counting()
    conv = torch.nn.Conv2d(4, 8, 3)
    w = conv.weight
    w._esr_dconv_param = True
    a = dconv._packed(w, ('fwd',), make(w))
    b = dconv._packed(w, ('fwd',), make(w))
    assert len(calls) == 1 and a is b
    dconv._packed(w, ('dgrad', 1, 1, 0, 0), make(w))  # another key: its own entry
    assert len(calls) == 2
    w.grad = torch.ones_like(w)
    torch.optim.Adam([w], lr=0.1).step()  # in place: version bump
    c = dconv._packed(w, ('fwd',), make(w))
    assert len(calls) == 3 and torch.equal(c[0], w.detach())
    conv.load_state_dict({'weight': torch.zeros_like(w), 'bias': conv.bias.detach()})
    d = dconv._packed(w, ('fwd',), make(w))
    assert len(calls) == 4 and not d[0].any()
    w.data = torch.randn_like(w)  # new storage, same version counter
    e = dconv._packed(w, ('fwd',), make(w))
    assert len(calls) == 5 and torch.equal(e[0], w.detach())


def test_memo_follows_a_flat_adam_step():
    calls, make = _counting()
    conv = torch.nn.Conv2d(4, 8, 3)
    conv.weight._esr_dconv_param = True
    opt = FlatAdam(list(conv.parameters()), lr=0.1)
    w = conv.weight
    dconv._packed(w, ('fwd',), make(w))
    v = w._version
    conv(torch.randn(1, 4, 5, 5)).sum().backward()
    opt.step()  # updates the shared buffer: w's own version counter does not move
    assert w._version == v
    p = dconv._packed(w, ('fwd',), make(w))
    assert len(calls) == 2 and torch.equal(p[0], w.detach())


def test_unmarked_tensors_are_not_memoised():
    calls, make = _counting()
    g = torch.randn(8, 4, 3, 3)  # e.g. a weight-gradient tensor used as weights in the double backward
    dconv._packed(g, ('fwd',), make(g))
    dconv._packed(g, ('fwd',), make(g))
    assert len(calls) == 2 and not hasattr(g, '_esr_packs')


def presplit_reference(wp):
    """The layout of include/esr_amd.h esr_dconv_fwd_sd w_split / w_exp restated with PyTorch ops (test reference for
    esr_dconv_presplit): v = wp·2^E, E = 14 - floor(log2 max|wp|), hi = f16(v), lo = f16(v - hi), each 128-byte
    (t, chunk, n) row's logical 16-B slot piece·4 + k stored at position ^ ((n >> 1) & 7)."""
    import torch
    T, nck, n_pad, _ = wp.shape
    amax = wp.abs().amax()
    E = torch.where(amax > 0, 14.0 - torch.floor(torch.log2(amax)), torch.zeros_like(amax))
    v = wp * torch.exp2(E)
    hi = v.half()
    lo = (v - hi.float()).half()
    logical = torch.stack([hi, lo], 3).view(T, nck, n_pad, 8, 8)
    n = torch.arange(n_pad, device=wp.device)
    idx = torch.arange(8, device=wp.device).view(1, 8) ^ ((n.view(-1, 1) >> 1) & 7)
    rows = torch.gather(logical, 3, idx.view(1, 1, n_pad, 8, 1).expand(T, nck, n_pad, 8, 8))
    return rows, E.to(torch.int32).view(1)


def test_presplit_weight_layout():
    """The reference restatement of the pre-split layout: hi + lo = w·2^E to f16-pair accuracy, max |w|·2^E in
    [2^14, 2^15), hi exact f16 rounding; tests/test_gpu_disc.py checks esr_dconv_presplit against it bitwise."""
    import torch
    g = torch.Generator().manual_seed(3)
    wt = torch.randn(9, 70, 100, generator=g) * 0.03
    wp, nck, n_pad = dconv._pack(wt, 100)
    rows, e = presplit_reference(wp)
    E = int(e.item())
    assert 2 ** 14 <= float(wp.abs().max()) * 2 ** E < 2 ** 15
    assert rows.dtype == torch.float16 and rows.shape == (9, nck, n_pad, 8, 8)
    n = torch.arange(n_pad)
    idx = torch.arange(8).view(1, 8) ^ ((n.view(-1, 1) >> 1) & 7)   # position p holds logical slot idx[n, p]
    logical = torch.empty_like(rows)
    logical.scatter_(3, idx.view(1, 1, n_pad, 8, 1).expand_as(rows), rows)
    hi = logical[..., 0:4, :].reshape(9, nck, n_pad, 32).float()
    lo = logical[..., 4:8, :].reshape(9, nck, n_pad, 32).float()
    v = wp * 2.0 ** E
    assert torch.equal(hi, v.half().float())
    assert float((hi + lo - v).abs().max()) <= 2.0 ** -9  # (|v| < 2^15: the pair carries ~22 bits)
