"""State hazards of the cached executors: recorded inference op lists must survive the training
path swapping the x3 weight tensors, and a second grad-enabled forward before the first one's backward must not
overwrite the first forward's saved activations."""
import pytest
import torch

from conftest import fixture_input, fixture_params, golden

import esr_amd
from esr_amd import CEMnet as C

pytestmark = pytest.mark.gpu


def _model(params, dev, nb=1):
    net = esr_amd.RRDBNet(3, 3, 64, nb, num_latent_channels=0)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    return model.to(dev)


def test_recorded_inference_survives_training_forward(gpu_device):
    """inference (records the op list) -> grad forward + backward with G unchanged (train_x3 swaps each layer's x3
    weights for its persistent training views; no optimiser step, so the plan key is unchanged) -> the freed blocks
    are reallocated and poisoned -> inference replays the recorded list: bitwise equal to the first inference and to a
    fresh model's eager output."""
    d = golden('grad_plain_nb1')
    _, params = fixture_params(d)
    x = fixture_input(d).to(gpu_device)
    model = _model(params, gpu_device).eval()
    with torch.no_grad():
        first = model(x).clone()
        again = model(x).clone()
    assert torch.equal(first, again)
    model.train()
    (model(x) * torch.from_numpy(d['R']).to(gpu_device)).sum().backward()
    model.eval()
    poison = [torch.full((1 << k,), float('nan'), device=gpu_device, dtype=torch.float16) for k in range(8, 22)
              for _ in range(4)]
    with torch.no_grad():
        replay = model(x).clone()
    del poison
    assert torch.equal(replay, first)
    fresh = _model(params, gpu_device).eval()
    with torch.no_grad():
        assert torch.equal(fresh(x), first)


def test_second_grad_forward_keeps_first_activations(gpu_device):
    """Two generator calls inside one loss (y1 from x1, y2 from x2, then one backward through both): each call must
    back-propagate through its own saved activations; the summed gradients equal the sum of two separate steps."""
    d = golden('grad_plain_nb1')
    _, params = fixture_params(d)
    x1 = fixture_input(d).to(gpu_device)
    x2 = torch.flip(x1, dims=[3]).contiguous()
    R = torch.from_numpy(d['R']).to(gpu_device)

    def grads(xs):
        model = _model(params, gpu_device).train()
        loss = sum((model(x) * R).sum() for x in xs)
        loss.backward()
        return [p.grad.clone() for p in model.parameters() if p.requires_grad]

    both = grads([x1, x2])
    g1, g2 = grads([x1]), grads([x2])
    for b, a1, a2 in zip(both, g1, g2):
        ref = a1 + a2
        assert float((b - ref).norm() / ref.norm().clamp_min(1e-30)) < 1e-5


def test_retained_graph_second_backward_raises_after_reuse(gpu_device):
    """A forward whose workspace was handed to a later forward after its backward ran: a second backward through the
    retained graph would read the later forward's activations, so it raises instead of returning wrong gradients."""
    d = golden('grad_plain_nb1')
    _, params = fixture_params(d)
    x = fixture_input(d).to(gpu_device)
    model = _model(params, gpu_device).train()
    y = model(x)
    y.sum().backward(retain_graph=True)
    model(torch.flip(x, dims=[2]).contiguous()).sum().backward()
    with pytest.raises(RuntimeError, match='overwritten'):
        y.sum().backward()


def test_activation_scale_ratchet(gpu_device):
    """engine.lower_act_scale: an x3 forward whose scaled activations leave f16's range is redone in
    exact fp32 (bitwise the f32 output), the model's activation scale A drops 16× and the reduction is counted and
    warned about; A stays lowered for later in-range forwards (a deliberate one-way ratchet), which still run x3."""
    from esr_amd import engine
    d = golden('grad_plain_nb1')
    _, params = fixture_params(d)
    x = fixture_input(d).to(gpu_device)
    model = _model(params, gpu_device).eval()
    ref = _model(params, gpu_device).eval()
    engine.set_precision(ref, 'f32')
    rrdb = model.generated_image_model
    assert engine.act_scale(rrdb) == engine.ACT_SCALE
    red0, rer0 = engine.ACT_SCALE_REDUCTIONS, engine.OVERFLOW_RERUNS
    with torch.no_grad(), pytest.warns(RuntimeWarning, match='activation scale'):
        big = model(x * 3e5)
    assert engine.OVERFLOW_RERUNS == rer0 + 1 and engine.ACT_SCALE_REDUCTIONS == red0 + 1
    assert engine.act_scale(rrdb) == engine.ACT_SCALE / 16
    with torch.no_grad():
        assert torch.equal(big, ref(x * 3e5))
        small = model(x)
        exact = ref(x)
    assert engine.act_scale(rrdb) == engine.ACT_SCALE / 16  # not raised again
    assert engine.OVERFLOW_RERUNS == rer0 + 1
    err = float((small - exact).abs().max() / exact.abs().max())
    assert 0 < err < 1e-5, err  # x3 (not bitwise the fp32 path), fp32-level accuracy


def test_lagged_overflow_check_returns_exact_fp32_output(gpu_device):
    """engine.lagged_overflow_checks(): forward N's x3 overflow flag is read only after forward N + 1 is enqueued; an
    overflowed N (inputs × 3e5 leave the f16 range) still returns N's exact-fp32 output — recomputed into the tensor N
    returned — and N + 1 (enqueued before N was found to overflow, at the old activation scale) its own x3 output;
    each bitwise equal to a fresh model's forward of the same input with the same precision and scale."""
    from esr_amd import engine
    d = golden('grad_plain_nb1')
    _, params = fixture_params(d)
    x_ok = fixture_input(d).to(gpu_device)
    x_big = (x_ok * 3e5).contiguous()
    with torch.no_grad():
        ref_ok = _model(params, gpu_device).eval()(x_ok).clone()  # x3 at the default activation scale
        f32 = _model(params, gpu_device).eval()
        engine.set_precision(f32, 'f32')
        ref_big = f32(x_big).clone()
        model = _model(params, gpu_device).eval()
        before = engine.OVERFLOW_RERUNS
        with engine.lagged_overflow_checks():
            o_big = model(x_big)
            o_ok = model(x_ok)
            o_big2 = model(x_big)  # (at the lowered scale: overflows again, redone at the block's end)
    assert engine.OVERFLOW_RERUNS == before + 2
    assert torch.equal(o_big, ref_big) and torch.equal(o_big2, ref_big)
    assert torch.equal(o_ok, ref_ok)
