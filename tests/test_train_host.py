"""CPU tests of the training-step host side: discriminator layout + forward/GP/range losses vs the reference's golden
vector, and the multi-process (gloo, world size 2) gradient / statistics reductions of SRRaGANModel."""
import json
import copy
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import golden, normwise_rel

from esr_amd.discriminator import Discriminator_VGG_128_
from esr_amd import loss as L
from esr_amd import SRRaGAN_model as M
from esr_amd.flat_optim import FlatAdam
from oracle.recipe import seeded_params


def _disc_from_fixture(d, D=None):
    """The fixture's seeded parameters loaded into D (default: the oracle's torch.nn restatement, CPU)."""
    if D is None:
        from oracle.esr_oracle import reference_discriminator
        D = reference_discriminator(nb=6)
    ref_keys = json.loads(str(d['keys']))
    assert [(k, list(v.shape)) for k, v in D.state_dict().items()] == [(k, list(s)) for k, s in ref_keys]
    params = seeded_params([(k, s) for k, s in ref_keys if 'running' not in k and 'num_batches' not in k],
                           int(d['seed']), w_scale=1.0)
    D.load_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
    return D.train()


def test_discriminator_and_wgan_gp_losses_match_reference():
    # the fixture ran with 8 CPU threads; another count changes the order of oneDNN's fp32 reductions, which the
    # WGAN-GP term (a gradient norm through 10 conv layers) amplifies to a few 1e-6
    torch.set_num_threads(8)
    d = golden('disc_vgg128_nb6')
    D = _disc_from_fixture(d)
    real, fake, rp = (torch.from_numpy(d[k]) for k in ('real', 'fake', 'rp'))
    cri_gan, cri_gp = L.GANLoss('wgan-gp'), L.GradientPenaltyLoss()
    pred_real, pred_fake = D(real), D(fake)
    assert normwise_rel(pred_real.detach(), d['pred_real']) < 1e-5
    assert normwise_rel(pred_fake.detach(), d['pred_fake']) < 1e-5
    l_d_real, l_d_fake = 2 * cri_gan(pred_real, True), 2 * cri_gan(pred_fake, False)
    interp = rp * fake + (1 - rp) * real
    interp.requires_grad = True
    l_d_gp = 10 * cri_gp(interp, D(interp))
    l_d_total = (l_d_real + l_d_fake) / 2 + l_d_gp
    l_d_total.backward()
    for k in ('l_d_real', 'l_d_fake', 'l_d_gp', 'l_d_total'):
        assert abs(float(locals()[k]) - float(d[k])) <= 2e-5 * max(1.0, abs(float(d[k]))), k
    for k, p in D.named_parameters():
        assert normwise_rel(p.grad, d['grad:' + k]) < 1e-4, k
    for k, v in D.state_dict().items():
        if 'running' in k:
            assert normwise_rel(v, d['buf:' + k]) < 1e-5, k


def test_hip_discriminator_module_tree_and_no_cpu_path():
    """esr_amd's Discriminator_VGG_128_ keeps the reference's state_dict keys/shapes/order (positional checkpoint
    loading, base_model.py:117-141) with HipConv2d convolutions, and refuses CPU tensors (no silent fallback)."""
    d = golden('disc_vgg128_nb6')
    D = Discriminator_VGG_128_(in_nc=3, base_nf=64, norm_type='batch', act_type='leakyrelu', mode='CNA',
                               input_patch_size=80, nb=6)
    ref_keys = json.loads(str(d['keys']))
    assert [(k, list(v.shape)) for k, v in D.state_dict().items()] == [(k, list(s)) for k, s in ref_keys]
    convs = [m for m in D.modules() if isinstance(m, torch.nn.Conv2d)]
    assert len(convs) == 8 and all(type(m).__name__ == 'HipConv2d' for m in convs)
    with pytest.raises(RuntimeError, match='no CPU path'):
        D(torch.zeros(1, 3, 80, 80))


def test_range_loss_matches_reference():
    d = golden('disc_vgg128_nb6')
    rng = np.random.default_rng(int(d['range_seed']))
    for name in ('real', 'fake', 'rp'):  # advance the stream exactly as the generator did
        rng.random(d[name].shape)
    x = torch.from_numpy((rng.random((2, 3, 8, 8)) * 1.6 - 0.3).astype(np.float32))
    assert abs(float(L.CreateRangeLoss([0, 1])(x)) - float(d['range_loss'])) < 1e-7


def _dist_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.manual_seed(rank)
        p = [torch.nn.Parameter(torch.zeros(3, 4)), torch.nn.Parameter(torch.zeros(5))]
        p[0].grad = torch.full((3, 4), float(rank + 1))
        p[1].grad = torch.arange(5, dtype=torch.float32) * (rank + 1)
        M._allreduce_grads(p)
        m = M.SRRaGANModel.__new__(M.SRRaGANModel)
        pred_real = torch.full((2, 1, 3, 3), 1.0 + rank)          # per-image diffs: rank 0: (+1,+1)
        pred_fake = torch.tensor([0.0, 3.0 + rank]).view(2, 1, 1, 1).expand(2, 1, 3, 3)  # rank 1: (+2,-2)
        diff, correct, d_real, d_fake = m._d_statistics(pred_real, pred_fake)
        # bucketed all-reduce launched from inside the backward (several buckets), against a flat average
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 16), torch.nn.ReLU(),
                                  torch.nn.Linear(16, 4))
        ref_net = copy.deepcopy(net)
        x = torch.randn(5, 8, generator=torch.Generator().manual_seed(10 + rank))
        buckets = M.GradBuckets(list(net.parameters()), cap_bytes=600)
        buckets.arm()
        net(x).square().sum().backward()
        launched = buckets.launched_in_backward
        buckets.finish()
        cs = buckets.comm_stats()
        comm = (cs['allreduces'] == len(buckets.buckets),
                cs['allreduce_bytes'] == sum(p_.numel() * 4 for p_ in net.parameters()))
        ref_net(x).square().sum().backward()
        M._allreduce_grads(list(ref_net.parameters()))
        same = all(torch.allclose(a.grad, b.grad, rtol=1e-6, atol=1e-7) for a, b in zip(net.parameters(),
                                                                                         ref_net.parameters()))
        # an unarmed backward (not the last accumulation micro-step) leaves the local gradients alone
        net.zero_grad()
        net(x).square().sum().backward()
        local = [q_.grad.clone() for q_ in net.parameters()]
        buckets.finish()
        untouched = all(torch.equal(a, q_.grad) for a, q_ in zip(local, net.parameters()))
        # BatchNorm running buffers: rank 0's everywhere
        bn = torch.nn.BatchNorm2d(3)
        bn.running_mean.fill_(rank + 1.0)
        bn.num_batches_tracked.fill_(7 * (rank + 1))
        M._broadcast_buffers(bn)
        bufs = (float(bn.running_mean[0]), int(bn.num_batches_tracked))
        # generator_step gating on ranks whose LOCAL D statistics disagree: rank 0's two images are both classified
        # correctly (a local 'current' check would pass), rank 1 has one wrong; the global batch has 3 of 4 correct
        g = M.SRRaGANModel.__new__(M.SRRaGANModel)
        g.gradient_step_num, g.cur_D_update_ratio, g.D_init_iters, g.step = 4, 2, 0, 8
        g.grad_accumulation_steps_D = g.grad_accumulation_steps_G = 1
        t = {'min_D_prob_ratio_4_G': 1.01, 'min_mean_D_correct': 0.6, 'D_valid_Steps_4_G_update': 1}
        pr = torch.full((2, 1, 2, 2), 1.0)
        pf = torch.tensor([0.0, 0.0 if rank == 0 else 3.0]).view(2, 1, 1, 1).expand(2, 1, 2, 2)
        gd, gc, _, _ = g._d_statistics(pr, pf)
        g.D_verification = 'current'
        cur = g._gate_generator_step(t, True, gd, gc)
        g.D_verification = 'past'  # history of all-reduced values, identical on every rank
        g.log_dict = {'D_logits_diff': [(3, 0.5)], 'Correctly_distinguished': [(3, 0.75)]}
        past = g._gate_generator_step(t, True, gd, gc)
        # the generator's FlatAdam under the bucketed all-reduce: p.grad are views of its flat buffer, the buckets
        # average into them in place, and two steps equal per-tensor Adam on flat-averaged gradients, bit for bit
        torch.manual_seed(1)
        fnet = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
        rnet = copy.deepcopy(fnet)
        fopt = FlatAdam(list(fnet.parameters()), lr=1e-2, foreach=False)
        ropt = torch.optim.Adam(list(rnet.parameters()), lr=1e-2, foreach=False)
        fb = M.GradBuckets(list(fnet.parameters()), cap_bytes=300)
        for _ in range(2):
            fopt.zero_grad()
            ropt.zero_grad()
            fb.arm()
            fnet(x).square().sum().backward()
            fb.finish()
            rnet(x).square().sum().backward()
            M._allreduce_grads(list(rnet.parameters()))
            fopt.step()
            ropt.step()
        flat = (all(torch.equal(a, b) for a, b in zip(fnet.parameters(), rnet.parameters())),
                float(sum(float(a.double().sum()) for a in fnet.parameters())))
        # tensors travel as NumPy copies: a tensor in a multiprocessing queue is handed over through a file descriptor
        # of the sending process, which may already have exited
        q.put((rank, p[0].grad.numpy().copy(), p[1].grad.numpy().copy(), diff, correct, d_real, d_fake, launched, same,
               untouched, bufs, gd, gc, cur, past, flat, comm))
    finally:
        dist.destroy_process_group()


def test_ddp_gradient_average_and_consistent_statistics():
    """World size 2 over gloo: grads are averaged over ranks, and the D statistics that decide generator_step are the
    global-batch values on every rank (DataParallel semantics, SRRaGAN_model.py:400-431)."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for pr in procs:
        pr.join(60)
        assert pr.exitcode == 0
    for r in res:
        assert torch.equal(torch.from_numpy(r[1]), torch.full((3, 4), 1.5))
        assert torch.allclose(torch.from_numpy(r[2]), torch.arange(5, dtype=torch.float32) * 1.5)
    # images: rank0 diffs (1-0, 1-3) = (1,-2); rank1 (2-0, 2-4) = (2,-2) -> mean -0.25, correct 0.5
    for r in res:
        assert abs(r[3] - (-0.25)) < 1e-6 and abs(r[4] - 0.5) < 1e-6
    assert res[0][3:7] == res[1][3:7]
    for r in res:
        launched, same, untouched, bufs = r[7:11]
        assert launched >= 2, launched  # at least two buckets went out before backward() returned
        assert same and untouched
        assert bufs == (1.0, 7)
        gd, gc, cur, past = r[11:15]
        assert abs(gc - 0.75) < 1e-6 and abs(gd - 0.25) < 1e-6  # global batch: diffs (1, 1, 1, -2)
        assert cur is False  # 3 of 4 correct globally: no G step on either rank (rank 0 alone would say yes)
        assert past is True  # the shared history passes 'past' on both ranks
    assert res[0][11:15] == res[1][11:15]
    assert res[0][15][0] and res[1][15][0]  # FlatAdam + buckets == per-tensor Adam + flat average
    assert res[0][15][1] == res[1][15][1]   # and the ranks hold the same parameters
    assert all(res[0][16]) and all(res[1][16])  # comm_stats: one all-reduce per bucket, every gradient byte once


class _SlicedFlat(torch.autograd.Function):
    """A stand-in for the HIP generator's sliced backward (train_engine._GeneratorFn._sliced_backward) over a toy
    linear model y = x @ W: the autograd input is the optimiser's flat parameter, the backward adds its gradient into
    flat.grad itself from the END of the flat buffer in chunks, calling the flat-mode GradBuckets sink after each, and
    returns no gradient for the flat parameter."""

    @staticmethod
    def forward(ctx, x, flat, shape, sink, chunks):
        ctx.save_for_backward(x)
        ctx.shape, ctx.sink, ctx.chunks, ctx.flat = shape, sink, chunks, flat
        return x @ flat.view(shape)

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        g = (x.t() @ gy).reshape(-1)
        n = g.numel()
        hi = n
        for lo in sorted(ctx.chunks, reverse=True) + [0]:
            ctx.flat.grad[lo:hi] += g[lo:hi]
            hi = lo
            ctx.sink.ready_from(lo)
            _SlicedFlat.launched_at.append(ctx.sink.launched_in_backward)
        return None, None, None, None, None


def _flat_dist_worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        # (1) flat-mode GradBuckets fed by a producer that writes the flat gradient in slices (the sliced G backward)
        torch.manual_seed(3)
        ps = [torch.nn.Parameter(torch.randn(8, 4)) for _ in range(4)]  # 4 x 32 floats = 4 x 128 B
        ref = [p.detach().clone() for p in ps]
        opt = FlatAdam(ps, lr=1e-2, foreach=False)
        sink = M.GradBuckets(ps, cap_bytes=256, flat_opt=opt)  # 2 parameters per bucket: 2 buckets
        x = torch.randn(5, 32, generator=torch.Generator().manual_seed(20 + rank))
        opt.zero_grad()
        sink.arm()
        _SlicedFlat.launched_at = []  # bucket count after each slice of the backward
        y = _SlicedFlat.apply(x, opt.flat, (32, 4), sink, [lo for lo in sink.emit_offsets() if lo > 0])
        y.square().sum().backward()
        launched = (sink.launched_in_backward, list(_SlicedFlat.launched_at))
        sink.finish()
        # reference: autograd through the plain parameters, then one flat average
        W = torch.cat([r.reshape(-1) for r in ref]).view(32, 4).requires_grad_(True)
        (x @ W).square().sum().backward()
        gref = W.grad.reshape(-1).clone()
        dist.all_reduce(gref)
        gref /= world
        flat_ok = torch.allclose(opt.flat.grad, gref, rtol=1e-6, atol=1e-6)
        views_ok = all(p.grad.data_ptr() == opt.flat.grad[o:o + p.numel()].data_ptr()
                       for p, o in zip(ps, range(0, 128, 32)))
        cs = sink.comm_stats()
        # (2) the D BatchNorm buffers as one flat tensor: ONE broadcast carries all of them (rank 0's values)
        bnet = torch.nn.Sequential(torch.nn.BatchNorm2d(3), torch.nn.BatchNorm2d(5))
        for m in bnet:
            m.running_mean.fill_(rank + 1.0)
            m.running_var.fill_(10.0 * (rank + 1))
        fb = M.FlatBuffers(bnet)
        calls = []
        orig = dist.broadcast
        dist.broadcast = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
        try:
            M._broadcast_buffers(bnet, fb)
        finally:
            dist.broadcast = orig
        bufs = (len(calls), [float(m.running_mean[0]) for m in bnet], [float(m.running_var[-1]) for m in bnet],
                [int(m.num_batches_tracked) for m in bnet])
        # (3) relativistic vanilla GAN loss with the global-batch means (DataParallel gathers the batch):
        # the ranks' averaged D gradient equals the single-process gradient over the concatenated batch
        torch.manual_seed(5)
        Dnet = torch.nn.Linear(6, 1)
        Dref = copy.deepcopy(Dnet)
        real = torch.randn(4, 6, generator=torch.Generator().manual_seed(40 + rank))
        fake = torch.randn(4, 6, generator=torch.Generator().manual_seed(50 + rank))
        m = M.SRRaGANModel.__new__(M.SRRaGANModel)
        m.cri_gan = L.GANLoss('vanilla')
        pr, pf = Dnet(real), Dnet(fake)
        l_real = m.cri_gan(pr - m._batch_mean(pf), True)
        l_fake = m.cri_gan(pf - m._batch_mean(pr), False)
        ((l_real + l_fake) / 2).backward()
        M._allreduce_grads(list(Dnet.parameters()))
        allr = [torch.zeros_like(real) for _ in range(world)]
        allf = [torch.zeros_like(fake) for _ in range(world)]
        dist.all_gather(allr, real)
        dist.all_gather(allf, fake)
        R_, F_ = torch.cat(allr), torch.cat(allf)
        prg, pfg = Dref(R_), Dref(F_)
        lr_g = m.cri_gan(prg - pfg.mean(), True)
        lf_g = m.cri_gan(pfg - prg.mean(), False)
        ((lr_g + lf_g) / 2).backward()
        rel = all(torch.allclose(a.grad, b.grad, rtol=1e-5, atol=1e-7) for a, b in zip(Dnet.parameters(),
                                                                                       Dref.parameters()))
        # the logged losses averaged over ranks are the global-batch losses
        logs = m._global_log_means([l_real, l_fake])
        log_ok = abs(float(logs[0]) - float(lr_g)) < 1e-6 and abs(float(logs[1]) - float(lf_g)) < 1e-6
        # rank-local means would NOT give the global gradient for this non-linear loss (the test can tell them apart)
        Dloc = copy.deepcopy(Dref)
        Dloc.zero_grad()
        pr2, pf2 = Dloc(real), Dloc(fake)
        ((m.cri_gan(pr2 - pf2.mean(), True) + m.cri_gan(pf2 - pr2.mean(), False)) / 2).backward()
        M._allreduce_grads(list(Dloc.parameters()))
        local_differs = not all(torch.allclose(a.grad, b.grad, rtol=1e-5, atol=1e-7)
                                for a, b in zip(Dloc.parameters(), Dref.parameters()))
        q.put((rank, launched, flat_ok, views_ok, (cs['allreduces'], len(sink.buckets)), bufs, rel, log_ok,
               local_differs))
    finally:
        dist.destroy_process_group()


def test_ddp_flat_buckets_sliced_backward_global_means():
    """World size 2 over gloo: (1) flat-mode GradBuckets (the generator's FlatAdam buffer) all-reduced in place by a
    backward that finalises the flat gradient in slices from its end, with buckets launched before backward() returns;
    (2) the D BatchNorm buffers in ONE broadcast; (3) relativistic vanilla-GAN terms over the global batch
    (SRRaGAN_model.py:380-382: torch.mean over DataParallel's gathered batch) give the single-process gradient."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 2000)
    procs = [ctx.Process(target=_flat_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for pr in procs:
        pr.join(60)
        assert pr.exitcode == 0
    for r in res:
        (n_launched, per_slice), flat_ok, views_ok, (n_ar, n_buckets), bufs, rel, log_ok, local_differs = r[1:]
        assert n_buckets == 2 and n_launched == 2 and per_slice[0] >= 1, (n_launched, per_slice)  # first bucket
        # went out after the first slice, while the backward still had a slice to produce
        assert flat_ok and views_ok and n_ar == n_buckets
        assert bufs == (1, [1.0, 1.0], [10.0, 10.0], [0, 0])
        assert rel and log_ok and local_differs
