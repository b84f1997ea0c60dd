"""Config 4's data-parallel step at its PER-RANK production shape (B=16 × 96² LR crops per rank, RRDB-23, latent, CEM
train mode, WGAN-GP as shipped) on the box's one GPU: two ranks on GPU 0 over gloo (as bench_launch's ESR_SHARE_GPU
rehearsal: RCCL needs a GPU per rank; the driver's 8-GPU run takes the same code with nccl) against single-process
runs of each rank's half of a B=32 batch.

The reference's counterpart is nn.DataParallel (models/networks.py:99-101,125-126) over a batch of nGPU × 16
(options/options.py:85-87): each replica's BatchNorm normalises its own 16 images, every loss is a mean over the
gathered 32 (wgan-gp: linear in the D outputs), so the DataParallel gradient is the average of the gradients each
replica's half would give alone.  Checked: the first D step's and the first G step's averaged gradients (two ranks)
against the mean of the two single-process half-batch gradients, ≤ 1e-5 relative L2 (the D learning rate is 0 so
that the G step of micro-step 1 sees the same D in every run), the generator_step decisions, and that the G
gradient's all-reduce buckets went out from inside the generator's backward while it still had RRDBs to do
(train_engine._GeneratorFn._sliced_backward with the flat-mode GradBuckets), with the optimiser's flat buffer as the
one autograd input (the single-process step's flat path) and one D BatchNorm-buffer broadcast per D optimiser step."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _cfg():
    from train_recipe import C3_GRID_CFG
    return dict(C3_GRID_CFG, lr_D=0.0)


def _run_half(half, dev):
    """One SRRaGANModel on images [16·half, 16·half + 16) of the B=32 batch, 2 micro-steps: the gradient each
    optimiser applies first, the generator_step flags, and the sliced-backward / broadcast records."""
    from train_recipe import step_data, train_opt
    from oracle.recipe import seeded_params
    from esr_amd.SRRaGAN_model import SRRaGANModel
    import torch.distributed as dist
    cfg = _cfg()
    B = cfg['batch']
    torch.manual_seed(0)
    model = SRRaGANModel(train_opt(cfg), accumulation_steps_per_batch=cfg['acc'], device=dev)
    gsd, dsd = model.netG.state_dict(), model.netD.state_dict()
    gp = seeded_params([(k, tuple(v.shape)) for k, v in gsd.items()], cfg['seed'], w_scale=cfg['w_scale_G'])
    dp = seeded_params([(k, tuple(v.shape)) for k, v in dsd.items() if 'running' not in k and 'num_batches' not in k],
                       cfg['seed'] + 1, w_scale=1.0)
    model.netG.load_state_dict({k: torch.from_numpy(v) for k, v in gp.items()}, strict=False)
    model.netD.load_state_dict({k: torch.from_numpy(v) for k, v in dp.items()}, strict=False)
    rng = np.random.default_rng(cfg['seed'] + 300 + half)
    model._interp_points = lambda n: torch.from_numpy(rng.random((n, 1, 1, 1)).astype(np.float32)).to(dev)
    first = {}
    d_steps = []  # micro-steps with a D optimiser step (none at gradient step 0 with D_init_iters 0: SRRaGAN_model.py:360)
    cur = [0]
    for o, tag in ((model.optimizer_G, 'G'), (model.optimizer_D, 'D')):
        def step(*a, _o=o, _step=o.step, _tag=tag, **kw):
            if _tag == 'D':
                d_steps.append(cur[0])
            if _tag not in first:
                _o._sync_views()
                first[_tag] = _o.flat.grad.detach().double().cpu().numpy()
            return _step(*a, **kw)
        o.step = step
    local = {}  # rank-local flat gradient ranges as each bucket went out (first launch per tag and range)
    for tag, bk in [(t_, b_) for t_, b_ in (('G', model._g_buckets), ('D', model._d_buckets)) if b_.ranges]:
        def launch(b, _bk=bk, _tag=tag, _orig=bk._launch):
            lo, hi = _bk.ranges[b]
            local.setdefault(_tag, {}).setdefault((lo, hi), _bk.flat_opt.flat.grad[lo:hi].detach().double().cpu().numpy())
            return _orig(b)
        bk._launch = launch
    slices = []  # (lo, buckets launched so far) at each ready_from of the G buckets
    rf = model._g_buckets.ready_from if model._g_buckets.ranges else (lambda lo: None)

    def ready_from(lo):  # (also the flat parameter's post-accumulate hook: must return None)
        rf(lo)
        slices.append((lo, model._g_buckets.launched_in_backward))
    model._g_buckets.ready_from = ready_from
    bcast = []  # torch.distributed.broadcast calls during the steps (the D BatchNorm buffers): (micro-step, caller)
    bb = dist.broadcast

    def counted(*a, **k):
        import traceback
        bcast.append((cur[0], ' <- '.join('%s:%d' % (os.path.basename(f.filename), f.lineno)
                                          for f in traceback.extract_stack()[-5:-1])))
        return bb(*a, **k)
    dist.broadcast = counted
    flat_in = []
    import esr_amd.train_engine as TE
    fwd = TE._GeneratorFn.apply
    fwd_in = []  # (input hash, flat parameter hash, activation scale, precision) of each training forward
    fresh = []  # generator output norms right after each training forward (the step's end may differ: corruption)

    def apply(*a):
        flat_in.append(len(a) == 4)
        out = fwd(*a)
        fresh.append(out.detach().double().flatten(1).norm(dim=1).cpu().numpy())
        import hashlib
        from esr_amd import engine as E_
        fwd_in.append((hashlib.sha256(a[0].detach().cpu().numpy().tobytes()).hexdigest()[:12],
                       hashlib.sha256(a[3].detach().cpu().numpy().tobytes()).hexdigest()[:12] if len(a) == 4 else None,
                       E_.act_scale(a[1]), getattr(a[1], 'esr_precision', None)))
        return out
    TE._GeneratorFn.apply = apply
    try:
        flags, fake = [], []
        for k in range(cfg['steps']):
            cur[0] = k
            lr, hr, z = step_data(dict(cfg, batch=2 * B), k)
            sl = slice(half * B, (half + 1) * B)
            t = lambda a: torch.from_numpy(np.ascontiguousarray(a[sl])).to(dev)  # noqa: E731
            model.feed_data({'LR': t(lr), 'HR': t(hr), 'Z': t(z)})
            model.optimize_parameters()
            flags.append(bool(model.generator_step))
            fake.append(model.fake_H.detach().double().flatten(1).norm(dim=1).cpu().numpy())
    finally:
        dist.broadcast = bb
        TE._GeneratorFn.apply = fwd
    world = dist.get_world_size() if dist.is_initialized() else 1
    n_buckets = len(model._g_buckets.buckets)
    dshapes = [(k, v.numel()) for k, v in model.netD.named_parameters()]
    from esr_amd import engine as E
    loc = {}
    for tag, d in local.items():
        n = max(hi for lo, hi in d)
        v = np.full(n, np.nan)
        for (lo, hi), x in d.items():
            v[lo:hi] = x
        loc[tag] = v
    return {'first': first, 'flags': flags, 'fake': fake, 'dshapes': dshapes, 'local': loc, 'fresh': fresh, 'fwd_in': fwd_in,
            'logs': {k: [x[1] for x in v] for k, v in model.log_dict.items() if v},
            'reruns': (E.OVERFLOW_RERUNS, E.ACT_SCALE_REDUCTIONS), 'slices': slices, 'n_buckets': n_buckets, 'bcast': bcast, 'd_steps': d_steps,
            'flat_in': flat_in, 'world': world, 'comm': model._g_buckets.comm_stats()}


def _worker(rank, world, port, half, q):
    for p_ in (HERE, os.path.join(HERE, 'golden'), os.path.dirname(HERE),
               os.path.join(os.path.dirname(HERE), 'explorable-super-resolution_old_amd')):
        if p_ not in sys.path:
            sys.path.insert(0, p_)
    import torch.distributed as dist
    try:
        dev = torch.device('cuda', 0)
        torch.cuda.set_device(dev)
        if world > 1:
            os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
            dist.init_process_group('gloo', rank=rank, world_size=world)
        if os.environ.get('C4_NOFLAT'):  # diagnostic: '1' = no flat-mode buckets (round-5 per-tensor cat buckets)
            from esr_amd import SRRaGAN_model as SM
            init = SM.GradBuckets.__init__
            SM.GradBuckets.__init__ = lambda self, params, cap_bytes=16 << 20, flat_opt=None: init(self, params,
                                                                                                   cap_bytes, None)
        if os.environ.get('C4_SYNC') == '1':  # diagnostic: a device-wide synchronize before every collective
            from esr_amd import SRRaGAN_model as SM
            coll = SM.collective
            SM.collective = lambda *a, **k: (torch.cuda.synchronize(), coll(*a, **k))[1]
        if os.environ.get('C4_NANFILL') == '1':  # diagnostic: every torch.empty filled with NaN
            torch.use_deterministic_algorithms(True, warn_only=True)
            torch.utils.deterministic.fill_uninitialized_memory = True
        q.put((rank, _run_half(half, dev), None))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, traceback.format_exc()))
    finally:
        if world > 1 and dist.is_initialized():
            dist.destroy_process_group()


def _run(world, half=None):
    """world ranks (rank r on half r), or one single-process run on `half`, each in a fresh process."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, r if half is None else half, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    for r in res:
        assert r[2] is None, r[2]
    return [r[1] for r in res]


def test_c4_two_ranks_per_rank_production_shape():
    halves = [_run(1, half=h)[0] for h in (0, 1)]
    ranks = _run(2)
    again = _run(1, half=0)[0]
    print('overflow reruns / act-scale reductions: halves', [h['reruns'] for h in halves], 'ranks',
          [r['reruns'] for r in ranks], 'half 0 again', again['reruns'])
    print('half 0 run twice: first D grads equal', np.array_equal(again['first']['D'], halves[0]['first']['D']),
          'fake_H equal', all(np.array_equal(a, b) for a, b in zip(again['fake'], halves[0]['fake'])))
    assert halves[0]['flags'] == halves[1]['flags'] == ranks[0]['flags'] == ranks[1]['flags'] == [False, True]
    for tag in ('D', 'G'):
        ref = 0.5 * (halves[0]['first'][tag] + halves[1]['first'][tag])
        for i, r in enumerate(ranks):
            rel = float(np.linalg.norm(r['first'][tag] - ref) / np.linalg.norm(ref))
            own = float(np.linalg.norm(r['first'][tag] - halves[i]['first'][tag]) / np.linalg.norm(ref))
            print('C4 per-rank shape: first %s step, averaged two-rank gradient vs the mean of the single-process '
                  'half-batch gradients: %.2e relative L2 (vs rank %d\'s own half alone: %.2e; the halves differ by '
                  '%.2e)' % (tag, rel, i, own, float(np.linalg.norm(halves[0]['first'][tag] - halves[1]['first'][tag]) /
                                                     np.linalg.norm(ref))))
            if tag in r['local']:
                lv = r['local'][tag]
                print('rank %d local %s gradient (as its buckets went out) vs its half alone: bitwise %s, rel %.2e' % (
                    i, tag, np.array_equal(lv, halves[i]['first'][tag]),
                    float(np.linalg.norm(lv - halves[i]['first'][tag]) / np.linalg.norm(halves[i]['first'][tag]))))
            if rel > 1e-5 and tag == 'D':
                o, rows = 0, []
                for k, n in r['dshapes']:
                    a, b = r['first'][tag][o:o + n], ref[o:o + n]
                    rows.append((float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)), k,
                                 float(np.linalg.norm(a - halves[i]['first'][tag][o:o + n]) / max(np.linalg.norm(b), 1e-30))))
                    o += n
                print('worst D params (rel err vs avg, vs own half):', sorted(rows)[::-1][:8])
                print('fake_H norms: rank', [f.tolist() for f in r['fake']], 'half', [f.tolist() for f in halves[i]['fake']])
                print('logs rank', r['logs'], 'halves', halves[0]['logs'], halves[1]['logs'])
            assert rel <= 1e-5, (tag, rel, own)
    for r in ranks:
        # the G buckets went out from inside the generator's backward, most of them while RRDBs were still to come
        early = max([n for lo, n in r['slices'] if lo > 0] or [0])
        print('G buckets: %d; launched at the backward\'s slices (lo, count): %s; comm %s' % (
            r['n_buckets'], r['slices'], r['comm']))
        assert r['n_buckets'] >= 4 and early >= r['n_buckets'] - 1, (r['slices'], r['n_buckets'])
        assert r['slices'][-1] == (0, r['n_buckets'])
        assert r['comm']['allreduces'] == r['n_buckets']  # one G gradient step: every bucket once
        assert all(r['flat_in']) and r['flat_in']  # the flat parameter as the generator's one autograd input
        print('D steps at micro-steps %s; broadcasts (micro-step, caller): %s' % (r['d_steps'], r['bcast']))
        # one D-buffer broadcast per D optimiser step, not one per buffer
        assert r['d_steps'] and [b[0] for b in r['bcast']] == r['d_steps']
    for h in halves:
        assert all(h['flat_in']) and h['slices'] == [] and h['world'] == 1
