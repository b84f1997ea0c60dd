"""Diagnostic (GPU): WHERE does the generator's training forward stop being bitwise reproducible when two processes run
it in lockstep on the one GPU (tools/race_probe.py --mode train: the outputs differ)?  Each process builds the same
seeded latent RRDB + CEM train-mode model and input, meets the other at a barrier, runs `--iters` eager training
forwards (HIP graphs off), and after each one hashes every buffer of the training workspace in forward order (the
concat buffers Q per channel slice [Z | x | x1..x4]).  Printed: per forward, the first buffer (and slice) whose hash
differs between the processes or from the process's own first forward.

    python tools/race_ws_probe.py [--procs 2] [--iters 4] [--nb 23]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
for p_ in (REPO, os.path.join(REPO, 'explorable-super-resolution_old_amd')):
    sys.path.insert(0, p_)


def _hash(t):
    v = t.contiguous().view(torch.int32).reshape(-1).to(torch.int64)
    w = torch.arange(1, v.numel() + 1, device=v.device, dtype=torch.int64) % 1000003
    return int((v * w).sum().item())


def _ws_hashes(ws):
    rows = [('first', _hash(ws.first)), ('fea', _hash(ws.fea))]
    zc = ws.zc
    bounds = [(0, zc), (zc, zc + 64)] + [(zc + 64 + 32 * i, zc + 96 + 32 * i) for i in range(4)]
    for i, q in enumerate(ws.Q):
        for j, (a, b) in enumerate(bounds):
            if b > a:
                rows.append(('Q%d[%s]' % (i, ['Z', 'x', 'x1', 'x2', 'x3', 'x4'][j]), _hash(q[..., a:b])))
    rows.append(('U0', _hash(ws.U0)))
    if ws.U1 is not None:
        rows.append(('U1', _hash(ws.U1)))
    for i, h in enumerate(ws.HR):
        rows.append(('HR%d' % i, _hash(h)))
    rows.append(('overflow', _hash(ws.overflow)))
    return rows


def worker(k, args, barrier, q):
    try:
        _worker(k, args, barrier, q)
    except Exception:  # noqa: BLE001
        import traceback
        q.put((k, traceback.format_exc()))
        barrier.abort()


def _worker(k, args, barrier, q):
    import esr_amd
    from esr_amd import CEMnet as C, train_engine as TE
    from oracle.recipe import seeded_inputs, seeded_params
    TE.USE_GRAPHS = False
    from esr_amd import engine as E
    stash = {}

    def cem_apply(lib, cem, gen, lr, Bn, H, W, M, stream, sf=4):  # engine.cem_apply keeping its intermediates
        from esr_amd import _lib
        stash['gen'], stash['lr'] = gen, lr
        ph = E.cem_phase(sf)
        wd, wi, wu = (cem.DownscaleOP.Filter_OP.weight, cem.Conv_LR_with_Inv_hTh_OP.Filter_OP.weight,
                      cem.Upscale_OP.Filter_OP.weight)
        kd, ki = wd.shape[-1], wi.shape[-1]
        r = stash['r'] = torch.empty(Bn, 3, H, W, device=gen.device)
        q = stash['q'] = torch.empty_like(r)
        out = torch.empty(Bn, 3, sf * H - 2 * M, sf * W - 2 * M, device=gen.device)
        _lib.check(lib.esr_cem_down(gen.data_ptr(), lr.data_ptr(), r.data_ptr(), Bn, H, W, sf, ph,
                                    wd[0, 0].contiguous().data_ptr(), kd, 0, stream), 'esr_cem_down')
        _lib.check(lib.esr_cem_inv(r.data_ptr(), q.data_ptr(), Bn, H, W, wi[0, 0].contiguous().data_ptr(), ki,
                                   stream), 'esr_cem_inv')
        _lib.check(lib.esr_cem_up_add(q.data_ptr(), gen.data_ptr(), out.data_ptr(), Bn, H, W, sf, ph,
                                      wu[0, 0].contiguous().data_ptr(), kd, M, stream), 'esr_cem_up_add')
        return out
    E.cem_apply = cem_apply
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    if args.offset_mb:  # process k first allocates k × offset_mb MB: different device address layouts per process
        keep = torch.empty(max(1, k * args.offset_mb) << 18, device=dev)  # noqa: F841
        stash['keep'] = keep
    B, h, nb = args.batch, args.lr, args.nb
    net = esr_amd.RRDBNet(3, 3, 64, nb, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net, training_patch_size=4 * h)
    sd = model.state_dict()
    params = seeded_params([(n, tuple(v.shape)) for n, v in sd.items()], 800, w_scale=0.1)
    model.load_state_dict({n: torch.from_numpy(v) for n, v in params.items()}, strict=False)
    model = model.to(dev).train()
    lr, z = seeded_inputs(801, (B, 3, h, h), (B, 3, 4 * h, 4 * h), z_mode='pixel')
    x = torch.cat([torch.from_numpy(z).view(B, 48, h, h), torch.from_numpy(lr)], 1).to(dev)
    hashes = []
    for it in range(args.iters + 1):
        out = model(x)
        torch.cuda.synchronize()
        ws = net._esr_cache['train_ws'][1]
        hashes.append(_ws_hashes(ws) + [('gen', _hash(stash['gen'])), ('cem_lr', _hash(stash['lr'])),
                                         ('cem_r', _hash(stash['r'])), ('cem_q', _hash(stash['q'])),
                                         ('out', _hash(out.detach()))])
        del out
        if it == 0:
            barrier.wait()
    q.put((k, hashes))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=2)
    ap.add_argument('--iters', type=int, default=4)
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--lr', type=int, default=96)
    ap.add_argument('--nb', type=int, default=23)
    ap.add_argument('--offset-mb', type=int, default=0)
    args = ap.parse_args()
    ctx = mp.get_context('spawn')
    barrier, q = ctx.Barrier(args.procs), ctx.Queue()
    procs = [ctx.Process(target=worker, args=(k, args, barrier, q)) for k in range(args.procs)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=200) for _ in range(args.procs)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    for k, hs in res:
        assert not isinstance(hs, str), hs
    ref = res[0][1][0]  # process 0's solo first forward (before the barrier)
    for k, hs in res:
        for it, rows in enumerate(hs):
            bad = [name for (name, v), (_, r) in zip(rows, ref) if v != r]
            print('process %d forward %d (%s): %d of %d buffers differ from process 0 forward 0; first: %s' % (
                k, it, 'solo' if it == 0 else 'lockstep', len(bad), len(rows), bad[:6]), flush=True)


if __name__ == '__main__':
    main()
