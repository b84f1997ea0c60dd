"""Diagnostic (GPU): is the generator's training forward (config 3/4 shape: latent RRDB-23 + CEM train mode, B=16 × 96²,
define_G's init scale) bitwise reproducible when two processes run it in lockstep on the one GPU?  Each process builds
the same seeded model and input, meets the other at a barrier, then runs `--iters` forwards; every output is compared
bitwise with the process's first, and the per-image output norms with the other process's.  A mismatch is localised:
per image, the LR-grid bounding box of the HR pixels that differ (|d| > 1e-6 relative to the image max).

    python tools/race_probe.py [--procs 2] [--iters 6] [--mode train|eval]
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


def worker(k, args, barrier, q):
    import esr_amd
    from esr_amd import CEMnet as C
    from oracle.recipe import seeded_inputs, seeded_params
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    B, h, nb = args.batch, args.lr, args.nb
    net = esr_amd.RRDBNet(3, 3, 64, nb, latent_input='all_layers_HR_downscaled', num_latent_channels=3)
    model = C.CEMnet(C.Get_CEM_Config(4)).WrapArchitecture_PyTorch(net, training_patch_size=4 * h)
    sd = model.state_dict()
    params = seeded_params([(n, tuple(v.shape)) for n, v in sd.items()], 800, w_scale=0.1)
    model.load_state_dict({n: torch.from_numpy(v) for n, v in params.items()}, strict=False)
    model = model.to(dev)
    model.train(args.mode == 'train')
    lr, z = seeded_inputs(801, (B, 3, h, h), (B, 3, 4 * h, 4 * h), z_mode='pixel')
    x = torch.cat([torch.from_numpy(z).view(B, 48, h, h), torch.from_numpy(lr)], 1).to(dev)
    if args.mode == 'cem':  # the CEM stencils alone (engine.cem_apply) on a fixed generator output, train mode (M=0)
        from esr_amd import _lib, engine as E
        gen = torch.from_numpy(np.random.default_rng(5).standard_normal((B, 3, 4 * h, 4 * h)).astype(np.float32)).to(dev)
        lrt = torch.from_numpy(lr).to(dev)
        lib = _lib.load()
        st = __import__('ctypes').c_void_p(torch.cuda.current_stream().cuda_stream)
        run = lambda: E.cem_apply(lib, model, gen, lrt, B, h, h, 0, st)  # noqa: E731
    elif args.mode == 'train':
        for p in model.parameters():
            p.requires_grad_(p.requires_grad)
        run = lambda: model(x)  # noqa: E731  (parameters require grad: the training forward)
    else:
        def run():
            with torch.no_grad():
                return model(x)
    outs = [run().detach().clone()]
    torch.cuda.synchronize()
    barrier.wait()
    for _ in range(args.iters):
        outs.append(run().detach().clone())
    torch.cuda.synchronize()
    ref = outs[0]
    rows = []
    for i, o in enumerate(outs[1:]):
        o = o.view_as(ref)
        if torch.equal(o, ref):
            continue
        d = (o - ref).abs()
        for b in range(B):
            db = d[b].amax(0)
            thr = 1e-6 * float(ref[b].abs().max())
            ys, xs = torch.nonzero(db > thr, as_tuple=True)
            if len(ys):
                rows.append((i + 1, b, int(len(ys)), float(db.max()), (int(ys.min()), int(ys.max()),
                                                                     int(xs.min()), int(xs.max())),
                             sorted(set(int(v) for v in xs.tolist()))[:20]))
    q.put((k, [o.double().flatten(1).norm(dim=1).cpu().numpy() for o in outs], rows))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--procs', type=int, default=2)
    ap.add_argument('--iters', type=int, default=6)
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--lr', type=int, default=96)
    ap.add_argument('--nb', type=int, default=23)
    ap.add_argument('--mode', choices=['train', 'eval', 'cem'], default='train')
    args = ap.parse_args()
    ctx = mp.get_context('spawn')
    barrier, q = ctx.Barrier(args.procs), ctx.Queue()
    procs = [ctx.Process(target=worker, args=(k, args, barrier, q)) for k in range(args.procs)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(args.procs)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    base = res[0][1][0]
    for k, norms, rows in res:
        print('process %d (%s): %d of %d forwards differ from its first; first forward vs process 0\'s: %s' % (
            k, args.mode, len({r[0] for r in rows}), args.iters, bool(np.array_equal(norms[0], base))), flush=True)
        for r in rows[:12]:
            print('   forward %d image %d: %d HR px differ, max |d| %.3e, HR box y %d-%d x %d-%d, columns %s' % (
                r[:4] + r[4] + (r[5],)), flush=True)


if __name__ == '__main__':
    main()
