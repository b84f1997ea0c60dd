#!/usr/bin/env python3
"""Where does the first Z iteration of each Z_optimizer.optimize() call go?  (round-4 review item 1)

Builds the bench_zopt config-5 leg, then calls optimize() several times with max_iters=3, recording per-iteration wall
times (each iteration ends with a device sync), and profiles the first iteration of the last call with torch.profiler
(CPU ops, top by self CPU time).   usage: python tools/zopt_iter_probe.py [calls]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'explorable-super-resolution_old_amd'))

import torch  # noqa: E402

import bench_zopt  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    from esr_amd.SRRaGAN_model import SRRaGANModel
    from esr_amd.Z_optimization import Z_optimizer
    from esr_amd import networks
    args = bench_zopt.leg_args()
    opt = {'is_train': False, 'scale': 4, 'gpu_ids': [0], 'range': [0, 1],
           'network_G': {'which_model_G': 'RRDB_net', 'CEM_arch': 1, 'latent_input': 'all_layers',
                         'latent_input_domain': 'HR_downscaled', 'latent_channels': 'SVDinNormedOut_structure_tensor',
                         'norm_type': None, 'mode': 'CNA', 'nf': 64, 'nb': args.nb, 'in_nc': 3, 'out_nc': 3, 'gc': 32}}
    torch.manual_seed(1234)
    model = SRRaGANModel(opt, kernel=bench_zopt.learned_kernel(), device=dev)
    networks.init_weights(model.netG.module, scale=0.1)
    g = torch.Generator().manual_seed(99)
    B, h = args.batch, args.lr_size
    data = {'LR': torch.rand(B, 3, h, h, generator=g).to(dev),
            'Z': (torch.rand(B, 3, 4 * h, 4 * h, generator=g) * 2 - 1).to(dev)}
    model.feed_data(data, need_HR=False)
    model.test()
    model.netG.eval()
    zo = Z_optimizer('max_STD', [4 * h, 4 * h], model, 1.0, 3, data=data, initial_LR=0.01, batch_size=B)
    for c in range(calls):
        stamps = []
        zo.on_iteration = lambda _: stamps.append(time.perf_counter())
        prof = None
        if c == calls - 1:
            orig = zo._iteration
            state = {'n': 0}

            def first_profiled(z_iter):
                state['n'] += 1
                if state['n'] != 1:
                    return orig(z_iter)
                nonlocal prof
                with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as p:
                    r = orig(z_iter)
                    torch.cuda.synchronize()
                prof = p
                return r
            zo._iteration = first_profiled
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        zo.optimize()
        torch.cuda.synchronize()
        ms = [round((b - a) * 1e3, 2) for a, b in zip([t0] + stamps[:-1], stamps)]
        print('call %d: iteration ms %s' % (c, ms), flush=True)
        if prof is not None:
            print(prof.key_averages().table(sort_by='self_cpu_time_total', row_limit=25), flush=True)


if __name__ == '__main__':
    main()
