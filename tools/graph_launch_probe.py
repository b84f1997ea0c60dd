#!/usr/bin/env python3
"""How far the host can run ahead of the GPU on this ROCm stack: host time to enqueue a chain of N short kernels
(eager launches, and one HIP graph replay of the same chain) against the chain's GPU time.  In the config-3 trace
(tools/prof_train_api.sh) hipGraphLaunch of the generator's backward graph returned only ~0.6 ms before the graph's
last kernel ran, so the host's next Python work left the GPU idle.
    usage: python tools/graph_launch_probe.py [N ...]      (runs each configuration in this process; env knobs are
                                                            read by the HIP runtime at start-up, so vary them per run)
"""
import os
import sys
import time

import torch


MODE = os.environ.get('PROBE_MODE', 'kernels')
_Y = {}


def chain(x, n):
    """n kernels; PROBE_MODE=memset / memcpy puts a memset (zero_ of a side buffer) / a device-to-device copy after
    every 20th kernel (the nodes torch records for zero_() / copy_() inside a captured graph)."""
    y = _Y.setdefault('y', torch.empty_like(x))
    for i in range(n):
        x.mul_(1.0000001)
        if i % 20 == 19:
            if MODE == 'memset':
                y.zero_()
            elif MODE == 'memcpy':
                y.copy_(x)


def main():
    ns = [int(a) for a in sys.argv[1:]] or [100, 400, 1200]
    dev = torch.device('cuda', 0)
    x = torch.ones(8 << 20, device=dev)  # 32 MB: ~10-15 us per mul_
    env = {k: os.environ[k] for k in sorted(os.environ) if k.startswith(('ROC_', 'DEBUG_CLR', 'DEBUG_HIP', 'HIP_'))}
    print('env', env, flush=True)
    for n in ns:
        for _ in range(2):
            chain(x, n)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        chain(x, n)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            chain(x, 3)
            with torch.cuda.graph(g, stream=s):
                chain(x, n)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        g.replay()
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        print('N=%5d  eager: enqueue %7.2f ms, total %7.2f ms | graph: replay() returns after %7.2f ms, total %7.2f ms'
              % (n, (t1 - t0) * 1e3, (t2 - t0) * 1e3, (t4 - t3) * 1e3, (t5 - t3) * 1e3), flush=True)
        del g


if __name__ == '__main__':
    main()
