#!/usr/bin/env python3
"""Do independent branches of a captured HIP graph run concurrently on this stack?  Two single-thread spin kernels
(torch.cuda._sleep) on two forked streams, eagerly and captured in one graph; concurrent ≈ T, serialised ≈ 2T.
Also the same with the side stream at a different priority."""
import time

import torch


def timed(fn, n=20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    cyc = 2_000_000
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, 'priority_range') else (0, -1)
    print('priority range', lo, hi)
    for prio in (0, hi):
        side = torch.cuda.Stream(dev, priority=prio)

        def fork():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            torch.cuda._sleep(cyc)
            with torch.cuda.stream(side):
                torch.cuda._sleep(cyc)
            cur.wait_stream(side)

        one = timed(lambda: torch.cuda._sleep(cyc))
        eager = timed(fork)
        g = torch.cuda.CUDAGraph()
        fork()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            fork()
        graph = timed(g.replay)
        print('side priority %d: one spin %.3f ms, two forked eager %.3f ms, two forked in a graph %.3f ms'
              % (prio, one, eager, graph), flush=True)


if __name__ == '__main__':
    main()
