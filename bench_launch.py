"""Rank launcher shared by bench.py, bench_train.py and bench_zopt.py: `--gpus N` means N ranks, one per GPU.

* Under an external launcher (`python -m torch.distributed.run ... bench.py --gpus N`, the driver's form) WORLD_SIZE
  is set: it must equal N, otherwise the run exits non-zero instead of timing a different number of GPUs.
* Run directly with `--gpus N > 1` (WORLD_SIZE unset), the process starts `torch.distributed.run` for N ranks on
  127.0.0.1 as a CHILD process (never an exec: nothing here has touched the GPU, and the parent only waits), and exits
  with its status.  The ranks inherit stdout, so rank 0's JSON line is the run's output.

The reference's counterpart is nn.DataParallel over every visible GPU with `batch_size *= nGPU`
(codes/models/networks.py:99-101,125-126; codes/options/options.py:85-87): one process per GPU here, B per rank.
"""
import json
import os
import socket
import subprocess
import sys


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def ranks(gpus, script, argv, check_devices=True):
    """Call first in main(), before any GPU call.  Returns the world size this process belongs to (1 or N) when it
    is (one of) the bench rank(s); when it is the launcher parent it does not return (exits with the ranks' status)."""
    env_world = os.environ.get('WORLD_SIZE')
    if env_world is not None:
        world = int(env_world)
        if gpus is not None and gpus != world:
            raise SystemExit('--gpus %d but the launcher started WORLD_SIZE=%d ranks: refusing to time a different '
                             'number of GPUs' % (gpus, world))
        return world
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit('--gpus must be >= 1')
    if n == 1:
        return 1
    if check_devices and not share_gpu():
        import torch  # device_count() does not initialise the GPU on this stack
        have = torch.cuda.device_count()
        if have < n:
            raise SystemExit('--gpus %d but only %d GPU(s) are visible' % (n, have))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(n),
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), script] + list(argv)
    rc = subprocess.call(cmd)
    sys.exit(rc)


def share_gpu():
    """ESR_SHARE_GPU=1 (rehearsal only): every rank on GPU 0, gloo instead of RCCL (RCCL needs one GPU per rank) — runs
    the N-rank path of a bench on a one-GPU box; its times are not a scaling measurement."""
    return os.environ.get('ESR_SHARE_GPU') == '1'


def local_device_index():
    return 0 if share_gpu() else int(os.environ.get('LOCAL_RANK', '0'))


def init(dev, world):
    """Join the process group (RCCL on the GPU; gloo for the CPU launcher check and ESR_SHARE_GPU) and confirm its
    size."""
    import torch.distributed as dist
    if world == 1:
        return 1
    if dev.type == 'cuda' and not share_gpu():
        dist.init_process_group('nccl', device_id=dev)
    else:
        dist.init_process_group('gloo')
    got = dist.get_world_size()
    if got != world:
        raise SystemExit('process group has %d ranks, WORLD_SIZE says %d' % (got, world))
    return got


def launcher_check(world, rank):
    """`--launcher-check`: bring the ranks up on the CPU (gloo), have them agree on the world size, print one JSON
    line from rank 0 and stop — the launch path of an N-GPU run without a GPU."""
    import torch
    import torch.distributed as dist
    torch.manual_seed(0)
    if world > 1:
        dist.init_process_group('gloo')
        sizes = [None] * world
        dist.all_gather_object(sizes, (dist.get_rank(), dist.get_world_size(), int(os.environ['LOCAL_RANK'])))
        dist.destroy_process_group()
    else:
        sizes = [(0, 1, 0)]
    if rank == 0:
        print(json.dumps({'launcher_check': True, 'n_gpus': world, 'ranks': [s[0] for s in sizes],
                          'world_sizes': [s[1] for s in sizes], 'local_ranks': [s[2] for s in sizes]}), flush=True)
