"""Does an x3 Z-optimisation iteration with inputs beyond f16's range set the deferred overflow flags?"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
import torch  # noqa: E402
import test_gpu_zopt as T  # noqa: E402
from esr_amd import engine, train_engine as TE  # noqa: E402

dev = torch.device('cuda', 0)
orig_add = TE.DeferredOverflow.add


def add(self, overflow, bad, reset):
    print('deferred add: overflow', int(overflow.item()), 'bad', int(bad.item()), flush=True)
    return orig_add(self, overflow, bad, reset)


TE.DeferredOverflow.add = add
print('reruns before', engine.OVERFLOW_RERUNS)
try:
    T.test_z_optimizer_overflow_redo_equals_fp32_loop(dev)
    print('PASSED')
except AssertionError as e:
    print('FAILED', e)
print('reruns after', engine.OVERFLOW_RERUNS)
