"""esr_amd — MI355X-native RRDB-23 + CEM ×4 super-resolution hot path behind the reference's module API.

Drop-in counterparts (reference paths relative to codes/):
  esr_amd.architecture.RRDBNet        models/modules/architecture.py:102-175
  esr_amd.CEMnet.{CEMnet, CEM_PyTorch, Get_CEM_Config, Adjust_State_Dict_Keys}   CEM/CEMnet.py
  esr_amd.networks.{define_G, init_weights}                                     models/networks.py
The compute runs in libesr_amd.so (hand-written HIP for gfx950, C ABI in include/esr_amd.h).
"""
from . import _lib  # noqa: F401
from .architecture import RRDBNet  # noqa: F401
from . import CEMnet  # noqa: F401  (module, as the reference's `import CEM.CEMnet as CEMnet`)
from .networks import define_G, init_weights  # noqa: F401

__all__ = ['RRDBNet', 'CEMnet', 'define_G', 'init_weights']
