"""irlmx -- MI355X-native MaxEnt-IRL inner loop.

Host side in Python on PyTorch-ROCm tensors, compute in hand-written HIP
kernels for gfx950 behind the C ABI of ``libirlmx.so`` (include/irlmx.h).

* ``irlmx.DeviceMDP``  -- transition model resident in HBM (stencil / ELL)
* ``irlmx.ops``        -- batched device ops: backward, forward SVF, soft VI, VI
* ``irlmx.batch``      -- batched IRL gradient steps (B instances per call)
* ``maxent`` / ``solver`` (next to this package) -- numpy drop-ins for the
  reference modules of the same names.
"""

from ._lib import IrlmxError, load, require_device  # noqa: F401
from .mdp import DeviceMDP  # noqa: F401
from . import ops  # noqa: F401

__version__ = "0.1.0"
