"""MI355X-native distributed K-FAC for PyTorch-ROCm.

Public surface mirrors the reference `kfac` package (kfac/__init__.py:1-5):

    import distributed_kfac_pytorch_amd as kfac
    preconditioner = kfac.KFAC(model, comm_method=kfac.CommMethod.COMM_OPT, ...)
    scheduler = kfac.KFACParamScheduler(preconditioner, ...)

Subpackages: `layers` (per-layer K-FAC state), `modules` (K-FAC-friendly
LSTM), `ops` (gfx950 HIP kernels via ctypes), `parallel` (execution plan,
bucketed RCCL collectives, DDP bootstrap), `models` (ResNets, LSTM and
Transformer LMs), `utils` (LPT/worker allocation, tracing), `comm`.
"""
from . import comm
from . import utils
from . import modules
from . import layers
from . import ops
from . import parallel
from . import graphs
from .preconditioner import KFAC, CommMethod
from .scheduler import KFACParamScheduler

__version__ = '0.1.0'

__all__ = ['KFAC', 'CommMethod', 'KFACParamScheduler', 'comm', 'utils', 'modules', 'layers',
           'ops', 'parallel', '__version__']
