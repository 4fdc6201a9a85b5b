"""dcnn_amd — an MI355X-native (gfx950 / CDNA4, ROCm) CNN training framework with the
capabilities of tungphambasement/DCNN: Sequential/builder API, model zoo, checkpoint format,
losses/optimizers/schedulers, trainers, data loaders/augmentation, data-parallel training over
RCCL and a sync / semi-async pipeline runtime — on hand-written HIP kernels (MFMA implicit-GEMM
convolutions, fused BatchNorm/ReLU/residual, fused loss, flat-buffer optimizers).
"""
__version__ = "0.1.0"

import os as _os

# ProcessGroupNCCL's event cache hands an event of a finished eager collective (still queued for
# the watchdog) to a collective recorded inside a hipGraph capture; the watchdog's query of it then
# fails ("operation not permitted on an event last recorded in a capturing stream") and aborts the
# rank. Every captured step issues its bucket all-reduces under capture, so keep the cache off
# unless the launcher set it (read when a process group is created).
_os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")

from .device import Device, DeviceManager, DeviceType, Flow, Task, get_cpu, get_device, get_gpu  # noqa: F401
from .nn import *  # noqa: F401,F403
from . import models  # noqa: F401
