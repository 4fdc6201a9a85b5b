"""dcnn_amd — an MI355X-native (gfx950 / CDNA4, ROCm) CNN training framework with the
capabilities of tungphambasement/DCNN: Sequential/builder API, model zoo, checkpoint format,
losses/optimizers/schedulers, trainers, data loaders/augmentation, data-parallel training over
RCCL and a sync / semi-async pipeline runtime — on hand-written HIP kernels (MFMA implicit-GEMM
convolutions, fused BatchNorm/ReLU/residual, fused loss, flat-buffer optimizers).
"""
__version__ = "0.1.0"

from .device import Device, DeviceManager, DeviceType, Flow, Task, get_cpu, get_device, get_gpu  # noqa: F401
from .nn import *  # noqa: F401,F403
from . import models  # noqa: F401
