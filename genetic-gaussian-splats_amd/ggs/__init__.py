"""ggs — MI355X-native 2D Gaussian-splat render + fitness (host side).

Plain Python + numpy over libggs.so (hand-written HIP for gfx950, C ABI in
include/ggs.h).  The drop-in modules with the reference's names live in
``modules/`` next to this package.
"""
from ._lib import (GGS_FIT_BOOST, GGS_FIT_NONE, GGS_FIT_WEIGHTED, GGSDeviceError,  # noqa: F401
                   GGSError, GGSInputError, LIB_PATH, ensure_init, lib, runtime_info, select_devices)
from .parallel import RcclGather  # noqa: F401
from .api import (TargetPlan, as_f32, encode, fitness, fitness_device,  # noqa: F401
                  fitness_population, preprocess, profile_enable, profile_read, profile_reset,
                  render, render_device)

__version__ = "0.1.0"
