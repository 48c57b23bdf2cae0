"""cekirdekler_amd — an MI355X-native multi-device compute runtime with the
capabilities of jonike/Cekirdekler.

User kernels are HIP C++ (or OpenCL-C dialect) strings JIT-compiled by hiprtc
for gfx950; one 1-D global range is split across devices (the GPUs of a node,
logical devices, the host CPU) and an iterative load balancer re-weights the
split on every call with the same compute id.
"""
from ._native import CekError, cek, gpu_available
from .arrays import (BFLOAT16, ClArray, ClBf16Array, ClByteArray, ClCharArray, ClDoubleArray,
                     ClFloatArray, ClIntArray, ClLongArray, ClParameterGroup, ClUIntArray, FastArr)
from .cruncher import (PIPELINE_DRIVER, PIPELINE_EVENT, AcceleratorType, ClComputeError,
                       ClNumberCruncher, ClUserEvent, Cores)
from .aux_functions import ClBuiltInAuxilliaryFunctions
from .license import license_text
from .hardware import ClDevice, ClDevices, ClPlatform, ClPlatforms

__version__ = "0.1.0"

__all__ = [
    "AcceleratorType", "BFLOAT16", "ClBuiltInAuxilliaryFunctions", "CekError", "ClArray", "ClBf16Array", "ClByteArray", "ClCharArray",
    "ClComputeError", "ClDevice", "ClDevices", "ClDoubleArray", "ClFloatArray", "ClIntArray",
    "ClLongArray", "ClNumberCruncher", "ClParameterGroup", "ClPlatform", "ClPlatforms", "ClUIntArray", "ClUserEvent",
    "Cores", "FastArr", "PIPELINE_DRIVER", "PIPELINE_EVENT", "cek", "gpu_available", "license_text",
]
