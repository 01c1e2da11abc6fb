"""veneur_amd -- MI355X-native per-flush sketch aggregation engine for veneur.

The product path is the HIP library libveneur_amd.so (hand-written gfx950 kernels behind
the C-ABI in include/veneur_amd.h).  This package is the host-side handle used by tests
and the benchmark; importing it without the built library raises ImportError.
"""
from . import _abi
from .engine import DeviceBuffer, Engine, EngineError, FlushOutput, device_count, metro64_device, synth

__all__ = ["Engine", "EngineError", "FlushOutput", "DeviceBuffer", "device_count", "metro64_device", "synth",
           "_abi"]
