"""veneur_amd -- MI355X-native per-flush sketch aggregation engine for veneur.

The product path is the HIP library libveneur_amd.so (hand-written gfx950 kernels behind
the C-ABI in include/veneur_amd.h).  This package is the host-side handle used by tests
and the benchmark -- Engine (the C-ABI) and Worker (veneur's Worker / samplers API over it);
importing it without the built library raises ImportError.
"""
from . import _abi
from .engine import (Comm, DeviceBuffer, DeviceStream, Engine, EngineError, FlushOutput, HostWindows, device_count,
                     metro64_device,
                     synth, synth_key_counts)
from .worker import (Aggregate, HistogramAggregates, InterMetric, JSONMetric, MetricKey, MetricScope, MetricType,
                     UDPMetric, Worker, WorkerMetrics)

__all__ = ["Comm", "DeviceStream", "HostWindows", "synth_key_counts", "Engine", "EngineError", "FlushOutput", "DeviceBuffer", "device_count", "metro64_device", "synth",
           "_abi", "Worker", "WorkerMetrics", "UDPMetric", "JSONMetric", "MetricKey", "MetricScope", "MetricType",
           "InterMetric", "Aggregate", "HistogramAggregates"]
