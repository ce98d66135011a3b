"""partisan_amd -- MI355X-native simulator of partisan's HyParView membership
and Plumtree broadcast (hot path of BASELINE.json north_star).

The product is the HIP library partisan_amd/csrc/libpartisan_gpu_sim.so behind
the C ABI in include/partisan_gpu_sim.h; this package is its Python host side.
"""
from .sim import NONE, SimError, Simulator, default_config  # noqa: F401
from . import workloads  # noqa: F401

__all__ = ["Simulator", "SimError", "default_config", "workloads", "NONE"]
