"""distributed_amd — MI355X-native placement engine for the dask.distributed scheduler
hot path (decide_worker / worker_objective, WorkStealing.balance, frontier release).

Submodules:
  graphs   synthetic task graphs (numpy only)
  engine   PlacementEngine: host wrapper of the HIP engine (libdgplace.so, C ABI in include/dgplace.h)
"""
__all__ = ["graphs", "engine"]
__version__ = "0.1.0"
