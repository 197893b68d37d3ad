"""ctypes binding of ``libdgplace.so`` (C ABI: ``include/dgplace.h``).

The HIP library is the product path: there is no CPU fallback. If the shared
library is missing or no GPU is visible, the calls raise instead of silently
computing placements some other way.
"""
from __future__ import annotations

import ctypes as C
import os

PKG = os.path.dirname(os.path.abspath(__file__))
# DGP_LIB (debugging / A-B runs only): a variant build of the same sources
LIB_PATH = os.environ.get("DGP_LIB") or os.path.join(PKG, "libdgplace.so")
# the stream kernel's two window builds, both in the library (dgp_set_window, ABI 19)
WINDOWS = (32, 64)

_P = C.c_void_p
_i32p = C.POINTER(C.c_int32)

# name -> (restype, argtypes); the list is also what tests check the library exports
SIGNATURES = {
    "dgp_abi_version": (C.c_int, []),
    "dgp_create": (_P, [C.c_int]),
    "dgp_destroy": (None, [_P]),
    "dgp_last_error": (C.c_char_p, [_P]),
    "dgp_set_config": (C.c_int, [_P, C.c_int64, C.c_int64, C.c_double, C.c_double]),
    "dgp_set_workers": (C.c_int, [_P, C.c_int32, _P]),
    "dgp_set_graph": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P, C.c_int32, _P, _P, C.c_int32, _P, _P]),
    "dgp_set_task_results": (C.c_int, [_P, _P, _P, _P]),
    "dgp_set_restrictions": (C.c_int, [_P, _P, _P, _P]),
    "dgp_update_restrictions": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P]),
    "dgp_set_rootish": (C.c_int, [_P, C.c_int64, _P, _P]),
    "dgp_reset": (C.c_int, [_P]),
    "dgp_update_graph": (C.c_int, [_P]),
    "dgp_run_rounds": (C.c_int, [_P, C.c_int64, _P]),
    "dgp_tasks_finished": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dgp_set_resident": (C.c_int, [_P, C.c_int]),
    "dgp_set_task_messages": (C.c_int, [_P, C.c_int]),
    "dgp_tasks_finished_post": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P, _P, _P]),
    "dgp_tasks_finished_wait": (C.c_int, [_P, _P, _P]),
    "dgp_move_task": (C.c_int, [_P, C.c_int32, C.c_int32]),
    "dgp_add_worker": (C.c_int, [_P, C.c_int32, _P]),
    "dgp_add_worker_at": (C.c_int, [_P, C.c_int32, C.c_int32, C.c_int32, _P]),
    "dgp_add_graph": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P, C.c_int32, _P, _P, C.c_int32, _P, _P, _P]),
    "dgp_set_priorities": (C.c_int, [_P, _P]),
    "dgp_remap_prefixes": (C.c_int, [_P, C.c_int32, _P, _P]),
    "dgp_graph_stimulus": (C.c_int, [_P, _P]),
    "dgp_graph_stimulus_ordered": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P, _P]),
    "dgp_reschedule": (C.c_int, [_P, C.c_int32, _P]),
    "dgp_release_tasks": (C.c_int, [_P, C.c_int64, _P, _P, _P]),
    "dgp_add_graph_deferred": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P, C.c_int32, _P, _P, C.c_int32, _P, _P]),
    "dgp_snapshot": (C.c_int, [_P]),
    "dgp_num_placements": (C.c_int64, [_P]),
    "dgp_get_placements": (C.c_int, [_P, C.c_int64, C.c_int64, _P, _P, _P, _P, _P, _P]),
    "dgp_task_messages": (C.c_int, [_P, C.c_int64, C.c_int64, _P, _P, _P, _P, _P, _P, _P]),
    "dgp_enable_snapshots": (C.c_int, [_P, C.c_int64]),
    "dgp_get_snapshots": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dgp_get_task_states": (C.c_int, [_P, _P]),
    "dgp_kernel_times": (C.c_int, [_P, _P, _P, C.c_int32]),
    "dgp_set_timing": (C.c_int, [_P, C.c_int]),
    "dgp_stats": (C.c_int, [_P, _P, C.c_int32]),
    "dgp_conflict_depth": (C.c_int, [C.c_int64, _P, _P, _P, C.c_int64, _P, _P, C.c_int64, _P, _P]),
    "dgp_steal_balance": (C.c_int, [_P, C.c_int32, _P, _P, _P, _P, _P, _P, C.c_double, C.c_int64, C.c_int64,
                                    C.c_int64, _P, _P, _P, _P, _P, C.c_int64, _P, _P, _P, _P, _P, _P, _P,
                                    _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dgp_steal_load": (C.c_int, [_P, C.c_int32, _P, _P, _P, _P, _P, _P, C.c_double, C.c_int64, C.c_int64,
                                 C.c_int64, _P, _P, _P, _P, _P, C.c_int64, _P, _P, _P, _P, _P, _P, _P,
                                 _P, _P, _P, _P]),
    "dgp_steal_thief_rows": (C.c_int, [_P, C.c_int64, C.c_int64]),
    "dgp_steal_row_bytes": (C.c_int64, []),
    "dgp_steal_pack_rows": (C.c_int, [_P, C.c_int64, C.c_int64, _P]),
    "dgp_steal_unpack_rows": (C.c_int, [_P, C.c_int64, C.c_int64, _P]),
    "dgp_steal_run": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dgp_add_replicas": (C.c_int, [_P, C.c_int64, _P, _P]),
    "dgp_remove_replicas": (C.c_int, [_P, C.c_int64, _P, _P]),
    "dgp_set_worker_status": (C.c_int, [_P, C.c_int32, C.c_int32, _P]),
    "dgp_long_running": (C.c_int, [_P, C.c_int32, C.c_double, _P]),
    "dgp_heartbeat": (C.c_int, [_P, C.c_double, C.c_int64, _P, _P]),
    "dgp_set_worker_flags": (C.c_int, [_P, C.c_int64, _P, _P, _P]),
    "dgp_set_wanted": (C.c_int, [_P, C.c_int64, _P, _P]),
    "dgp_task_erred": (C.c_int, [_P, C.c_int32, _P]),
    "dgp_remove_worker": (C.c_int, [_P, C.c_int32]),
    "dgp_lose_worker": (C.c_int, [_P, C.c_int32, C.c_int64, _P, C.c_int64, _P, _P]),
    "dgp_lose_worker_ordered": (C.c_int, [_P, C.c_int32, C.c_int64, _P, _P, C.c_int64, _P, C.c_int64, _P, _P, _P, _P,
                                          _P]),
    "dgp_steal_order": (C.c_int, [_P, C.c_int64, _P, _P]),
    "dgp_set_window": (C.c_int, [_P, C.c_int32]),
    "dgp_get_window": (C.c_int, [_P]),
    "dgp_sync_placements": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P, _P, _P]),
    "dgp_sync_tasks": (C.c_int, [_P, C.c_int64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dgp_sync_workers": (C.c_int, [_P, C.c_int32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "dgp_sync_globals": (C.c_int, [_P, C.c_int64, C.c_double, C.c_int32, _P, _P, C.c_int64, _P, _P, _P, C.c_double,
                                   _P, _P, _P]),
}

ABI_VERSION = 21
_libs: dict = {}


class DgpError(RuntimeError):
    pass


def load() -> C.CDLL:
    """Load libdgplace.so; raises if it was not built."""
    path = LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise DgpError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                       " (the HIP engine has no CPU fallback)")
    # One HIP runtime per process: torch bundles its own libamdhip64 (same soname,
    # libamdhip64.so.7, as /opt/rocm's), and a second runtime loaded beside an
    # initialised one sees no GPU. Importing torch first makes the engine bind to the
    # runtime torch uses, so engine pointers and torch device tensors (the all-gather
    # buffers of shard.py) live in one address space.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dgp_abi_version() != ABI_VERSION:
        raise DgpError(f"{os.path.basename(path)} ABI {lib.dgp_abi_version()} != {ABI_VERSION}")
    _libs[path] = lib
    return lib
