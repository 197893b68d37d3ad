"""The C ABI: libdgplace.so loads and exports exactly what include/dgplace.h declares.
CPU-only (no compute calls without a GPU)."""
import os
import re

import numpy as np
import pytest

from conftest import REPO
from distributed_amd import _lib

HEADER = os.path.join(REPO, "include", "dgplace.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dgp_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()  # both stream-window builds live in it (dgp_set_window)
    names = declared()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_lib.SIGNATURES) == declared()


def test_abi_version():
    assert _lib.load().dgp_abi_version() == _lib.ABI_VERSION


def test_create_without_gpu_returns_null_or_engine():
    import torch

    lib = _lib.load()
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    assert not lib.dgp_create(0)


def test_auto_window_choice():
    """PlacementEngine.auto_window (engine.py): 64 for restrictions or a task with at least
    WIDE_FRONTIER dependents, else 32."""
    from distributed_amd import graphs
    from distributed_amd.engine import PlacementEngine as PE

    g = graphs.random_dag(20_000, 64, seed=1)
    assert PE.auto_window(g) == 32
    assert PE.auto_window(graphs.restrict(g, 0.1, seed=1)) == 64
    assert PE.auto_window(graphs.shuffle_graph(PE.WIDE_FRONTIER, 64)) == 64  # the barrier's fan-out
    assert PE.auto_window(graphs.shuffle_graph(PE.WIDE_FRONTIER // 4, 64)) == 32
    g2 = dict(g, restr_flags=np.zeros(g["n_tasks"], np.uint8))  # flags present, nothing restricted
    assert PE.auto_window(g2) == 32


@pytest.mark.parametrize("bad", [48, 128, 0, "64"])
def test_window_is_validated(bad):
    from distributed_amd.engine import PlacementEngine as PE

    with pytest.raises(ValueError):
        PE(0, window=bad)
