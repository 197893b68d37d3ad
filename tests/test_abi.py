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


class _WindowLib:
    """dgp_set_window / dgp_get_window of a library handle, recorded (no GPU)."""

    def __init__(self, window):
        self.window, self.calls = window, []

    def dgp_set_window(self, h, w):
        self.calls.append(w)
        self.window = w
        return 0

    def dgp_get_window(self, h):
        return self.window

    def dgp_update_restrictions(self, *a):
        return 0


def _engine_with(window, current):
    from distributed_amd.engine import PlacementEngine as PE

    e = object.__new__(PE)  # the host logic only: no device handle
    e.window, e.lib, e.h, e.n_tasks = window, _WindowLib(current), 1, 100
    return e


def test_later_graph_moves_an_auto_engine_to_the_64_slot_build():
    """engine.py later_graph_window / update_restrictions: the first later graph (or run-time
    restriction update) that wants the 64-slot build moves an "auto" engine there, once; a
    forced window never moves."""
    from distributed_amd import graphs

    plain = graphs.random_dag(2_000, 16, seed=1)
    restricted = graphs.restrict(plain, 0.1, seed=1)
    e = _engine_with("auto", 32)
    e.later_graph_window(plain)
    assert e.lib.calls == []
    e.later_graph_window(restricted)
    assert e.lib.calls == [64]
    e.later_graph_window(restricted)  # already there
    assert e.lib.calls == [64]
    e = _engine_with("auto", 32)
    e.update_restrictions([5], [[1, 2]], [1])
    assert e.lib.calls == [64]
    e = _engine_with("auto", 32)
    e.update_restrictions([5], [[1, 2]], [0])  # flags 0: nothing restricted
    assert e.lib.calls == []
    e = _engine_with(32, 32)  # forced
    e.later_graph_window(restricted)
    e.update_restrictions([5], [[1, 2]], [1])
    assert e.lib.calls == []
