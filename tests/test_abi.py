"""The C ABI: libdgplace.so loads and exports exactly what include/dgplace.h declares.
CPU-only (no compute calls without a GPU)."""
import os
import re

import pytest

from conftest import REPO
from distributed_amd import _lib

HEADER = os.path.join(REPO, "include", "dgplace.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dgp_[a-z_]+)\s*\(", src)))


@pytest.mark.parametrize("window", [32, 64])
def test_library_exports_every_declared_symbol(window):
    lib = _lib.load(window)  # libdgplace.so and the 64-slot window build libdgplace_w64.so
    names = declared()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_lib.SIGNATURES) == declared()


def test_abi_version():
    assert _lib.load().dgp_abi_version() == _lib.ABI_VERSION
    assert _lib.load(64).dgp_abi_version() == _lib.ABI_VERSION


def test_create_without_gpu_returns_null_or_engine():
    import torch

    lib = _lib.load()
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    assert not lib.dgp_create(0)
