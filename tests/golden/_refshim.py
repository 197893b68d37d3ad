"""Import shim that lets the reference's ``distributed.scheduler`` / ``distributed.stealing``
import unmodified under the image's python3.9 (dask 2021.10).

Test infrastructure only (used by ``gen_golden.py`` in this container; never on the
GPU box, never by the product). The reference pins dask 2024.3.1
(``/root/reference/pyproject.toml:31``); the names below are the only ones it needs
that dask 2021.10 lacks, and none of them is on the placement path:

* ``dask.typing.Key / NoDefault / no_default``  — type annotations only
* ``dask.core.iskey / validate_key``            — ``Scheduler.validate_key`` (validate=True only)
* ``dask.utils.shorten_traceback``, ``dask.utils.is_namedtuple_instance``,
  ``dask.base.TokenizationError``               — client/protocol code paths
"""
import sys
import types

REFERENCE = "/root/reference"


def install():
    import dask
    import dask.base
    import dask.core
    import dask.utils
    from typing import Hashable

    if "dask.typing" not in sys.modules:
        m = types.ModuleType("dask.typing")
        m.Key = Hashable

        class NoDefault:
            pass

        m.NoDefault = NoDefault
        m.no_default = NoDefault()
        sys.modules["dask.typing"] = m
        dask.typing = m

    def iskey(k):
        if type(k) is tuple:
            return all(iskey(i) for i in k)
        return type(k) in {bytes, int, float, str}

    def validate_key(k):
        if not iskey(k):
            raise TypeError(f"Unexpected key type {type(k)} (value: {k!r})")

    dask.core.iskey = iskey
    dask.core.validate_key = validate_key
    if not hasattr(dask.utils, "shorten_traceback"):
        dask.utils.shorten_traceback = lambda *a, **k: None
    if not hasattr(dask.utils, "is_namedtuple_instance"):
        dask.utils.is_namedtuple_instance = lambda o: isinstance(o, tuple) and hasattr(o, "_fields")
    if not hasattr(dask.base, "TokenizationError"):
        class TokenizationError(RuntimeError):
            pass
        dask.base.TokenizationError = TokenizationError
    if sys.path[0] != REFERENCE:
        sys.path.insert(0, REFERENCE)
