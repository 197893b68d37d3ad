"""Build the HIP engine (``libdgplace.so``, gfx950) in-tree with hipcc."""
from __future__ import annotations

import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
SRC = [os.path.join(PKG, "csrc", "dgplace.hip")]
DEPS = [os.path.join(PKG, "csrc", "dgp_device.h"), os.path.join(PKG, "csrc", "dgp_stream.h"),
        os.path.join(PKG, "csrc", "dgp_steal.h"), os.path.join(PKG, "csrc", "dgp_service.h"),
        os.path.join(PKG, "csrc", "dgp_events.h"), os.path.join(PKG, "csrc", "dgp_svcmsg.h"),
        os.path.join(PKG, "csrc", "dgp_msgs.h")]
OUT = os.path.join(PKG, "libdgplace.so")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
# -ffp-contract=off: no fused multiply-add, so fp64 results round exactly like the
# reference's CPython arithmetic (the parity contract is bit-exact objectives).
# module-wide LDS lowering: the stream roles run out of line (one register budget each) and
# reach the engine's LDS blocks at fixed addresses, not through a per-kernel offset table
# re-read (scalar load + lgkmcnt wait) on every access.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-shared",
         "-Wall", "-mllvm", "-amdgpu-lower-module-lds-strategy=module"]


# the extension's graph ingestion pass (host C against the stable Python ABI; ext.py loads
# it with ctypes.PyDLL): one build for any CPython >= 3.9
INGEST_SRC = os.path.join(PKG, "csrc", "dgp_ingest.c")
INGEST_OUT = os.path.join(PKG, "libdgpingest.so")


def build_ingest(force: bool = False) -> str:
    import sysconfig

    if force or not os.path.exists(INGEST_OUT) or os.path.getmtime(INGEST_OUT) < os.path.getmtime(INGEST_SRC):
        subprocess.run([shutil.which("gcc") or "cc", "-O2", "-Wall", "-shared", "-fPIC",
                        "-I" + sysconfig.get_paths()["include"], "-o", INGEST_OUT + ".tmp", INGEST_SRC],
                       check=True, capture_output=True, text=True)
        os.replace(INGEST_OUT + ".tmp", INGEST_OUT)
    return INGEST_OUT


def build(force: bool = False) -> str:
    """The engine library (both stream-window builds in one: dgp_stream.h is included twice)
    and the ingestion pass; returns the library's path."""
    try:  # optional: ext.py falls back to its Python ingestion passes without it
        build_ingest(force)
    except (OSError, subprocess.CalledProcessError) as e:
        out = getattr(e, "stderr", None) or getattr(e, "output", None) or ""
        print(f"dgplace build: graph ingestion library not built ({e}){': ' + out[-2000:] if out else ''}")
    stale = os.path.join(PKG, "libdgplace_w64.so")  # the separate 64-slot build of ABI <= 18
    if os.path.exists(stale):
        os.remove(stale)
    newest = max(os.path.getmtime(p) for p in SRC + DEPS + [os.path.join(PKG, "..", "include", "dgplace.h")])
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= newest:
        return OUT
    r = subprocess.run([HIPCC, *FLAGS, "-o", OUT + ".tmp", *SRC], capture_output=True, text=True)
    if r.returncode != 0:
        if os.path.exists(OUT + ".tmp"):
            os.remove(OUT + ".tmp")
        raise subprocess.CalledProcessError(r.returncode, f"hipcc -> {OUT}", output=(r.stdout + r.stderr)[-4000:])
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True))
