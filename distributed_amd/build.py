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
# the same sources with a 64-slot stimulus window and no wait-in-place claims: graphs with
# restrictions run this build (engine.py PlacementEngine.load)
OUT_W64 = os.path.join(PKG, "libdgplace_w64.so")
W64_FLAGS = ["-DDGP_WIN=64", "-DDGP_WAITC=0"]
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
    """Both builds, compiled side by side (and the ingestion pass); returns the default
    library's path."""
    build_ingest(force)
    newest = max(os.path.getmtime(p) for p in SRC + DEPS + [os.path.join(PKG, "..", "include", "dgplace.h")])
    jobs = []
    for out, extra in ((OUT, []), (OUT_W64, W64_FLAGS)):
        if not force and os.path.exists(out) and os.path.getmtime(out) >= newest:
            continue
        log = open(out + ".log", "w")  # one diagnostics file per job: the two never interleave
        jobs.append((out, log, subprocess.Popen([HIPCC, *FLAGS, *extra, "-o", out + ".tmp", *SRC],
                                                stdout=log, stderr=subprocess.STDOUT)))
    failed = []
    for out, log, proc in jobs:  # every job is waited for before anything is raised
        rc = proc.wait()
        log.close()
        if rc != 0:
            failed.append((out, rc))
    for out, log, proc in jobs:
        if any(out == f for f, _ in failed):
            if os.path.exists(out + ".tmp"):
                os.remove(out + ".tmp")
            continue
        os.replace(out + ".tmp", out)
        os.remove(out + ".log")
    if failed:
        out, rc = failed[0]
        msg = open(out + ".log").read()[-4000:]
        raise subprocess.CalledProcessError(rc, f"hipcc -> {out}", output=msg)
    return OUT


if __name__ == "__main__":
    print(build(force=True))
