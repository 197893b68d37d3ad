"""ORACLE (test infrastructure, not product code): ctypes binding of ``liborc_replay.so``,
the CPU restatement of the reference placement replay (see ``replay.cpp``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
import this module — as the checker / the timed CPU baseline, never as the product.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborc_replay.so")

_P = C.c_void_p


class OrcGraph(C.Structure):
    _fields_ = [
        ("n_tasks", C.c_int64), ("n_workers", C.c_int64), ("n_prefixes", C.c_int64), ("n_groups", C.c_int64),
        ("dep_ptr", _P), ("dep_idx", _P), ("prio", _P), ("prefix_id", _P), ("group_id", _P),
        ("wanted", _P), ("rootish_override", _P), ("nbytes", _P), ("start", _P), ("stop", _P),
        ("nthreads", _P), ("group_prefix", _P), ("prefix_default_dur", _P),
        ("bandwidth", C.c_int64), ("default_data_size", C.c_int64), ("unknown_duration", C.c_double),
        ("saturation", C.c_double), ("restr_ptr", _P), ("restr_idx", _P), ("restr_flags", _P),
        ("n_joins", C.c_int64), ("join_before", _P), ("join_nthreads", _P),
        ("next", _P), ("next_before", C.c_int64),
    ]


class OrcResult(C.Structure):
    _fields_ = [
        ("pl_task", _P), ("pl_worker", _P), ("pl_comm", _P), ("pl_start", _P), ("pl_wsnbytes", _P),
        ("pl_route", _P), ("n_placements", C.c_int64),
        ("max_rounds", C.c_int64), ("snap_stride", C.c_int64), ("n_rounds", C.c_int64), ("round_nplaced", _P), ("round_occ", _P),
        ("round_wnbytes", _P), ("round_nproc", _P), ("round_idle", _P), ("round_sat", _P), ("round_itc", _P),
        ("round_nqueued", _P), ("final_state", _P), ("seconds", C.c_double), ("error", C.c_char * 256),
    ]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_replay.argtypes = [C.POINTER(OrcGraph), C.POINTER(OrcResult)]
        _lib.orc_replay.restype = C.c_int
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def replay(g: dict, config: dict, *, snapshots: bool = True, max_rounds: int | None = None,
           joins: tuple | None = None, second: tuple | None = None) -> dict:
    """Replay graph ``g`` (graph dict, ``distributed_amd/graphs.py``) under ``config``
    ({bandwidth, default_data_size, unknown_duration, saturation}) and return the
    placement records + per-round snapshots as numpy arrays. ``joins``: (before, nthreads)
    arrays of workers joining before the given completion (0-based, replay order); the
    snapshots are then as wide as the final worker count. ``second``: (graph dict, before)
    — a later, independent graph (engine-wide prefix / group ids, priorities after ``g``'s)
    submitted before the given completion; its tasks follow ``g``'s in the outputs."""
    n = int(g["n_tasks"])
    w0 = len(g["nthreads"])
    w = w0 + (len(joins[0]) if joins is not None else 0)
    sat = config["saturation"]
    sat = math.inf if sat == "inf" else float(sat)
    keep = []

    def arr(x, dt):
        a = np.ascontiguousarray(x, dtype=dt)
        keep.append(a)
        return a

    gs = OrcGraph(
        n_tasks=n, n_workers=w0, n_prefixes=len(g["prefix_default_dur"]), n_groups=len(g["group_prefix"]),
        dep_ptr=_ptr(arr(g["dep_ptr"], np.int64)), dep_idx=_ptr(arr(g["dep_idx"], np.int32)),
        prio=_ptr(arr(g["prio"], np.int64)), prefix_id=_ptr(arr(g["prefix_id"], np.int32)),
        group_id=_ptr(arr(g["group_id"], np.int32)), wanted=_ptr(arr(g["wanted"], np.uint8)),
        rootish_override=_ptr(arr(g["rootish_override"], np.int8)), nbytes=_ptr(arr(g["nbytes"], np.int64)),
        start=_ptr(arr(g["start"], np.float64)), stop=_ptr(arr(g["stop"], np.float64)),
        nthreads=_ptr(arr(g["nthreads"], np.int32)), group_prefix=_ptr(arr(g["group_prefix"], np.int32)),
        prefix_default_dur=_ptr(arr(g["prefix_default_dur"], np.float64)),
        bandwidth=int(config["bandwidth"]), default_data_size=int(config["default_data_size"]),
        unknown_duration=float(config["unknown_duration"]), saturation=sat,
    )
    gs2 = None
    if second is not None:
        h, before = second
        gs2 = OrcGraph(
            n_tasks=len(h["prio"]), n_workers=w0, n_prefixes=len(h["prefix_default_dur"]),
            n_groups=len(h["group_prefix"]), dep_ptr=_ptr(arr(h["dep_ptr"], np.int64)),
            dep_idx=_ptr(arr(h["dep_idx"], np.int32)), prio=_ptr(arr(h["prio"], np.int64)),
            prefix_id=_ptr(arr(h["prefix_id"], np.int32)), group_id=_ptr(arr(h["group_id"], np.int32)),
            wanted=_ptr(arr(h["wanted"], np.uint8)), rootish_override=_ptr(arr(h["rootish_override"], np.int8)),
            nbytes=_ptr(arr(h["nbytes"], np.int64)), start=_ptr(arr(h["start"], np.float64)),
            stop=_ptr(arr(h["stop"], np.float64)), prefix_default_dur=_ptr(arr(h["prefix_default_dur"], np.float64)),
        )
        gs.next = C.cast(C.pointer(gs2), C.c_void_p)
        gs.next_before = int(before)
        n += len(h["prio"])
    if joins is not None:
        gs.n_joins = len(joins[0])
        gs.join_before = _ptr(arr(joins[0], np.int64))
        gs.join_nthreads = _ptr(arr(joins[1], np.int32))
    if g.get("restr_flags") is not None:  # worker restrictions, resolved to indices (graphs.restrict)
        gs.restr_ptr = _ptr(arr(g["restr_ptr"], np.int64))
        gs.restr_idx = _ptr(arr(g["restr_idx"], np.int32))
        gs.restr_flags = _ptr(arr(g["restr_flags"], np.uint8))
    R = int(max_rounds or (n + 2))
    out = dict(
        pl_task=np.zeros(n, np.int32), pl_worker=np.zeros(n, np.int32), pl_comm=np.zeros(n, np.int64),
        pl_start=np.zeros(n, np.float64), pl_wsnbytes=np.zeros(n, np.int64), pl_route=np.zeros(n, np.int8),
        round_nplaced=np.zeros(R, np.int32), final_state=np.zeros(n, np.uint8),
    )
    res = OrcResult(pl_task=_ptr(out["pl_task"]), pl_worker=_ptr(out["pl_worker"]), pl_comm=_ptr(out["pl_comm"]),
                    pl_start=_ptr(out["pl_start"]), pl_wsnbytes=_ptr(out["pl_wsnbytes"]),
                    pl_route=_ptr(out["pl_route"]), max_rounds=R, snap_stride=w, round_nplaced=_ptr(out["round_nplaced"]),
                    final_state=_ptr(out["final_state"]))
    if snapshots:
        snap = dict(round_occ=np.zeros((R, w)), round_wnbytes=np.zeros((R, w), np.int64),
                    round_nproc=np.zeros((R, w), np.int32), round_idle=np.zeros((R, w), np.uint8),
                    round_sat=np.zeros((R, w), np.uint8), round_itc=np.zeros((R, w), np.uint8),
                    round_nqueued=np.zeros(R, np.int32))
        out.update(snap)
        for k, v in snap.items():
            setattr(res, k, _ptr(v))
    rc = lib().orc_replay(C.byref(gs), C.byref(res))
    if rc != 0:
        raise RuntimeError("oracle replay failed: " + res.error.decode())
    np_ = int(res.n_placements)
    nr = int(res.n_rounds)
    for k in ("pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route"):
        out[k] = out[k][:np_]
    for k in list(out):
        if k.startswith("round_"):
            out[k] = out[k][:nr]
    out["seconds"] = float(res.seconds)
    out["n_rounds"] = nr
    return out


def load_fixture(path: str):
    """Load a ``tests/golden/*.npz`` fixture -> (graph dict, config, expected outputs)."""
    import json

    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    g = {k: z[k] for k in ("dep_ptr", "dep_idx", "prio", "prefix_id", "group_id", "wanted", "rootish_override",
                           "nbytes", "start", "stop", "nthreads", "group_prefix", "prefix_default_dur")}
    for k in ("restr_ptr", "restr_idx", "restr_flags"):
        if k in z.files:
            g[k] = z[k]
    g["n_tasks"] = len(g["prio"])
    g["prefix_names"] = meta["prefix_names"]
    g["group_names"] = meta["group_names"]
    g["name"] = meta["name"]
    exp = {k: z[k] for k in z.files if k.startswith(("pl_", "round_", "final_", "stim_"))}
    return g, meta["config"], exp, meta


# ----------------------------------------------------------------- WorkStealing
STEAL_INPUTS = ("nthreads", "occ", "nproc", "wnbytes", "idle", "sat", "victim", "duration", "fast", "dep_ptr",
                "dep_idx", "data_nbytes", "data_get_nbytes", "data_holder")


def holder_csr(data_holder):
    """who_has of each data task as CSR (a single holder, or none when released)."""
    h = np.asarray(data_holder, np.int32)
    ptr = np.zeros(len(h) + 1, np.int64)
    ptr[1:] = np.cumsum(h >= 0)
    return ptr, h[h >= 0].astype(np.int32)


def steal_balance(p: dict) -> dict:
    """steal_time_ratio for every task + one WorkStealing.balance() over problem ``p``
    (the input arrays of a ``tests/golden/steal_*.npz`` fixture)."""
    L = lib()
    fn = L.orc_steal_balance
    W = len(p["nthreads"])
    T = len(p["victim"])
    keep = []

    def a(x, dt):
        v = np.ascontiguousarray(x, dtype=dt)
        keep.append(v)
        return _ptr(v)

    if "holder_ptr" in p:  # who_has with any number of holders
        hptr, hidx = np.asarray(p["holder_ptr"], np.int64), np.asarray(p["holder_idx"], np.int32)
    else:
        hptr, hidx = holder_csr(p["data_holder"])
    out = dict(level=np.zeros(T, np.int8), st_task=np.zeros(T, np.int32), st_victim=np.zeros(T, np.int32),
               st_thief=np.zeros(T, np.int32), st_level=np.zeros(T, np.int32), st_cost=np.zeros(T),
               st_occ_victim=np.zeros(T), st_occ_thief=np.zeros(T), inflight_occ=np.zeros(W),
               inflight_tasks=np.zeros(W, np.int32), idle_after=np.zeros(W, np.uint8), sat_after=np.zeros(W, np.uint8),
               checked=np.zeros(W, np.uint8))
    n = C.c_int64(0)
    fn.restype = C.c_int
    rc = fn(C.c_int32(W), a(p["nthreads"], np.int32), a(p["occ"], np.float64), a(p["nproc"], np.int32),
            a(p["wnbytes"], np.int64), a(p["idle"], np.uint8), a(p["sat"], np.uint8), C.c_double(float(p["total_occ"])),
            C.c_int64(int(p["total_nthreads"])), C.c_int64(int(p["bandwidth"])), C.c_int64(T),
            a(p["victim"], np.int32), a(p["duration"], np.float64), a(p["fast"], np.uint8), a(p["dep_ptr"], np.int64),
            a(p["dep_idx"], np.int32), a(p["data_nbytes"], np.int64), a(p["data_get_nbytes"], np.int64),
            a(hptr, np.int64), a(hidx, np.int32),
            *((a(p["restr_ptr"], np.int64), a(p["restr_idx"], np.int32), a(p["restr_flags"], np.uint8))
              if p.get("restr_flags") is not None else (None, None, None)),
            a(p["level_in"], np.int8) if p.get("level_in") is not None else None,
            a(p["inflight_occ_in"], np.float64) if p.get("inflight_occ_in") is not None else None,
            a(p["inflight_tasks_in"], np.int32) if p.get("inflight_tasks_in") is not None else None,
            *[_ptr(out[k]) for k in ("level", "st_task", "st_victim", "st_thief", "st_level", "st_cost",
                                     "st_occ_victim", "st_occ_thief")],
            C.byref(n), *[_ptr(out[k]) for k in ("inflight_occ", "inflight_tasks", "idle_after", "sat_after",
                                                 "checked")])
    if rc != 0:
        raise RuntimeError(f"oracle steal_balance failed ({rc})")
    k = int(n.value)
    for key in ("st_task", "st_victim", "st_thief", "st_level", "st_cost", "st_occ_victim", "st_occ_thief"):
        out[key] = out[key][:k]
    return out


def load_steal_fixture(path: str):
    """Load a ``tests/golden/steal_*.npz`` fixture -> (problem inputs, expected outputs, meta)."""
    import json

    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    p = {k: z[k] for k in STEAL_INPUTS}
    for k in ("total_occ", "total_nthreads", "bandwidth"):
        p[k] = z[k][()]
    for k in ("holder_ptr", "holder_idx", "restr_ptr", "restr_idx", "restr_flags"):
        if k in z.files:
            p[k] = z[k]
    exp = {k: z[k] for k in ("level", "st_task", "st_level", "st_cost", "st_victim", "st_occ_victim", "st_thief",
                             "st_occ_thief", "inflight_occ", "inflight_tasks", "idle_after", "sat_after")}
    return p, exp, meta


def load_steal_problems(path: str):
    """Load a multi-problem steal fixture (``tests/golden/steal_reftests.npz``,
    ``gen_steal_ref.py``) -> list of (name, problem inputs, expected outputs)."""
    import json

    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    out = []
    for k, name in enumerate(meta["problems"]):
        p = {key: z[f"p{k}__{key}"] for key in STEAL_INPUTS + ("holder_ptr", "holder_idx")}
        for key in ("total_occ", "total_nthreads", "bandwidth"):
            p[key] = z[f"p{k}__{key}"][()]
        exp = {key: z[f"p{k}__{key}"] for key in ("level", "st_task", "st_level", "st_cost", "st_victim",
                                                  "st_occ_victim", "st_thief", "st_occ_thief", "inflight_occ",
                                                  "inflight_tasks", "idle_after", "sat_after")}
        out.append((name, p, exp))
    return out
