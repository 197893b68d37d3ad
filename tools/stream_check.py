"""Quick GPU check of the stream engine: fixtures + random DAGs vs the oracle, then timing."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs  # noqa: E402
from distributed_amd.engine import PlacementEngine  # noqa: E402
from oracle import oracle  # noqa: E402

PL = ("pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route")
RK = ("round_nplaced", "round_occ", "round_wnbytes", "round_nproc", "round_idle", "round_sat", "round_itc", "round_nqueued")


def cmp(out, exp, keys):
    bad = []
    for k in keys:
        a, b = np.asarray(out[k]), np.asarray(exp[k])
        if a.shape != b.shape:
            bad.append(f"{k}: shape {a.shape} vs {b.shape}")
            continue
        idx = np.nonzero(a.reshape(-1) != b.reshape(-1))[0]
        if len(idx):
            bad.append(f"{k}: {len(idx)} diffs, first {idx[0]}: {a.reshape(-1)[idx[0]]!r} vs {b.reshape(-1)[idx[0]]!r}")
    return bad


which = sys.argv[1] if len(sys.argv) > 1 else "all"
gold = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
if which in ("all", "fix"):
    for f in sorted(os.listdir(gold)):
        if not f.endswith(".npz") or f.startswith("steal_"):
            continue
        g, cfg, exp, meta = oracle.load_fixture(os.path.join(gold, f))
        R = len(exp["round_nplaced"]) + 2
        t = time.time()
        with PlacementEngine(0) as e:
            e.load(g, cfg, snapshots=R)
            try:
                e.replay()
                out = e.placements()
                out.update(e.snapshots(R))
                bad = cmp(out, exp, PL + RK)
                st = e.task_states()
                if not np.array_equal(st, exp["final_state"]):
                    bad.append("final_state")
            except Exception as ex:  # noqa: BLE001
                st = e.stats()
                bad = [f"EXC {ex}", "seq reg pre bld log ready busy gpend flags pred sid done walk rec qlen rend",
                       [st[f"wave_phase{i}"] for i in range(16)]]
        print(f"{f:28s} {'OK ' if not bad else 'BAD'} {time.time() - t:6.2f}s {bad[:3]}", flush=True)
if which in ("all", "rnd"):
    for n, w, sat in ((100_000, 1024, 1.1), (100_000, 1024, "inf"), (30_000, 4096, 1.1)):
        g = graphs.random_dag(n, w, seed=42)
        cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": sat}
        ref = oracle.replay(g, cfg, snapshots=False)
        with PlacementEngine(0) as e:
            e.load(g, cfg)
            t = time.time()
            try:
                e.replay()
                dt = time.time() - t
                bad = cmp(e.placements(), ref, PL)
            except Exception as ex:  # noqa: BLE001
                dt, bad = time.time() - t, [f"EXC {ex}"]
            st = e.stats()
        print(f"rnd {n} {w} {sat}: {'OK ' if not bad else 'BAD'} {dt:.3f}s {n / dt / 1e6:.2f} M/s {bad[:3]} prof={st}", flush=True)
if which in ("all", "big"):
    g = graphs.random_dag(1_000_000, 1024, seed=0)
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
    with PlacementEngine(0) as e:
        e.load(g, cfg)
        for i in range(3):
            e.reset()
            t = time.time()
            e.update_graph()
            e.run_rounds(-1)
            n = e.num_placements()
            dt = time.time() - t
            print(f"1M: {n} placements {dt:.3f}s {n / dt / 1e6:.3f} M/s stats={e.stats()}", flush=True)
        out = e.placements()
    ref = oracle.replay(g, cfg, snapshots=False)
    print("1M parity:", cmp(out, ref, PL) or "OK", flush=True)
