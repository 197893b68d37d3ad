"""Locate the first per-round snapshot difference between the engine and a fixture."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.engine import PlacementEngine  # noqa: E402
from oracle import oracle  # noqa: E402

name = sys.argv[1]
gold = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", name)
g, cfg, exp, meta = oracle.load_fixture(gold)
R = len(exp["round_nplaced"]) + 2
with PlacementEngine(0) as e:
    e.load(g, cfg, snapshots=R)
    e.replay()
    out = e.placements()
    out.update(e.snapshots(R))
n = min(len(out["round_nplaced"]), len(exp["round_nplaced"]))
cum = np.cumsum(exp["round_nplaced"])
for r in range(n):
    for k in ("round_nproc", "round_occ", "round_wnbytes", "round_idle", "round_sat", "round_itc", "round_nqueued", "round_nplaced"):
        a, b = np.asarray(out[k][r]), np.asarray(exp[k][r])
        if not np.array_equal(a, b):
            idx = np.nonzero(np.atleast_1d(a != b))[0]
            print(f"round {r} (placements up to {cum[r]}): {k} differs at {idx[:10]}: mine {np.atleast_1d(a)[idx[:5]]} ref {np.atleast_1d(b)[idx[:5]]}")
            if k.startswith("round_") and a.ndim:
                for w in idx[:3]:
                    print(f"   worker {w}: mine nproc {out['round_nproc'][r][w]} occ {out['round_occ'][r][w]!r} nb {out['round_wnbytes'][r][w]}"
                          f" | ref nproc {exp['round_nproc'][r][w]} occ {exp['round_occ'][r][w]!r} nb {exp['round_wnbytes'][r][w]}")
            sys.exit(0)
pl = out["pl_worker"]
print("rounds identical; first pl diff", np.nonzero(pl != exp["pl_worker"][: len(pl)])[0][:5])
