"""BASELINE.json C5 (map + tree-reduce, fan-in 8) on the device: replay time and a
digest of the placement log; --check also replays the oracle and compares.

    python tools/c5_run.py N_MAP N_WORKERS [--check]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs  # noqa: E402
from distributed_amd.engine import PlacementEngine  # noqa: E402

CFG = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
KEYS = graphs.PLACEMENT_KEYS
digest = graphs.placement_digest


def main():
    m, W = int(sys.argv[1]), int(sys.argv[2])
    g = graphs.map_tree_reduce(m, W)
    e = PlacementEngine(0)
    t0 = time.perf_counter()
    e.load(g, CFG)
    t1 = time.perf_counter()
    e.set_timing(True)
    e.reset()
    e.update_graph()
    e.run_rounds(-1)
    kt = e.kernel_times()
    t2 = time.perf_counter()
    out = e.placements()
    res = {"n_map": m, "n_tasks": int(g["n_tasks"]), "n_workers": W, "load_s": round(t1 - t0, 2),
           "replay_s": round(t2 - t1, 3), "placements": int(len(out["pl_task"])),
           "rounds": int(e.stats()["rounds"]), "kernels_ms": {k: round(v[0], 2) for k, v in kt.items()},
           "digest": digest(out)}
    res["placements_per_s"] = round(res["placements"] / res["replay_s"], 1)
    print(json.dumps(res), flush=True)
    if "--check" in sys.argv:
        from oracle import oracle

        ref = oracle.replay(g, CFG, snapshots=False)
        same = {k: bool(np.array_equal(out[k], ref[k])) for k in KEYS}
        print(json.dumps({"oracle_s": round(ref["seconds"], 2), "same": same, "oracle_digest": digest(ref)}), flush=True)
        if not all(same.values()):
            sys.exit(1)
    e.close()


if __name__ == "__main__":
    main()
