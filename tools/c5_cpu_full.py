"""The C5 CPU baseline on the FULL graph (BASELINE.json configs[4]: map 8.75M + tree-reduce,
16,384 workers): oracle/replay.cpp (the 1-core port) replays it once; the placement digest is
checked against the GPU's pinned one (tests/golden/c5_full_digest.json). Test / measurement
infrastructure (imports the oracle): python tools/c5_cpu_full.py > profiles/<round>_c5_cpu_full.json"""
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from distributed_amd import graphs  # noqa: E402
from oracle import oracle  # noqa: E402

CONFIG = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
pin = json.load(open(os.path.join(REPO, "tests", "golden", "c5_full_digest.json")))
t0 = time.perf_counter()
g = graphs.map_tree_reduce(pin["n_map"], pin["n_workers"], seed=3)
t1 = time.perf_counter()
ref = oracle.replay(g, CONFIG, snapshots=False)
n = len(ref["pl_task"])
print(json.dumps({"leg": "c5 cpu baseline, full graph", "n_tasks": int(g["n_tasks"]), "n_workers": pin["n_workers"],
                  "placements": n, "seconds": round(ref["seconds"], 2),
                  "placements_per_s": round(n / ref["seconds"], 1), "cores": 1, "kind": "port",
                  "graph_seconds": round(t1 - t0, 1), "digest_matches_gpu_pin": graphs.placement_digest(ref) == pin["digest"],
                  "host": platform.processor() or platform.machine()}), flush=True)
