"""Regenerate tests/golden/c5_full_digest.json: the oracle's placement-log digest of the
full BASELINE.json C5 replay (10M tasks x 16,384 workers; ~6 min on one host core).

    python tools/c5_digest.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import c5_run  # noqa: E402
from distributed_amd import graphs  # noqa: E402
from oracle import oracle  # noqa: E402

M, W = 8_750_000, 16_384
g = graphs.map_tree_reduce(M, W)
r = oracle.replay(g, c5_run.CFG, snapshots=False)
out = {"n_map": M, "n_workers": W, "n_placements": int(len(r["pl_task"])), "digest": c5_run.digest(r),
       "oracle_s": round(r["seconds"], 1), "config": c5_run.CFG,
       "generator": "tools/c5_digest.py (digest = tools/c5_run.py:digest over the six placement arrays)"}
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                    "c5_full_digest.json")
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out))
