import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.engine import PlacementEngine
from oracle import oracle
name, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
g, cfg, exp, meta = oracle.load_fixture(os.path.join("tests/golden", name))
with PlacementEngine(0) as e:
    e.load(g, cfg)
    e.replay()
    out = e.placements()
for i in range(a, min(b, len(out["pl_task"]))):
    m = (out["pl_task"][i], out["pl_worker"][i], out["pl_comm"][i], out["pl_start"][i], out["pl_wsnbytes"][i], out["pl_route"][i])
    r = (exp["pl_task"][i], exp["pl_worker"][i], exp["pl_comm"][i], exp["pl_start"][i], exp["pl_wsnbytes"][i], exp["pl_route"][i])
    print(i, "OK " if m == r else "BAD", m, r, "prefix", g["prefix_id"][r[0]], "deps", list(g["dep_idx"][g["dep_ptr"][r[0]]:g["dep_ptr"][r[0]+1]]))
