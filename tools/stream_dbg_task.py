import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.engine import PlacementEngine
from oracle import oracle
name, pl = sys.argv[1], int(sys.argv[2])
g, cfg, exp, meta = oracle.load_fixture(os.path.join("tests/golden", name))
x = int(exp["pl_task"][pl])
os.environ["DGP_DEBUG_TASK"] = str(x)
with PlacementEngine(0) as e:
    e.load(g, cfg)
    e.replay()
    buf = np.zeros(64 * 8)
    e.lib.dgp_debug_buf.argtypes = [C.c_void_p, C.c_void_p]
    e.lib.dgp_debug_buf(e.h, buf.ctypes.data_as(C.c_void_p))
    out = e.placements()
print("task", x, "ref worker", exp["pl_worker"][pl], "ref start", repr(exp["pl_start"][pl]), "mine", out["pl_worker"][pl], repr(out["pl_start"][pl]))
b = buf.reshape(64, 8)
for row in b:
    if row[1] != 0:
        print(" cand %d start %r nb %d comm %d occ %r nproc %d netocc %d plen %d stim %d" % (row[0], row[1], row[2], row[3], row[4], row[5], row[6], int(row[7]) % 100, int(row[7]) // 100))
