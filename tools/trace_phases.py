"""Executor phase latencies of sampled C2 stimuli (GPU, a DGP_TRACE=2 build):
DGP_LIB=distributed_amd/_var/lib_trace2.so python tools/trace_phases.py [lo] [n] [c3]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lo = int(sys.argv[1]) if len(sys.argv) > 1 else 400_000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000
os.environ["DGP_TRACE_LO"] = str(lo)
os.environ["DGP_TRACE_N"] = str(n)
from distributed_amd import graphs  # noqa: E402
from distributed_amd.engine import PlacementEngine  # noqa: E402

g = graphs.shuffle_graph(66_666, 512) if "c3" in sys.argv else graphs.random_dag(1_000_000, 1024, seed=0)
e = PlacementEngine(0)
e.load(g, {"saturation": 1.1})
e.reset()
e.update_graph()
e.run_rounds(-1)
buf = np.zeros(n * 32, np.uint64)
e.lib.dgp_debug_trace.argtypes = [C.c_void_p, C.c_void_p]
assert e.lib.dgp_debug_trace(e.h, buf.ctypes.data_as(C.c_void_p)) == 0
T = buf.reshape(n, 32).astype(np.int64)
T = T[(T[:, 2] > 0) & (T[:, 5] > 0) & (T[:, 0] > 0) & (T[:, 1] > 0) & (T[:, 3] > 0) & (T[:, 4] > 0) & (T[:, 6] > 0)]
seq = [("claimed -> precheck", 2, 0), ("precheck -> state loaded", 0, 1), ("loaded -> completion needs", 1, 3),
       ("needs -> occupancy + releases", 3, 4), ("releases -> frontier done", 4, 6), ("frontier -> done", 6, 5),
       ("claimed -> done", 2, 5)]
print(f"{len(T)} stimuli")
for name, a, b in seq:
    v = (T[:, b] - T[:, a]).astype(np.float64)
    print(f"  {name:32s} mean {v.mean():8.0f} p50 {np.percentile(v, 50):8.0f} p90 {np.percentile(v, 90):8.0f}")
