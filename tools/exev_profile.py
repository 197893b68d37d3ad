"""exe_v phase split (GPU, a DGP_TRACE=3 build): DGP_LIB=tools/_var/lib_trace3.so python tools/exev_profile.py [lo] [n]"""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lo = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000
os.environ["DGP_TRACE_LO"], os.environ["DGP_TRACE_N"] = str(lo), str(n)
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
g = graphs.random_dag(int(os.environ.get("N", 300_000)), 1024, seed=0)
e = PlacementEngine(0, window=32)
e.load(g, {"saturation": 1.1})
e.reset(); e.update_graph(); e.run_rounds(-1)
buf = np.zeros(n * 32, np.uint64)
e.lib.dgp_debug_trace.argtypes = [C.c_void_p, C.c_void_p]
assert e.lib.dgp_debug_trace(e.h, buf.ctypes.data_as(C.c_void_p)) == 0
T = buf.reshape(n, 32).astype(np.int64)
seq = [(2, 8, "claim->state+precheck"), (8, 10, "completion find"), (10, 11, "->wait"), (11, 12, "wait"),
       (12, 13, "writes+occ+rec+rel"), (13, 14, "argmin"), (14, 24, "place+line_all"), (24, 25, "needs vec"),
       (25, 26, "dict inc"), (26, 27, "occ"), (27, 15, "rec"), (15, 16, "more frontier"), (16, 17, "wb+release"),
       (17, 18, "refill+w release"), (18, 29, "flush+finish"), (2, 29, "TOTAL claim->finish")]
ok = (T[:, 2] > 0) & (T[:, 29] > 0) & (T[:, 8] > 0) & (T[:, 30] == 1)
print(f"exe_v finished {int((T[:, 30] == 1).sum())} of {n}")
print(f"{ok.sum()} of {n} via exe_v; nf mean {np.mean(T[ok, 22] & 0xff):.2f}")
for a, b, nm in seq:
    sel = ok & (T[:, a] > 0) & (T[:, b] > 0)
    d = T[sel, b] - T[sel, a]
    if len(d):
        print(f"  {nm:24s} n {len(d):6d} mean {d.mean():8.0f} p50 {np.percentile(d, 50):8.0f} p90 {np.percentile(d, 90):8.0f}")
