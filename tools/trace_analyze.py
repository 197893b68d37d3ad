"""Lifecycle of sampled stimuli in the C2 replay (GPU, a DGP_TRACE=1 build):
DGP_LIB=distributed_amd/_var/lib_trace.so python tools/trace_analyze.py [lo] [n] [c3]
Per stimulus (s_memtime ticks): registered -> ready (waiting for predecessors), ready ->
claimed (waiting for an executor), claimed -> non-w release / done, done -> retired (SEQ)."""
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
ok = (T[:, 0] > 0) & (T[:, 1] > 0) & (T[:, 2] > 0) & (T[:, 5] > 0) & (T[:, 6] > 0)
T = T[ok]
pred = T[:, 7] & 0xFFFF
nt = (T[:, 7] >> 16) & 0xFF
wave = (T[:, 7] >> 24) & 0xFF


def st(name, v):
    v = v.astype(np.float64)
    print(f"  {name:34s} mean {v.mean():9.0f}  p50 {np.percentile(v, 50):9.0f}  p90 {np.percentile(v, 90):9.0f}")


span = (T[:, 6].max() - T[:, 0].min())
print(f"{len(T)} stimuli traced, {span / len(T):.0f} ticks per stimulus wall")
st("registered -> ready", T[:, 1] - T[:, 0])
st("ready -> claimed", T[:, 2] - T[:, 1])
st("claimed -> non-w release", T[:, 4] - T[:, 2])
early = T[:, 3] > 0
if early.any():
    st("claimed -> early release (when done)", (T[early, 3] - T[early, 2]))
st("claimed -> done", T[:, 5] - T[:, 2])
st("done -> retired", T[:, 6] - T[:, 5])
st("registered -> retired (residence)", T[:, 6] - T[:, 0])
print(f"  predecessors at registration: mean {pred.mean():.2f}, zero {np.mean(pred == 0) * 100:.1f}%")
print(f"  touched workers: mean {nt.mean():.2f}")
# critical path: for ready events caused by a predecessor's release, the gap between the
# predecessor's release and this claim
for w in sorted(set(wave.tolist())):
    sel = wave == w
    print(f"  wave {w:2d}: {sel.sum():6d} stimuli, exec mean {np.mean(T[sel, 5] - T[sel, 2]):.0f}")
