"""Executor phase breakdown of a DGP_PHASE_PROBES=1 build (diagnostic, GPU):
DGP_LIB=distributed_amd/_var/lib_probe.so python tools/stream_phases.py"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
n = 1_000_000
g = graphs.random_dag(n, 1024, seed=0)
e = PlacementEngine(0)
e.load(g, {"saturation": 1.1})
for it in range(2):
    e.reset(); e.update_graph(); t = time.time(); e.run_rounds(-1); dt = time.time() - t
st = e.stats()
P = {i: st[f"wave_phase{i}"] for i in range(16)}
for i, k in enumerate(("cyc_setup", "cyc_local_steps", "cyc_global", "cyc_finish", "cyc_reserve", "cyc_max_step", "cyc_exec_max", "cyc_exec_sum")):
    P[16 + i] = st[k]
names = {11: "precheck", 16: "load state", 17: "completion needs_dec", 12: "occ + releases", 18: "frontier cand/comm",
         19: "frontier argmin", 20: "frontier commit", 13: "writeback+release+refill", 21: "(empty)", 14: "replica bookkeeping",
         15: "finish_slot", 22: "finish fence"}
print(f"{dt:.3f}s {e.num_placements() / dt / 1e6:.3f} M/s; exe claim->retire per stimulus {P[5] / n:.0f}")
for i in (11, 16, 17, 12, 18, 19, 20, 13, 21, 14, 15, 22):
    print(f"  [{i:2d}] {names[i]:28s} per stimulus {P[i] / n:8.1f}")
