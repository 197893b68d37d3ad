"""Stimulus lifecycle breakdown of a DGP_LIFE=1 build (diagnostic, GPU):
DGP_LIB=distributed_amd/_var/lib_life.so python tools/stream_life.py"""
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
print(f"{dt:.3f}s {e.num_placements() / dt / 1e6:.3f} M/s ({dt * 2.4e9 / n:.0f} clocks/stimulus at 2.4 GHz)")
for i, nm in zip(range(11, 16), ("registered -> ready", "ready -> claimed", "claimed -> w released", "w released -> done", "done -> retired")):
    print(f"  {nm:26s} {st[f'wave_phase{i}'] / n:9.0f} per stimulus")
print(f"  exe claim->retire sum       {st['wave_phase5'] / n:9.0f}; REG busy {st['wave_phase3'] / n:.0f}; win-full {st['stall0'] / n:.0f}")
