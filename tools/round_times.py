"""Wall time per replay round (GPU): which rounds of a replay dominate.
python tools/round_times.py c3|c3r|c2 [window]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
name = sys.argv[1]
win = int(sys.argv[2]) if len(sys.argv) > 2 else "auto"
g = (graphs.random_dag(1_000_000, 1024, seed=0) if name == "c2"
     else graphs.shuffle_graph(66_666, 512, restricted=name == "c3r"))
e = PlacementEngine(0, window=win)
e.load(g, {"saturation": 1.1})
e.reset(); e.update_graph(); e.run_rounds(-1)  # warm
e.reset(); e.update_graph()
rows, n0, tot = [], e.num_placements(), 0.0
for _ in range(100_000):
    t = time.perf_counter(); k = e.run_rounds(1); dt = time.perf_counter() - t
    n1 = e.num_placements()
    if k == 0 and n1 == n0:
        break
    rows.append((dt, n1 - n0)); tot += dt; n0 = n1
print(f"{name} window {e.get_window()}: {len(rows)} rounds, {tot:.4f} s, {n0} placements")
for i, (dt, n) in sorted(enumerate(rows), key=lambda x: -x[1][0])[:12]:
    print(f"  round {i:4d}: {dt * 1e3:8.2f} ms, placed {n:7d}")
e.close()
