"""Bench-step timing (reset + update_graph + replay) and update_graph alone (GPU):
python tools/time_steps.py [reps]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for name, g in (("c2", graphs.random_dag(1_000_000, 1024, seed=0)), ("c3", graphs.shuffle_graph(66_666, 512)),
                ("c3r", graphs.shuffle_graph(66_666, 512, restricted=True))):
    e = PlacementEngine(0)
    e.load(g, {"saturation": 1.1})
    e.reset(); e.update_graph(); e.run_rounds(-1)
    ug, st = [], []
    for it in range(reps):
        t0 = time.perf_counter(); e.reset(); e.update_graph(); t1 = time.perf_counter(); e.run_rounds(-1)
        t2 = time.perf_counter(); ug.append(t1 - t0); st.append(t2 - t0)
    n = e.num_placements()
    print(f"{name}: step {min(st):.4f}s ({n / min(st) / 1e6:.3f} M/s), reset+update_graph {min(ug) * 1e3:.2f} ms",
          flush=True)
    e.close()
