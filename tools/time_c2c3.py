"""Wall time of the C2 and C3 replays (GPU): python tools/time_c2c3.py [reps]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for name, g in (("c2", graphs.random_dag(1_000_000, 1024, seed=0)), ("c3", graphs.shuffle_graph(66_666, 512)),
                ("c3r", graphs.shuffle_graph(66_666, 512, restricted=True))):
    e = PlacementEngine(0)
    e.load(g, {"saturation": 1.1})
    ts = []
    for it in range(reps + 1):
        e.reset(); e.update_graph(); t = time.time(); e.run_rounds(-1); ts.append(time.time() - t)
    n = e.num_placements()
    print(f"{name}: {min(ts[1:]):.4f}s best of {reps}, {n / min(ts[1:]) / 1e6:.3f} M placements/s", flush=True)
    e.close()
