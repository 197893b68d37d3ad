"""C5 (map + tree-reduce) replay time on the 32-slot (wait-in-place) and 64-slot stream builds
of one library, same graph, alternating; the placement digests must agree:
python tools/c5_window_ab.py N_MAP N_WORKERS"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs  # noqa: E402
from distributed_amd.engine import PlacementEngine  # noqa: E402

CFG = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
m, W = int(sys.argv[1]), int(sys.argv[2])
g = graphs.map_tree_reduce(m, W, seed=3)
dig = {}
for rep in range(2):
    for win in (32, 64):
        e = PlacementEngine(0, window=win)
        e.load(g, CFG)
        e.reset()
        e.update_graph()
        t = time.perf_counter()
        e.run_rounds(-1)
        dt = time.perf_counter() - t
        d = graphs.placement_digest(e.placements())
        dig.setdefault(win, d)
        print(f"window {win} rep {rep}: {dt:.3f} s, {e.num_placements() / dt / 1e6:.3f} M placements/s, "
              f"digest {'same' if d == dig[32] else 'DIFFERENT'}", flush=True)
        e.close()
