"""Phase breakdown of the ordered commit on the C2 workload (GPU)."""
import sys
import time

sys.path.insert(0, ".")
from distributed_amd import graphs  # noqa: E402
from distributed_amd.engine import PlacementEngine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
w = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
g = graphs.random_dag(n, w, seed=0)
e = PlacementEngine(0)
e.load(g, {"saturation": 1.1})
t = time.time()
e.update_graph()
print("update_graph", round(time.time() - t, 4), flush=True)
t = time.time()
e.run_rounds()
dt = time.time() - t
st = e.stats()
print("rounds wall", round(dt, 3), "s", st, flush=True)
ghz = 0.1  # s_memtime ticks at the shader clock on gfx950? report raw and per-step
for k in ("cyc_setup", "cyc_local_steps", "cyc_global", "cyc_finish", "cyc_reserve", "cyc_exec_sum"):
    print(f"{k:18s} {st[k]:>16d} cycles  per round {st[k] / max(st['rounds'], 1):12.0f}")
print("per local step", st["cyc_local_steps"] / max(st["dr_steps"], 1), "max step", st["cyc_max_step"])
print("exec per event (avg)", st["cyc_exec_sum"] / max(st["placements"], 1), "exec max", st["cyc_exec_max"])
names = ["gather", "completion", "releases", "front_gather", "front_argmin", "front_line", "front_commit", "pops", "store"]
tot = sum(st[f"wave_phase{i}"] for i in range(9))
for i, nm in enumerate(names):
    v = st[f"wave_phase{i}"]
    print(f"  {nm:14s} {v / max(st['placements'], 1):10.0f} cyc/event  {100 * v / max(tot, 1):5.1f}%")
