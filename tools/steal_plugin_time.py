"""C4 balance(): the device call on host arrays, then GPUWorkStealing's plugin-state path
(bench.py steal_plugin_leg) on the scheduler-free stand-in (diagnostic)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_amd import graphs  # noqa: E402
from distributed_amd.engine import PlacementEngine  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000
eng = PlacementEngine(0)
p = graphs.steal_problem(4096, T, seed=1)
out = eng.steal_balance(p)
eng.set_timing(True)
t0 = time.perf_counter()
out = eng.steal_balance(p)
dt = time.perf_counter() - t0
kt = {k: round(v[0], 3) for k, v in eng.kernel_times().items() if k.startswith("steal")}
eng.set_timing(False)
print(json.dumps({"device_call_ms": round(dt * 1e3, 3), "kernels_ms": kt, "steals": int(len(out["st_task"]))}), flush=True)
t0 = time.perf_counter()
leg = bench.steal_plugin_leg(eng, p, out)
print(json.dumps(leg), f"(leg incl. stand-in build {time.perf_counter() - t0:.1f} s)", flush=True)
