"""Time WorkStealing.balance on the device for C4-shaped problems (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine

e = PlacementEngine(0)
for W, T in ((4096, 100_000), (4096, 500_000)):
    p = graphs.steal_problem(W, T, seed=1)
    e.steal_balance(p)  # warm-up
    e.set_timing(True)
    e.reset() if False else None
    t0 = time.perf_counter()
    out = e.steal_balance(p)
    dt = time.perf_counter() - t0
    kt = e.kernel_times()
    e.set_timing(False)
    ks = {k: round(v[0], 3) for k, v in kt.items() if k.startswith("steal")}
    print(f"W={W} T={T}: {len(out['st_task'])} steals, call {dt * 1e3:.1f} ms, kernels(ms) {ks}", flush=True)
