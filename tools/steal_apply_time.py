"""Host cost of GPUWorkStealing's bulk request application (apply_requests) at C4, CPU only:
the oracle stands in for the device (its outputs are the device's, tests/test_gpu_steal.py).
python tools/steal_apply_time.py [W] [T]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

from distributed_amd import graphs  # noqa: E402
from distributed_amd.stealing import apply_requests, balance_plan, ordered_problem  # noqa: E402
from oracle import oracle  # noqa: E402
from steal_standin import plugin_from_problem  # noqa: E402


class OracleEngine:
    def steal_balance(self, p):
        perm = np.lexsort((p["task_arrival"], p["task_prio"]))
        q, _ = ordered_problem(p, perm)
        out = dict(oracle.steal_balance(q))
        out["st_task"] = perm[np.asarray(out["st_task"], np.int64)].astype(np.int32)
        return out


W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T = int(sys.argv[2]) if len(sys.argv) > 2 else 500_000
p = graphs.steal_problem(W, T, nthreads=2, seed=1)
lv = oracle.steal_balance(p)["level"]
t0 = time.perf_counter()
plugin, slot_task = plugin_from_problem(p, lv)
print(f"stand-in {time.perf_counter() - t0:.1f}s", flush=True)
out, rows, wss = balance_plan(plugin, OracleEngine())
t0 = time.perf_counter()
log = apply_requests(plugin, out, plugin._last_problem, rows, wss, 0.0)
dt = time.perf_counter() - t0
print(f"apply_requests: {len(log)} requests in {dt * 1e3:.1f} ms ({dt / max(1, len(log)) * 1e6:.2f} us/request)")
