"""Host-side cost of GPUWorkStealing.balance() (python3.9 + the reference, build container):
the problem from the plugin's state at C4-like sizes: the full rebuild
(steal_problem_from_state) vs the incrementally kept task rows (GPUWorkStealing.problem).
PYTHONHASHSEED=0 /opt/conda/bin/python3.9 tools/steal_host_time.py [T ...]"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)
import gen_steal as GS  # noqa: E402

from distributed_amd.stealing import GPUWorkStealing, steal_problem_from_state  # noqa: E402

for T in [int(x) for x in sys.argv[1:]] or [100_000]:
    t0 = time.perf_counter()
    s, steal, *_ = GS.build(4096, T, 2, 0.1, 1, steal_base=GPUWorkStealing)
    t1 = time.perf_counter()
    for name, fn in (("full rebuild (steal_problem_from_state)", lambda: steal_problem_from_state(steal)),
                     ("incremental rows (GPUWorkStealing.problem)", steal.problem)):
        best = float("inf")
        for _ in range(3):
            a = time.perf_counter()
            p, tasks, wss = fn()
            best = min(best, time.perf_counter() - a)
        print(f"T={T} W=4096: state built in {t1 - t0:.1f} s; {name} {best * 1e3:.1f} ms "
              f"({len(tasks)} stealable tasks)", flush=True)
