"""GPUWorkStealing.balance()'s request application (stealing.apply_requests) inside the
reference scheduler state, beside the reference's own move_task_request per request
(tools/ref_python_time.py c4mtr, the same gen_steal.build scenario): build container,
python3.9 + the reference, the oracle standing in for the device (its outputs are the
device's: tests/test_gpu_steal.py).

    PYTHONHASHSEED=0 taskset -c 2 /opt/conda/bin/python3.9 tools/steal_apply_ref.py [T] [--out FILE]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
if os.environ.get("PYTHONHASHSEED") != "0":
    sys.exit(subprocess.call([sys.executable] + sys.argv, env=dict(os.environ, PYTHONHASHSEED="0")))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
sys.path.insert(0, REPO)
import warnings  # noqa: E402

warnings.filterwarnings("ignore")
import gen_steal as GS  # noqa: E402
from steal_ext_driver import OracleEngine  # noqa: E402

from distributed_amd.stealing import GPUWorkStealing, apply_requests, balance_plan  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    T = int(args[0]) if args else 100_000
    out_path = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    eng = OracleEngine()
    s, steal, *_ = GS.build(4096, T, 2, 0.1, 1, steal_base=GPUWorkStealing,
                            steal_kwargs=dict(engine_factory=lambda: eng))
    t0 = time.perf_counter()
    out, rows, wss = balance_plan(steal, eng)
    t1 = time.perf_counter()
    log = apply_requests(steal, out, steal._last_problem, rows, wss, t0)
    t2 = time.perf_counter()
    n = len(log)
    res = dict(config=f"C4: gen_steal.build(4096 workers, {T} tasks, nthreads 2, hot 10%, seed 1); one balance()",
               requests=n, apply_requests_ms=round(1e3 * (t2 - t1), 1),
               apply_requests_us_per_request=round(1e6 * (t2 - t1) / max(1, n), 2),
               plan_ms_oracle_engine=round(1e3 * (t1 - t0), 1), in_flight=len(steal.in_flight),
               python=sys.version.split()[0], cores=1, cpu_affinity=sorted(os.sched_getaffinity(0)),
               script="tools/steal_apply_ref.py")
    print(json.dumps(res, indent=1), flush=True)
    if out_path:
        json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
