"""One C4 balance() (500k x 4096) on the device: for rocprofv3 counter passes (diagnostic)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine

e = PlacementEngine(0)
p = graphs.steal_problem(4096, int(sys.argv[1]) if len(sys.argv) > 1 else 500_000, seed=1)
out = e.steal_balance(p)
print(len(out["st_task"]), "steals", flush=True)
