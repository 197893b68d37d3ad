"""Per-message latency of the resident service kernel through the bare C ABI, with the
device-side split and when each stream role finished (GPU): python tools/svc_latency.py"""
import sys, json
sys.path.insert(0, '.')
import bench
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
g = graphs.random_dag(20000, 1024, seed=5)
print(json.dumps(bench.c_call_latency(PlacementEngine, 0, g)))
