"""Wall time + parity of the round-kernel engine (graphs the stream engine does not take:
more than 8 prefixes, worker restrictions) at BASELINE sizes (GPU):
python tools/round_engine_check.py"""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
from oracle import oracle
cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}
for name, g in (("c3_restricted", graphs.shuffle_graph(66_666, 512, restricted=True)),
                ("c2_16prefixes", graphs.random_dag(1_000_000, 1024, seed=0, n_inner_prefixes=15))):
    e = PlacementEngine(0)
    e.load(g, cfg)
    ts = []
    for it in range(2):
        e.reset(); e.update_graph(); t = time.time(); e.run_rounds(-1); ts.append(time.time() - t)
        print(name, f"run {it}: {ts[-1]:.3f}s", flush=True)
    out = e.placements()
    e.close()
    ref = oracle.replay(g, cfg, snapshots=False)
    ok = all(np.array_equal(out[k], ref[k]) for k in ("pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route"))
    n = len(out["pl_task"])
    print(f"{name}: {min(ts):.4f}s, {n / min(ts) / 1e6:.3f} M placements/s, parity {ok}, oracle {n / ref['seconds'] / 1e6:.3f} M/s", flush=True)
