"""GPU quick check while iterating on the stream kernel: C2-shaped (n tasks), C3, restricted
C3, a 16-prefix C2 and c2mini-style small graphs vs the oracle (bit-exact placement log), then
wall times. python tools/quick_parity.py [n_tasks]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
from oracle import oracle

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
K = ("pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route")
cases = [("c2", graphs.random_dag(n, 1024, seed=0), 1.1), ("c2inf", graphs.random_dag(n // 3, 1024, seed=5), "inf"),
         ("c2p16", graphs.random_dag(n // 3, 1024, seed=1, n_inner_prefixes=16, random_durations=True), 1.1),
         ("c2nt", graphs.random_dag(n // 3, 512, seed=2, nthreads="random", random_durations=True), 1.1),
         ("c3", graphs.shuffle_graph(66_666, 512), 1.1), ("c3r", graphs.shuffle_graph(66_666, 512, restricted=True), 1.1),
         ("w4096", graphs.random_dag(30_000, 4096, seed=42), 1.1)]
bad = 0
for name, g, sat in cases:
    cfg = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": sat}
    for window in (32, 64):
        e = PlacementEngine(0, window=window)
        e.load(g, cfg)
        ts = []
        for it in range(2):
            e.reset(); e.update_graph(); t = time.time(); e.run_rounds(-1); ts.append(time.time() - t)
        out = e.placements()
        e.close()
        ref = oracle.replay(g, cfg, snapshots=False)
        ok = all(np.array_equal(np.asarray(out[k]), np.asarray(ref[k])) for k in K)
        first = -1
        if not ok:
            bad += 1
            a, b = out["pl_task"], ref["pl_task"]
            m = min(len(a), len(b))
            d = np.nonzero((a[:m] != b[:m]) | (out["pl_worker"][:m] != ref["pl_worker"][:m]))[0]
            first = int(d[0]) if len(d) else m
        print(f"{name:6s} w{window}: {'OK ' if ok else 'BAD'} {len(out['pl_task'])} placements, best {min(ts):.4f}s "
              f"{len(out['pl_task']) / min(ts) / 1e6:.3f} M/s {'' if ok else f'first diff {first}'}", flush=True)
sys.exit(1 if bad else 0)
