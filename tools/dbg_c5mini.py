"""Debug: the c5mini fixture replay under stream debug modes (GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import oracle
from distributed_amd.engine import PlacementEngine
name = sys.argv[1] if len(sys.argv) > 1 else "c5mini_sat1.1.npz"
g, cfg, exp, meta = oracle.load_fixture(os.path.join("tests/golden", name))
for dbg in ("1", "0"):
    os.environ["DGP_STREAM_DEBUG"] = dbg
    with PlacementEngine(0) as e:
        e.load(g, cfg)
        try:
            e.replay()
            out = e.placements()
            bad = np.nonzero(out["pl_task"] != exp["pl_task"][:len(out["pl_task"])])[0]
            print(f"dbg={dbg}: ok, {len(out['pl_task'])} placements, first task mismatch {bad[:3]}")
        except Exception as ex:
            st = e.stats()
            print(f"dbg={dbg}: {ex}; placements {e.num_placements()}; wave_phase {[st[f'wave_phase{i}'] for i in range(16)]}")
