"""Post-mortem of a failing stream replay on a fixture (diagnostic, GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.engine import PlacementEngine
from oracle import oracle
name = sys.argv[1] if len(sys.argv) > 1 else "c2mini_sat1.1.npz"
g, cfg, exp, meta = oracle.load_fixture(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", name))
R = len(exp["round_nplaced"]) + 2
e = PlacementEngine(0)
e.load(g, cfg, snapshots=R)
try:
    e.replay()
    print("ok", e.num_placements())
except Exception as ex:
    print("error:", ex)
st = e.stats()
names = ["seq_pos", "reg_pos", "pre_pos", "bld_pos", "log_len", "ready", "busy_exe", "global_pending", "rdone[sp]", "rdone[sp+1]",
         "slot(old)", "free_slots", "walk_pos", "rec_len", "qlen", "round_end"]
for i, nm in enumerate(names):
    v = st[f"wave_phase{i}"]
    print(f"  {nm:16s} {v} {hex(v & 0xffffffff) if nm in ('ready', 'free_slots', 'flags[old]') else ''}")
