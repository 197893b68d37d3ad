"""Per-role / per-phase cycle breakdown of the stream engine (s_memtime ticks)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd import graphs
from distributed_amd.engine import PlacementEngine
if len(sys.argv) > 1 and sys.argv[1] in ("c3", "c3r"):  # C3: P2P-shuffle shape, 66,666 partitions x 512 workers
    g = graphs.shuffle_graph(int(sys.argv[2]) if len(sys.argv) > 2 else 66_666, 512, restricted=sys.argv[1] == "c3r")
    n = g["n_tasks"]
else:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    g = graphs.random_dag(n, w, seed=0)
e = PlacementEngine(0)
e.load(g, {"saturation": 1.1})
for it in range(2):
    e.reset(); e.update_graph(); t = time.time(); e.run_rounds(-1); dt = time.time() - t
st = e.stats()
P = [st[f"wave_phase{i}"] for i in range(16)]
names = {0: "SEQ busy", 1: "BLD busy", 2: "PRE busy", 3: "REG busy", 4: "WLK busy", 5: "EXE claim->retire (sum)",
         6: "BLD batches", 7: "PRE batches", 8: "SEQ batches", 9: "global stimuli", 10: "requeued exact",
         11: "exe precheck", 12: "exe completion", 13: "exe frontier+pops", 14: "exe release", 15: "exe finish"}
print("rounds", st["rounds"], "global stimuli", st["global_stimuli"])
print(f"run_rounds {dt:.3f}s  {e.num_placements() / dt / 1e6:.3f} M placements/s")
for i in range(16):
    print(f"  [{i:2d}] {names[i]:28s} {P[i]:>15d}  per stimulus {P[i] / n:10.1f}")
X = [st[k] for k in ("cyc_setup", "cyc_local_steps", "cyc_global", "cyc_finish", "cyc_reserve", "cyc_max_step", "cyc_exec_max", "cyc_exec_sum")]
for i, nm in enumerate(["16 state load | global rootish", "17 compl. needs | REG fetch+A", "18 start/cand | REG phase B",
                        "19 argmin+early | REG prefetch", "20 commit | global kt>KT_MAX", "21 | global kx/desc full",
                        "22 | global touch/nf", "23 | global queue rule"]):
    print(f"  [x{i}] {nm:28s} {X[i]:>15d}  per stimulus {X[i] / n:10.1f}")

S = [st.get(f"stall{i}", 0) for i in range(8)]
for i, nm in enumerate(["REG window full", "REG desc not prefetched", "REG global pending", "REG batches",
                        "EXE idle (nothing ready)", "EXE ready but gated", "SEQ waits oldest slot", "REG stimuli registered"]):
    print(f"  [s{i}] {nm:28s} {S[i]:>15d}  per stimulus {S[i] / n:10.1f}")
