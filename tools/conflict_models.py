"""How long the C2 replay's chain of ordered stimuli is under three conflict models (CPU,
the oracle's placement log of a C2-shaped graph). Stimulus r completes placement r on its
worker w_r, releases its dependencies (their holders' ws.nbytes), and decides its frontier
tasks over their candidates (the holders of their dependencies), writing the chosen worker.

  any-touch   the engine's protocol: a stimulus waits for every earlier stimulus that
              touches one of its workers (read or write) -- dgp_conflict_depth's chain
  RAW+WAW     a perfect multi-version scheme: a read waits only for the last earlier WRITE
              of that worker, a write for the last earlier write (what speculation on
              candidates that were read but not chosen could reach at best)
  writes only the completing worker and the chosen workers alone (no candidate reads)

    python tools/conflict_models.py [n_tasks]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sim_protocol as SP  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
g, pt, pw, run, holder, fr, rel, relmask = SP.structure(n, 1024)
dp, di = g["dep_ptr"], g["dep_idx"]
R = len(pt)
fro = [[] for _ in range(R)]
for x in np.flatnonzero(fr >= 0).tolist():
    fro[fr[x]].append(x)
rels = [[] for _ in range(R)]
for d in np.flatnonzero(relmask).tolist():
    rels[rel[d]].append(d)
W = 1024


def sets(r):
    writes = {int(pw[r])} | {int(holder[d]) for d in rels[r]}
    reads = set()
    for x in fro[r]:
        reads.update(int(holder[di[k]]) for k in range(dp[x], dp[x + 1]))
        writes.add(int(holder[x]))
    return writes, reads


last_touch, last_write, last_w2 = np.zeros(W, np.int64), np.zeros(W, np.int64), np.zeros(W, np.int64)
d_any = d_raw = d_w = 0
for r in range(R):
    writes, reads = sets(r)
    a = 1 + max(last_touch[c] for c in writes | reads)
    for c in writes | reads:
        last_touch[c] = a
    b = 1 + max(last_write[c] for c in writes | reads)
    for c in writes:
        last_write[c] = b
    ww = {int(pw[r])} | {int(holder[x]) for x in fro[r]}
    c_ = 1 + max(last_w2[c] for c in ww)
    for c in ww:
        last_w2[c] = c_
    d_any, d_raw, d_w = max(d_any, a), max(d_raw, b), max(d_w, c_)
print(f"{R} stimuli: chain any-touch {d_any} (parallelism {R / d_any:.1f}), RAW+WAW {d_raw} ({R / d_raw:.1f}), "
      f"writes only {d_w} ({R / d_w:.1f})")
