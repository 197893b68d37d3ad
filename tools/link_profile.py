"""Per-link breakdown of the C2 replay's critical chain (GPU, a DGP_TRACE=3 build):
    tools/build_variants.sh trace3 "-DDGP_TRACE=3"
    DGP_LIB=tools/_var/lib_trace3.so python tools/link_profile.py [lo] [n] [c3|c5] [--out file.json]

Every traced stimulus records its executor's phases (s_memtime ticks) and which earlier
stimulus' release made it ready (its completing worker / release holders free: `pred` 0)
and which made its frontier candidates final (`predc` 0, the wait in place). The gate of a
stimulus is the later of the two events that its claim or its wait actually waited for; the
chain is followed backwards from the last stimulus of the window through the stimulus that
released each gate. A link is the time from one gate to the next: the predecessor's work
from its own gate up to the release, split by the phase in which the release happened."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
args = [a for a in sys.argv[1:] if not a.startswith("--")]
lo = int(args[0]) if len(args) > 0 else 400_000
n = int(args[1]) if len(args) > 1 else 20_000
out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
os.environ["DGP_TRACE_LO"] = str(lo)
os.environ["DGP_TRACE_N"] = str(n)
from distributed_amd import graphs  # noqa: E402
from distributed_amd.engine import PlacementEngine  # noqa: E402

c3 = "c3" in args
c5 = "c5" in args  # C5-shaped: map 1M + tree-reduce on 16,384 workers (the global worker-state path)
g = (graphs.shuffle_graph(66_666, 512) if c3 else graphs.map_tree_reduce(1_000_000, 16_384) if c5
     else graphs.random_dag(1_000_000, 1024, seed=0))
e = PlacementEngine(0, window=32)
e.load(g, {"saturation": 1.1})
e.reset()
e.update_graph()
e.run_rounds(-1)
buf = np.zeros(n * 32, np.uint64)
e.lib.dgp_debug_trace.argtypes = [C.c_void_p, C.c_void_p]
assert e.lib.dgp_debug_trace(e.h, buf.ctypes.data_as(C.c_void_p)) == 0
T = buf.reshape(n, 32).astype(np.int64)
PH = ["claim", "precheck", "state", "compl_needs", "pre_wait", "post_wait", "keys", "argmin_early", "commit1",
      "frontier", "refill", "w_release"]
IDX = [2, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18]
loc = (T[:, 2] > 0) & (T[:, 8] > 0) & (T[:, 18] > 0)  # exe_local stimuli, fully traced
res = {"window": [lo, n], "traced_local": int(loc.sum()), "phases": {}}
print(f"{loc.sum()} of {n} stimuli traced through exe_local")


def pct(v):
    v = v.astype(np.float64)
    return {"mean": float(v.mean()), "p50": float(np.percentile(v, 50)), "p90": float(np.percentile(v, 90))}


L = T[loc]
meta = L[:, 22]
nf = meta & 0xFF
print("  executor phases (ticks, claim -> w released):")
for a, b, nm in zip(IDX[:-1], IDX[1:], PH[1:]):
    sel = (L[:, a] > 0) & (L[:, b] > 0)
    if nm in ("keys", "argmin_early", "commit1"):
        sel &= nf > 0
    d = L[sel, b] - L[sel, a]
    res["phases"][nm] = pct(d)
    print(f"    {PH[IDX.index(a)]:>12s} -> {nm:12s} mean {d.mean():8.0f} p50 {np.percentile(d, 50):8.0f} "
          f"p90 {np.percentile(d, 90):8.0f}")
d = L[:, 18] - L[:, 2]
res["phases"]["claim_to_w_release"] = pct(d)
print(f"    claim -> w released total     mean {d.mean():8.0f} p50 {np.percentile(d, 50):8.0f}")
waited = L[:, 12] - L[:, 11]
res["wait_in_place"] = pct(waited)
print(f"  wait in place: mean {waited.mean():.0f}, p50 {np.percentile(waited, 50):.0f}, "
      f"zero {np.mean(waited < 200) * 100:.0f}%; frontier tasks per stimulus {nf.mean():.2f}")
rc = T[:, 2] - T[:, 1]
ok = (T[:, 1] > 0) & (T[:, 2] > 0)
res["ready_to_claim"] = pct(rc[ok])
SUB = [(14, 24, "place stores"), (24, 25, "line_load cb"), (25, 26, "needs_inc"), (26, 27, "line_store+dict_add"),
       (27, 28, "net_bw + ballot"), (28, 29, "occ_dict_r"), (29, 15, "rec stores")]
sel = (L[:, 24] > 0) & (L[:, 29] > 0) & (nf > 0)
if sel.any():
    print("  first commit, split:")
for a, b, nm in (SUB if sel.any() else ()):  # (only the commit-split probe build records these)
    d = L[sel, b] - L[sel, a]
    res["phases"]["commit:" + nm] = pct(d)
    print(f"    {nm:22s} mean {d.mean():8.0f} p50 {np.percentile(d, 50):8.0f}")
print(f"  ready -> claimed: mean {rc[ok].mean():.0f} p50 {np.percentile(rc[ok], 50):.0f}")

# ---- the critical chain, backwards
idx = {lo + i: i for i in range(n)}


def gate(i):
    """(time, releaser, kind) of what stimulus i last waited for."""
    rdy, rby = T[i, 1], T[i, 19]
    pc, pby = T[i, 20], T[i, 21]
    claim, wend, wstart = T[i, 2], T[i, 12], T[i, 11]
    g = (rdy, rby, "ready") if rdy > 0 and rby > 0 else (0, -1, "none")
    if pc > 0 and pby > 0 and wend > 0 and wstart > 0 and pc > wstart and pc > g[0]:
        g = (pc, pby, "cand")
    if claim > 0 and g[2] == "ready" and claim - rdy > 2000:
        g = (g[0], g[1], "ready_exe")  # ready long before an executor took it
    return g


last = int(np.argmax(np.where(T[:, 18] > 0, T[:, 18], 0)))
chain = []
i = last
while i is not None:
    t, by, kind = gate(i)
    if by < 0 or by not in idx or kind == "none":
        break
    chain.append((i, t, idx[by], kind))
    i = idx[by]
chain = chain[::-1]
links = []
for (i_prev, t_prev, _, k_prev), (i, t, j, kind) in zip(chain[:-1], chain[1:]):
    # j released what gated i (at t), j itself was gated at t_prev
    ph = "after_w_release"
    for a, nm in zip(IDX, PH):
        if T[j, a] > 0 and T[j, a] <= t:
            ph = nm
    links.append({"dt": int(t - t_prev), "kind": kind, "released_after": ph,
                  "gate_to_claim": int(max(0, T[j, 2] - t_prev)) if T[j, 2] > 0 else -1,
                  "waited_in_place": int(max(0, T[j, 12] - T[j, 11])) if T[j, 12] > 0 and T[j, 11] > 0 else 0,
                  "nf": int(T[j, 22] & 0xFF)})
if links:
    dts = np.array([x["dt"] for x in links], np.float64)
    print(f"  critical chain: {len(links)} links over the window's last {t - chain[0][1]} ticks, "
          f"link mean {dts.mean():.0f} p50 {np.percentile(dts, 50):.0f}")
    kinds = {}
    for x in links:
        kinds.setdefault((x["kind"], x["released_after"]), []).append(x["dt"])
    res["chain"] = {"links": len(links), "link": pct(dts), "by_kind": {}}
    for (k, ph), v in sorted(kinds.items(), key=lambda kv: -sum(kv[1])):
        print(f"    gate {k:9s} released in phase {ph:14s}: {len(v):6d} links, mean {np.mean(v):8.0f}, "
              f"share {sum(v) / dts.sum() * 100:5.1f}%")
        res["chain"]["by_kind"][f"{k}/{ph}"] = {"links": len(v), "mean": float(np.mean(v)),
                                                "share": float(sum(v) / dts.sum())}
    g2c = np.array([x["gate_to_claim"] for x in links if x["gate_to_claim"] >= 0], np.float64)
    wip = np.array([x["waited_in_place"] for x in links], np.float64)
    res["chain"]["pred_gate_to_claim_mean"] = float(g2c.mean()) if len(g2c) else None
    res["chain"]["pred_waited_in_place_mean"] = float(wip.mean())
    print(f"    on the chain: gate -> claim mean {g2c.mean():.0f}; waited in place mean {wip.mean():.0f}")
if out:
    json.dump(res, open(out, "w"), indent=1)
