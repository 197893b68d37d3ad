"""The replay dispatches of a rocprofv3 kernel trace (the bench's C2 / C3 / C5 replays are
single long k_stream launches; the service legs add many short ones that the --stats
average mixes in): python tools/replay_dispatches.py <kernel_trace.csv> [out.json]"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
groups = {}
for r in rows:
    name = r["Kernel_Name"]
    if "k_stream" not in name:
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # ms
    if d < 50:  # service-mode / probe launches
        continue
    key = ("st64" if "st64" in name else "st") + (" global-worker-state" if "<false>" in name else "")
    key += " >500ms" if d > 500 else " 50-500ms"
    groups.setdefault(key, []).append(d)
out = {k: {"dispatches": len(v), "avg_ms": round(sum(v) / len(v), 3), "min_ms": round(min(v), 3),
           "max_ms": round(max(v), 3)} for k, v in sorted(groups.items())}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
