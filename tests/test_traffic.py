"""roofline.traffic: the committed PMC passes price the replay kernel's HBM bytes with the
gfx950 correction (FETCH_SIZE doubled), and profiles/hbm_traffic.json is what they give."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hbm_traffic_matches_committed_counters(tmp_path):
    # the counters hbm_traffic.json cites (its "source")
    src = os.path.join(REPO, "profiles", "r02a")
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        os.makedirs(tmp_path / f"pmc_{c}")
        # dispatch 112 is the C2 replay; the later k_stream dispatches of that run are C3
        rows = list(csv.DictReader(open(os.path.join(src, f"pmc_{c.lower()}.csv"))))
        with open(tmp_path / f"pmc_{c}" / "run_counter_collection.csv", "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(r for r in rows if r["Dispatch_Id"] == "112" or "k_stream" not in r["Kernel_Name"])
    out = tmp_path / "t.json"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "pmc_traffic.py"), str(tmp_path), str(out)],
                          stdout=subprocess.DEVNULL)
    got = json.load(open(out))
    assert got["launches"] == {"FETCH_SIZE": 1, "WRITE_SIZE": 1}
    assert got["traffic_bytes_per_launch"] == (2 * got["fetch_size_kib_per_launch"] + got["write_size_kib_per_launch"]) * 1024
    pinned = json.load(open(os.path.join(REPO, "profiles", "hbm_traffic.json")))
    assert pinned["traffic_bytes_per_launch"] == got["traffic_bytes_per_launch"]
    assert (pinned["n_tasks"], pinned["n_workers"]) == (1_000_000, 1024)
