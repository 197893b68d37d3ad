"""roofline.traffic: the committed PMC passes price the replay kernel's HBM bytes with the
gfx950 correction (FETCH_SIZE doubled), profiles/hbm_traffic.json is what they give, and
bench.py reports it only for the engine sources it was measured on (src_sha256)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hbm_traffic_matches_committed_counters(tmp_path):
    pinned = json.load(open(os.path.join(REPO, "profiles", "hbm_traffic.json")))
    src = pinned["source"].split()[0]  # the profile directory holding the two passes
    out = tmp_path / "t.json"
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "pmc_traffic.py"), os.path.join(REPO, src),
                           str(out)], stdout=subprocess.DEVNULL)
    got = json.load(open(out))
    assert got["launches"] == {"FETCH_SIZE": 1, "WRITE_SIZE": 1}  # the C2 replay dispatch only
    assert got["traffic_bytes_per_launch"] == (2 * got["fetch_size_kib_per_launch"] + got["write_size_kib_per_launch"]) * 1024
    assert pinned["traffic_bytes_per_launch"] == got["traffic_bytes_per_launch"]
    assert (pinned["n_tasks"], pinned["n_workers"]) == (1_000_000, 1024)
    assert len(pinned["src_sha256"]) == 64
