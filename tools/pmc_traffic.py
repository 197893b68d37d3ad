"""HBM traffic per launch of the replay kernel from two rocprofv3 --pmc passes.

    python tools/pmc_traffic.py gpurun_out/<tag> profiles/hbm_traffic.json [n_tasks n_workers]

Reads <dir>/pmc_FETCH_SIZE/**/*counter_collection.csv and the WRITE_SIZE twin (one counter
per pass: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2), keeps the longest dispatch of
`k_stream` (the replay; bench.py's link-latency probe launches short ones too) and prices it
per the MI355X guide's gfx950 correction: FETCH_SIZE (KiB) reports half the bytes of a read,
so hbm = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. The engine sources' hash is recorded: bench.py
reports the result as roofline.traffic only for the workload and the sources it was measured on.
"""
import csv
import glob
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def engine_source_hash() -> str:
    """sha256 over the HIP sources of libdgplace.so (bench.py computes the same)."""
    h = hashlib.sha256()
    csrc = os.path.join(REPO, "distributed_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".h", ".hip")):
            h.update(f.encode())
            h.update(open(os.path.join(csrc, f), "rb").read())
    return h.hexdigest()


def counter(d: str, name: str, kernel: str = "k_stream") -> list:
    """[value] of the longest dispatch of `kernel` (one per file if several files)."""
    files = glob.glob(os.path.join(d, f"pmc_{name}", "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter csv under {d}/pmc_{name}")
    out = []
    for f in files:
        per, dur = {}, {}
        for row in csv.DictReader(open(f)):
            if kernel not in row.get("Kernel_Name", "") or row.get("Counter_Name") != name:
                continue
            key = row.get("Dispatch_Id") or row.get("Correlation_Id")
            per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
            dur[key] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        if per:
            out.append(per[max(dur, key=dur.get)])
    return out


def main():
    d, out = sys.argv[1], sys.argv[2]
    n_tasks = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
    n_workers = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
    fetch = counter(d, "FETCH_SIZE")
    write = counter(d, "WRITE_SIZE")
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    res = {"kernel": "k_stream", "n_tasks": n_tasks, "n_workers": n_workers,
           "launches": {"FETCH_SIZE": len(fetch), "WRITE_SIZE": len(write)},
           "fetch_size_kib_per_launch": f_kib, "write_size_kib_per_launch": w_kib,
           "traffic_bytes_per_launch": (2 * f_kib + w_kib) * 1024,
           "read_bytes_per_launch": 2 * f_kib * 1024, "write_bytes_per_launch": w_kib * 1024,
           "correction": "gfx950: FETCH_SIZE doubled (MI355X_MICROARCH.md HBM section); calibrated on this "
                         "kernel's own patterns in profiles/r02_calibration/calibration.json",
           "src_sha256": engine_source_hash(),
           "source": os.path.relpath(d, REPO) if os.path.isabs(d) else d}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
