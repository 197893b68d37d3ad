"""Benchmark: task placements/sec of the HIP placement engine on BASELINE.json's C2
workload (1M-task random DAG, fan-in <= 4, lognormal nbytes, 1,024 workers x 1
thread, worker-saturation 1.1), plus the HBM roofline of the dominant kernel and the
oracle CPU baseline.

One step = one full replay of the workload on the device (update_graph + every
completion round, ~1M placements), the graph already resident in HBM. For N GPUs
(torch.distributed.run, one rank per GPU) every rank replays its own copy of the
workload ("replicas only") and value = placements of all ranks / the
slowest rank's time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--tasks N] [--workers W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "task placements/sec at 1M tasks x 1,024 workers; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip-level parameters)
CONFIG = {"bandwidth": 100_000_000, "default_data_size": 1024, "unknown_duration": 0.5, "saturation": 1.1}


def algorithmic_bytes(g: dict, pl_worker_of_task: np.ndarray) -> dict:
    """Bytes each kernel must move over one full replay (DESIGN.md §3 lists the terms).

    k = fan-in, f = fan-out, c = distinct candidate workers, WB = bitset words per row.
    """
    n = g["n_tasks"]
    W = len(g["nthreads"])
    WB = (W + 63) // 64
    k = np.diff(g["dep_ptr"]).astype(np.int64)
    f = np.bincount(g["dep_idx"], minlength=n).astype(np.int64)
    src = np.repeat(np.arange(n), k)
    holder = pl_worker_of_task[g["dep_idx"]].astype(np.int64)
    # distinct (task, holder) pairs -> candidates per task (one replica per dependency in the replay)
    pairs = np.unique(src.astype(np.int64) * (W + 1) + holder)
    c = np.bincount(pairs // (W + 1), minlength=n).astype(np.int64)
    ready_later = k > 0  # tasks released by a completion (go through k_candidate_commbytes)
    release = (56 + 28 * (f + k)).sum() + 4 * ready_later.sum()
    cand = (33 + k * (12 + 8 * WB) + 12 * c)[ready_later].sum()
    commit = (64 + 25 * k + 17 * f).sum() + (96 + 52 * c + 12 * k + 33).sum()
    return {"frontier_release": float(release), "candidate_commbytes": float(cand), "commit": float(commit)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tasks", type=int, default=1_000_000)
    ap.add_argument("--workers", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    from distributed_amd import graphs
    from distributed_amd.engine import PlacementEngine

    g = graphs.random_dag(args.tasks, args.workers, seed=0)
    eng = PlacementEngine(local)
    eng.load(g, CONFIG)

    def step():
        eng.reset()
        eng.update_graph()
        eng.run_rounds(-1)

    def barrier():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        step()
    eng.set_timing(True)
    barrier()
    t0 = time.perf_counter()
    kt_total = {}
    for _ in range(args.steps):
        step()
        for name, (ms, n) in eng.kernel_times().items():  # resolves this step's events
            a = kt_total.setdefault(name, [0.0, 0])
            a[0] += ms
            a[1] += n
    barrier()
    elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    placements = eng.num_placements()
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_placements = placements * args.steps * world
    value = total_placements / elapsed

    out = eng.placements()
    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "placements/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64+f64",
        "data": "synthetic",
        "config": {"workload": "C2: random DAG, fan-in<=4 (window 4W), lognormal(10,2) nbytes, roots N/10, "
                               "workers x 1 thread, worker-saturation 1.1; full replay per step",
                   "n_tasks": args.tasks, "n_workers": args.workers, "parallelism": f"replicas{world}",
                   "placements_per_step": placements},
    }
    if rank == 0:
        pl_worker_of_task = np.empty(g["n_tasks"], np.int64)
        pl_worker_of_task[out["pl_task"]] = out["pl_worker"]
        ab = algorithmic_bytes(g, pl_worker_of_task)
        kernels = {}
        for name in ("frontier_release", "candidate_commbytes", "commit"):
            ms, n = kt_total.get(name, (0.0, 0))
            if n == 0:
                continue
            per_launch_bytes = ab[name] / (n / args.steps)
            avg_ms = ms / n
            kernels[name] = {"total_ms_per_step": ms / args.steps, "launches_per_step": n // args.steps,
                             "avg_us": 1e3 * avg_ms, "achieved_GBs": per_launch_bytes / (avg_ms * 1e-3) / 1e9}
        dom = max(kernels, key=lambda k: kernels[k]["total_ms_per_step"])
        ach = kernels[dom]["achieved_GBs"]
        result["roofline"] = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": None}
        result["kernels"] = {k: {kk: round(vv, 3) for kk, vv in v.items()} for k, v in kernels.items()}
        if world == 1 and not args.no_cpu_baseline:
            from oracle import oracle

            runs, secs, ref = 0, 0.0, None
            while runs < 1 or (secs < args.cpu_seconds and runs < 5):
                ref = oracle.replay(g, CONFIG, snapshots=False)
                secs += ref["seconds"]
                runs += 1
            n_ref = len(ref["pl_task"])
            result["cpu_baseline"] = {"value": round(n_ref * runs / secs, 1), "unit": "placements/s", "cores": 1,
                                      "kind": "port",
                                      "sample": f"oracle/replay.cpp, full C2 replay ({n_ref} placements) x {runs}"}
            result["parity"] = bool(all(np.array_equal(out[k], ref[k]) for k in (
                "pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route")))
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
