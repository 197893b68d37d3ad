"""Benchmark: task placements/sec of the HIP placement engine on BASELINE.json's C2
workload (1M-task random DAG, fan-in <= 4, lognormal nbytes, 1,024 workers x 1
thread, worker-saturation 1.1), plus the HBM roofline of the dominant kernel and the
oracle CPU baseline.

One step = one full replay of the workload on the device (update_graph + every
completion round, ~1M placements), the graph already resident in HBM. For N GPUs
(torch.distributed.run, one rank per GPU): the ordered replay does not
partition (every decision reads the state the one before it left), so the placement legs
run as independent schedulers, one per GPU: rank k replays its own C2-shaped graph (the
generator's seed + k; rank 0's is the pinned workload), each rank checks its own replay
bit-exact against the oracle, and value = the distinct placements all ranks made / the
slowest rank's time ("weak": the work per GPU is fixed; per_rank_value beside it). The
data-parallel part of the WorkStealing leg -- the per-task thief rows -- is sharded over
the ranks and all-gathered.

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


def algorithmic_bytes(g: dict, placed_tasks: np.ndarray, n_waves: int) -> float:
    """SURVEY.md §8(d) algorithmic bytes for placing `placed_tasks` over `n_waves` waves.

    Per placed task t: B_t = 8 + 12 k_t + 8 k_t ceil(W/64) + 12 + 8 + 12 f_t (dep row_ptr pair,
    dep idx + nbytes, replica bitset rows, worker + comm_bytes out, dependents row_ptr pair,
    dependent idx + remaining RMW), plus 48 W per wave (worker vector read + write).
    k_t / f_t are the generated graph's own fan-in / fan-out.
    """
    n = g["n_tasks"]
    W = len(g["nthreads"])
    WB = (W + 63) // 64
    k = np.diff(g["dep_ptr"]).astype(np.int64)[placed_tasks]
    f = np.bincount(g["dep_idx"], minlength=n).astype(np.int64)[placed_tasks]
    per_task = 8 + 12 * k + 8 * k * WB + 12 + 8 + 12 * f
    return float(per_task.sum() + 48 * W * n_waves)


def reduce_max(x: float, dist, device: str = "cuda") -> float:
    """The slowest rank's value (RCCL over xGMI on the GPU box, gloo in the CPU tests)."""
    if dist is None:
        return x
    import torch

    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(x: float, dist, device: str = "cuda") -> float:
    """The sum over ranks (the distinct work of independent per-GPU schedulers)."""
    if dist is None:
        return x
    import torch

    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def link_latency_us(eng_cls, local: int, n_workers: int = 1024) -> float:
    """The engine's link latency within a round: replays of a star (graphs.star: one
    completion places N leaves on one worker, whose N completions then run one after
    another) at two sizes; the slope of the replay time over N (best of 3 each)."""
    from distributed_amd import graphs

    t = {}
    for n in (10_000, 40_000):
        eng = eng_cls(local)
        eng.load(graphs.star(n, n_workers), CONFIG)
        best = float("inf")
        for _ in range(4):
            eng.reset()
            eng.update_graph()
            t0 = time.perf_counter()
            eng.run_rounds(-1)
            best = min(best, time.perf_counter() - t0)
        assert eng.num_placements() == n + 1
        eng.close()
        t[n] = best
    return 1e6 * (t[40_000] - t[10_000]) / 30_000


def latency_bound(g: dict, out: dict, link_us: float, achieved_ms: float) -> dict:
    """Latency roofline of an ordered replay: the longest chain of stimuli that share a
    worker (dgp_conflict_depth on the engine's own placement log) times the serial link
    latency. No engine that runs each stimulus in link_us can finish sooner."""
    from distributed_amd.engine import conflict_depth

    depth, touches = conflict_depth(g, out, 0)
    min_ms = depth * link_us / 1e3
    return {"bound": "latency", "critical_path_links": depth, "stimuli": int(len(out["pl_task"])),
            "average_parallelism": round(len(out["pl_task"]) / max(1, depth), 2),
            "touches": touches, "link_us": round(link_us, 3), "min_ms": round(min_ms, 3),
            "achieved_ms": round(achieved_ms, 3), "achieved_us_per_link": round(1e3 * achieved_ms / max(1, depth), 3),
            "frac": round(min_ms / achieved_ms, 4)}


def steal_leg(eng, args, world: int, dist=None, barrier=None) -> dict:
    """WorkStealing.balance on a C4-shaped state: one call per
    step, inputs uploaded by the call (the boundary hands over host arrays), device
    kernel times from HIP events, and the oracle (oracle/steal.cpp) on the host. With
    N ranks every rank takes part: the thief rows are sharded and all-gathered
    (distributed_amd/shard.py), the ordered walk runs on each rank."""
    from distributed_amd import graphs

    p = graphs.steal_problem(args.steal_workers, args.steal_tasks, seed=1)
    group = dist.group.WORLD if dist is not None else None
    eng.steal_balance(p, group=group)  # warm-up
    eng.set_timing(True)
    if barrier:
        barrier()
    t0 = time.perf_counter()
    n_call = 3
    for _ in range(n_call):
        out = eng.steal_balance(p, group=group)
    if barrier:
        barrier()
    dt = reduce_max((time.perf_counter() - t0) / n_call, dist)
    kt = eng.kernel_times()
    eng.set_timing(False)
    leg = {"metric": "WorkStealing.balance() calls/s", "workload": f"C4-shaped: {args.steal_workers} workers x 2 "
           f"threads, {args.steal_tasks} processing tasks, 10% hot (zipf 1.5), 8 prefixes 10ms*2^j",
           # GPUWorkStealing.balance()'s device path with a scheduler-free stand-in: the problem
           # as host arrays in, dgp_steal_balance (upload, levels, bins, thief rows, the ordered
           # walk), the ordered requests and per-worker accounts back; host-inclusive
           "ms_per_call": round(dt * 1e3, 3), "fits_100ms_interval": bool(dt <= 0.1),
           "boundary": "host arrays -> dgp_steal_balance -> request arrays (host-inclusive, ctypes included)",
           "steal_requests": int(len(out["st_task"])), "n_gpus": world,
           "parallelism": "thief rows sharded + all-gather, ordered walk replicated" if world > 1 else "single",
           "kernel_ms_per_call": {k: round(v[0] / n_call, 3) for k, v in kt.items() if k.startswith("steal")},
           "reference_python_seconds_per_call_at_100k_x_4096": 242.0}
    if world == 1:
        leg["plugin_path"] = steal_plugin_leg(eng, p, out)
    if world == 1 and not args.no_cpu_baseline:
        from oracle import oracle

        t0 = time.perf_counter()
        ref = oracle.steal_balance(p)
        leg["cpu_baseline"] = {"ms_per_call": round((time.perf_counter() - t0) * 1e3, 1), "cores": 1, "kind": "port",
                               "sample": "oracle/steal.cpp, one full balance() of the same problem"}
        leg["parity"] = bool(all(np.array_equal(np.asarray(out[k]), np.asarray(ref[k])) for k in ref))
    return leg


def steal_plugin_leg(eng, p, out_dev) -> dict:
    """GPUWorkStealing.balance() end to end from the plugin's state (stealing.py
    ``balance_plan``): the StealRows the transition hooks keep -> problem arrays (numpy over
    the rows; the dependencies' who_has kept by the replica hooks) -> dgp_steal_order +
    dgp_steal_balance -> the ordered requests as arrays, on a scheduler-free stand-in of the
    plugin state at the same C4 problem (distributed_amd/steal_standin.py; the tasks in the
    bins the device's levels give). Everything of balance() before move_task_request, which
    is the reference's own code (its per-request cost, measured in the reference, beside)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
    from steal_standin import plugin_from_problem
    from distributed_amd.stealing import apply_requests, balance_plan

    plugin, slot_task = plugin_from_problem(p, out_dev["level"])
    balance_plan(plugin, eng)  # warm-up
    n_call = 3
    t_prob = []
    t0 = time.perf_counter()
    for _ in range(n_call):
        t1 = time.perf_counter()
        plugin.rows.problem(plugin)  # the host half alone, for the breakdown
        t_prob.append(time.perf_counter() - t1)
    t_host = (time.perf_counter() - t0) / n_call
    t0 = time.perf_counter()
    for _ in range(n_call):
        plan = balance_plan(plugin, eng)
        out, rows, wss = plan
        req = slot_task[rows[out["st_task"]]]  # the request list: task of each request, in order
    dt = (time.perf_counter() - t0) / n_call
    # the whole product path once: balance_plan, then the requests applied in bulk (bins,
    # steal-request messages, in-flight records and accounts, log, metrics; apply_requests)
    t0 = time.perf_counter()
    out_a, rows_a, wss_a = balance_plan(plugin, eng)
    t1 = time.perf_counter()
    log = apply_requests(plugin, out_a, plugin._last_problem, rows_a, wss_a, t0)
    t_full = time.perf_counter() - t0
    t_apply = time.perf_counter() - t1
    nmsg = sum(len(c.buffer) for c in plugin.scheduler.stream_comms.values())
    applied_ok = bool(len(log) == len(plugin.in_flight) == nmsg == len(req)
                      and all(len(plugin.key_stealable) + len(req) == len(slot_task) for _ in (0,)))
    parity = bool(np.array_equal(req, out_dev["st_task"]) and all(
        np.array_equal(out[k], out_dev[k]) for k in ("st_victim", "st_thief", "st_level", "st_cost", "st_occ_victim",
                                                   "st_occ_thief", "inflight_occ", "inflight_tasks", "idle_after",
                                                   "sat_after", "checked")))
    leg = {"metric": "GPUWorkStealing.balance() from plugin state, ms per call",
           "ms_per_call": round(dt * 1e3, 3), "fits_100ms_interval": bool(dt <= 0.1),
           "host_problem_ms": round(min(t_prob) * 1e3, 3), "host_problem_ms_mean": round(t_host * 1e3, 3),
           "stealable_tasks": int(len(slot_task)), "steal_requests": int(len(req)),
           "boundary": "StealRows (plugin state) -> balance_plan -> request arrays",
           "with_requests_applied_ms": round(t_full * 1e3, 3), "apply_requests_ms": round(t_apply * 1e3, 3),
           "with_requests_boundary": "balance_plan + apply_requests (bulk move_task_request: bins, steal-request "
                                     "messages per victim, in_flight, accounts, log, metrics); the scheduler's "
                                     "check_idle_saturated of the visited victims excluded",
           "requests_applied_consistent": applied_ok,
           "parity_with_device_leg": parity}
    ref = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "ref_python_c4.json")
    if os.path.exists(ref):
        r = json.load(open(ref))
        if "move_task_request_us" in r:
            leg["reference_move_task_request_us_per_request"] = r["move_task_request_us"]
            leg["reference_apply_ms_for_these_requests"] = round(r["move_task_request_us"] * len(req) / 1e3, 1)
    return leg


def c3_leg(eng_cls, local: int, args, link_us: float | None = None) -> dict:
    """BASELINE.json C3: the P2P-shuffle-shaped graph (P inputs -> P shuffle-transfer ->
    1 shuffle-barrier of fan-in P -> P unpack tasks with _rootish False; shuffle/_shuffle.py
    :276-306) on 512 workers x 1 thread, placement only: one full replay per step, checked
    bit-exact against the oracle, which is also the CPU baseline (1 core)."""
    from distributed_amd import graphs

    g = graphs.shuffle_graph(args.c3_partitions, args.c3_workers)
    eng = eng_cls(local)
    eng.load(g, CONFIG)
    eng.reset()
    eng.update_graph()
    eng.run_rounds(-1)  # warm-up
    n_step = 3
    t0 = time.perf_counter()
    for _ in range(n_step):
        eng.reset()
        eng.update_graph()
        eng.run_rounds(-1)
    dt = (time.perf_counter() - t0) / n_step
    out = eng.placements()
    n = int(len(out["pl_task"]))
    leg = {"metric": "task placements/sec, C3 (P2P-shuffle-shaped graph, placement only)", "value": round(n / dt, 1),
           "unit": "placements/s", "seconds_per_replay": round(dt, 4), "placements_per_replay": n,
           "n_tasks": int(g["n_tasks"]), "n_partitions": args.c3_partitions, "n_workers": args.c3_workers,
           "stream_window": eng.get_window()}
    if link_us:
        leg["latency_bound"] = latency_bound(g, out, link_us, dt * 1e3)
    if not args.no_cpu_baseline:
        from oracle import oracle

        ref = oracle.replay(g, CONFIG, snapshots=False)
        leg["cpu_baseline"] = {"value": round(len(ref["pl_task"]) / ref["seconds"], 1), "unit": "placements/s",
                               "cores": 1, "kind": "port", "sample": "oracle/replay.cpp, one full C3 replay"}
        leg["parity"] = bool(all(np.array_equal(out[k], ref[k]) for k in (
            "pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route")))
    eng.close()
    return leg


def variant_legs(eng_cls, local: int, args) -> dict:
    """The C2 and C3 workloads in the forms that used to fall off the stream engine: C2 with
    16 task prefixes (15 inner + root; _calc_occupancy sums 16 prefix terms per worker in
    dict order) and C3 with each unpack pinned to its output partition's worker (the
    shuffle plugin's restrict_task, shuffle/_scheduler_plugin.py:101-115, range sharding
    _shuffle.py:612-617). A step is reset + update_graph + the replay, as in the C2 / C3 legs
(mean of 2 after a warm-up), checked bit-exact
    against the oracle, whose run is the CPU baseline (1 core)."""
    from distributed_amd import graphs

    legs = {}
    for name, g, what in (
            ("c2_16prefixes", graphs.random_dag(args.tasks, args.workers, seed=0, n_inner_prefixes=15),
             "C2 with 16 task prefixes"),
            ("c3_restricted", graphs.shuffle_graph(args.c3_partitions, args.c3_workers, restricted=True),
             "C3 with restricted unpacks (restrict_task)")):
        eng = eng_cls(local)
        eng.load(g, CONFIG)
        eng.reset()
        eng.update_graph()
        eng.run_rounds(-1)  # warm-up
        n_step = 2  # a step as in the C2 / C3 legs: reset + update_graph + the replay
        t0 = time.perf_counter()
        for _ in range(n_step):
            eng.reset()
            eng.update_graph()
            eng.run_rounds(-1)
        dt = (time.perf_counter() - t0) / n_step
        out = eng.placements()
        window = eng.get_window()
        eng.close()
        n = int(len(out["pl_task"]))
        leg = {"metric": f"task placements/sec, {what}", "value": round(n / dt, 1), "unit": "placements/s",
               "seconds_per_replay": round(dt, 4), "placements_per_replay": n, "n_tasks": int(g["n_tasks"]),
               "stream_window": window,
               "n_prefixes": len(g["prefix_names"]),
               "restricted_tasks": int((g["restr_flags"] != 0).sum()) if "restr_flags" in g else 0}
        if not args.no_cpu_baseline:
            from oracle import oracle

            ref = oracle.replay(g, CONFIG, snapshots=False)
            leg["cpu_baseline"] = {"value": round(len(ref["pl_task"]) / ref["seconds"], 1), "unit": "placements/s",
                                   "cores": 1, "kind": "port", "sample": "oracle/replay.cpp, one full replay"}
            leg["parity"] = bool(all(np.array_equal(out[k], ref[k]) for k in (
                "pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route")))
        legs[name] = leg
    return legs


def c_call_latency(eng_cls, local: int, g: dict) -> dict:
    """One task-finished message per dgp_tasks_finished call through the resident kernel,
    driven with ctypes on preallocated buffers (what a C / Cython caller pays): the replay
    protocol over g, each call's new placements read from the mailbox (task / worker)."""
    import ctypes as C

    eng = eng_cls(local)
    eng.load(g, CONFIG, results=False)
    eng.set_resident(True)
    eng.update_graph()
    lib, h = eng.lib, eng.h
    N = int(g["n_tasks"])
    ptask, pworker = np.zeros(N, np.int32), np.zeros(N, np.int32)
    m = {k: np.zeros(1, dt) for k, dt in (("t", np.int32), ("w", np.int32), ("r", np.int64), ("nb", np.int64),
                                          ("a", np.float64), ("b", np.float64), ("st", np.int8))}
    P = {k: v.ctypes.data_as(C.c_void_p) for k, v in m.items()}
    newp = C.c_int64(0)
    n = int(lib.dgp_num_placements(h))
    lib.dgp_get_placements(h, 0, n, ptask.ctypes.data_as(C.c_void_p), pworker.ctypes.data_as(C.c_void_p),
                           None, None, None, None)
    done, calls = 0, 0
    t0 = time.perf_counter()
    while done < n:
        t = int(ptask[done])
        m["t"][0], m["w"][0], m["r"][0] = t, pworker[done], done
        m["nb"][0], m["a"][0], m["b"][0] = g["nbytes"][t], g["start"][t], g["stop"][t]
        rc = lib.dgp_tasks_finished(h, 1, P["t"], P["w"], P["r"], P["nb"], P["a"], P["b"], P["st"], C.byref(newp))
        assert rc == 0 and m["st"][0] == 0
        k = newp.value
        if k:
            lib.dgp_get_placements(h, n, k, ptask[n:].ctypes.data_as(C.c_void_p),
                                   pworker[n:].ctypes.data_as(C.c_void_p), None, None, None, None)
            n += k
        done += 1
        calls += 1
    dt = time.perf_counter() - t0
    eng.set_resident(False)
    st = eng.stats()
    eng.close()
    k = max(st["res_requests"], 1)
    return {"calls": calls, "us_per_call": round(dt / calls * 1e6, 2), "messages_per_s": round(calls / dt, 1),
            "device_us_per_call": {"answer": round(st["res_append_ticks"] / k / 100, 2),
                                   "run_stimuli": round(st["res_run_ticks"] / k / 100, 2),
                                   "publish": round(st["res_publish_ticks"] / k / 100, 2)},
            # when each role last finished a batch, after the request's stimulus was appended
            "role_done_us_after_append": {r: round(st[f"res_role_{r}_ticks"] / k / 100, 2)
                                          for r in ("bld", "pre", "reg", "claim", "exe", "seq", "wlk")}}


def service_leg(eng_cls, local: int, args) -> dict:
    """The drop-in boundary as a live scheduler drives it (service mode): a C2-shaped graph
    (random DAG, fan-in 4, sat 1.1) on 1,024 workers whose completions arrive as
    task-finished messages through dgp_tasks_finished, the replay protocol's order, with the
    new placements' task / worker read back after every call (what GPUPlacementExtension
    does). Two granularities: one call per round (every completion of the previous round's
    placements) and one call per message; each launch-per-call and through the resident
    kernel (dgp_set_resident: mailbox in pinned host memory, no launch / copy / sync per
    call). ``per_message_overlap_ext`` is the extension's own path: each message posted
    (dgp_tasks_finished_post), ``--svc-window-us`` of host work standing in for the reference
    handler's Python before its first decision, then the wait and ``engine.answer``; its
    ``exposed_us_per_call`` is what the engine adds to the handler. Host-inclusive (ctypes
    included); checked bit-exact against the oracle's replay of the same protocol."""
    from distributed_amd import graphs

    g = graphs.random_dag(args.svc_tasks, 1024, seed=5)
    leg = {"metric": "task-finished messages/sec through dgp_tasks_finished (service mode, host-inclusive)",
           "workload": f"C2-shaped random DAG, {args.svc_tasks} tasks x 1024 workers, sat 1.1",
           "n_tasks": int(g["n_tasks"])}
    outs = {}
    cols = ("pl_task", "pl_worker")
    window = args.svc_window_us * 1e-6
    for mode in ("per_round", "per_message", "per_round_resident", "per_message_resident", "per_round_messages",
                 "per_message_resident_ext", "per_message_overlap_ext"):
        eng = eng_cls(local)
        eng.load(g, CONFIG, results=False)
        eng.set_resident("resident" in mode)
        if mode.endswith("_ext"):  # the answers carry the message fields (f3)
            eng.set_task_messages(True)
        if mode == "per_message_overlap_ext":
            eng.set_resident(True)
        eng.update_graph()
        done, calls = 0, 0
        n = eng.num_placements()
        t_msg, n_msg, n_dep = 0.0, 0, 0
        t0 = time.perf_counter()
        while n > done:  # each batch: the previous one's new placements, completed in run_id order
            p = eng.placements(done, n - done, columns=cols)
            t, w = p["pl_task"], p["pl_worker"]
            r = np.arange(done, n, dtype=np.int64)
            nb, a, b = g["nbytes"][t], g["start"][t], g["stop"][t]
            done = n
            if mode.startswith("per_round"):
                _, k = eng.tasks_finished(t, w, r, nb, a, b)
                if mode == "per_round_messages" and k:  # + the batch's compute-task who_has / nbytes
                    tm = time.perf_counter()
                    m = eng.task_messages(n, k)
                    t_msg += time.perf_counter() - tm
                    n_msg += 1
                    n_dep += len(m["dep_task"])
                n += k
                calls += 1
            elif mode == "per_message_overlap_ext":
                # GPUPlacementExtension's path: post the message, run the reference handler's
                # Python up to its first decision (stood in for by `window` of host work: the
                # overlap window tests/ext_driver.py measures), then the answer, the new
                # placements and their message fields through engine.answer
                tl, wl, rl, nbl, al, bl = t.tolist(), w.tolist(), r.tolist(), nb.tolist(), a.tolist(), b.tolist()
                for i in range(len(tl)):
                    eng.tasks_finished_post((tl[i],), (wl[i],), (rl[i],), (nbl[i],), (al[i],), (bl[i],))
                    t_end = time.perf_counter() + window
                    while time.perf_counter() < t_end:
                        pass
                    _, k = eng.tasks_finished_wait()
                    if k:
                        m = eng.answer(n, k, True)[2]
                        n_dep += len(m[1])
                    n += k
                    calls += 1
            else:
                ext = mode == "per_message_resident_ext"
                for i in range(len(t)):
                    _, k = eng.tasks_finished(t[i:i + 1], w[i:i + 1], r[i:i + 1], nb[i:i + 1], a[i:i + 1], b[i:i + 1])
                    if ext and k:  # what GPUPlacementExtension asks per message: the new placements
                        # and their compute-task who_has / nbytes (both from the mailbox)
                        eng.placements(n, k, columns=cols)
                        m = eng.task_messages(n, k)
                        n_dep += len(m["dep_task"])
                    n += k
                    calls += 1
        dt = time.perf_counter() - t0
        eng.set_resident(False)
        outs[mode] = eng.placements()
        if mode == "per_message_resident":
            # the same protocol through the bare C ABI (preallocated buffers, no numpy per
            # call): the engine's own latency per message, without the Python wrapper's
            lat = c_call_latency(eng_cls, local, g)
            leg["per_message_resident_c_abi"] = lat
        eng.close()
        leg[mode] = {"messages_per_s": round(g["n_tasks"] / dt, 1), "calls": calls,
                     "us_per_call": round(dt / max(calls, 1) * 1e6, 1), "seconds": round(dt, 4)}
        if mode == "per_message_overlap_ext":  # what the drop-in adds to the handler's own time
            leg[mode].update(host_window_us=args.svc_window_us,
                             exposed_us_per_call=round(dt / max(calls, 1) * 1e6 - args.svc_window_us, 1))
        if n_msg:  # dgp_task_messages (_task_to_msg fields) per batch, host-inclusive
            leg[mode].update(task_messages_calls=n_msg, task_messages_us_per_call=round(t_msg / n_msg * 1e6, 1),
                             task_messages_dependencies=n_dep)
    if not args.no_cpu_baseline:
        from oracle import oracle

        ref = oracle.replay(g, CONFIG, snapshots=False)
        leg["parity"] = bool(all(np.array_equal(o[k], ref[k]) for o in outs.values() for k in (
            "pl_task", "pl_worker", "pl_comm", "pl_start", "pl_wsnbytes", "pl_route")))
    return leg


def c5_leg(eng_cls, local: int, args, dist, barrier) -> dict:
    """BASELINE.json C5: the 10M-task map + tree-reduce (fan-in 8) DAG on 16,384 workers x 1
    thread, one full replay per rank (one independent scheduler per GPU, rank
    k replaying the generator's seed 3 + k; value = the placements all ranks made / the
    slowest rank's time). Rank 0's graph is pinned by tests/golden/c5_full_digest.json."""
    from distributed_amd import graphs

    rank = int(os.environ.get("RANK", "0"))
    g = graphs.map_tree_reduce(args.c5_map, args.c5_workers, seed=3 + rank)  # one scheduler per GPU
    eng = eng_cls(local)
    eng.load(g, CONFIG)
    barrier()
    t0 = time.perf_counter()
    eng.reset()
    eng.update_graph()
    eng.run_rounds(-1)
    barrier()
    dt = reduce_max(time.perf_counter() - t0, dist)
    out = eng.placements()
    n = int(len(out["pl_task"]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    n_all = reduce_sum(n, dist)
    leg = {"metric": "task placements/sec, C5 (10M-task map + tree-reduce, 16,384 workers)",
           "value": round(n_all / dt, 1), "unit": "placements/s", "n_gpus": world, "scaling": "weak",
           "per_rank_value": round(n / dt, 1),
           "seconds_per_replay": round(dt, 3), "placements_per_replay": n, "n_tasks": int(g["n_tasks"]),
           "n_workers": args.c5_workers,
           "parallelism": f"{world} independent schedulers (rank k: seed 3 + k)" if world > 1 else "single"}
    pin = os.path.join(REPO, "tests", "golden", "c5_full_digest.json")
    if os.path.exists(pin) and rank == 0:  # rank 0 replays the pinned graph
        ref = json.load(open(pin))
        if ref["n_map"] == args.c5_map and ref["n_workers"] == args.c5_workers:
            leg["parity"] = graphs.placement_digest(out) == ref["digest"]
    eng.close()
    if rank == 0 and world == 1 and not args.no_latency:
        # the chain of this replay (dgp_conflict_depth over its placement log) x the link of
        # the global worker-state path (the star at 16,384 workers)
        leg["latency_bound"] = latency_bound(g, out, link_latency_us(eng_cls, local, args.c5_workers), dt * 1e3)
    if int(os.environ.get("RANK", "0")) == 0 and world == 1 and not args.no_cpu_baseline and args.c5_cpu_map > 0:
        # a bounded sample on this box: the same map + tree-reduce shape and worker count,
        # fewer map tasks (the full 10M replay takes the 1-core port minutes). The port's
        # rootish queue scan is O(W) per root (oracle/replay.cpp: argmin over idle_task_count,
        # as scheduler.py:2195-2245), so its rate here falls with W, not with the graph.
        from oracle import oracle

        gs = graphs.map_tree_reduce(args.c5_cpu_map, args.c5_workers)
        ref = oracle.replay(gs, CONFIG, snapshots=False)
        leg["cpu_baseline"] = {"value": round(len(ref["pl_task"]) / ref["seconds"], 1), "unit": "placements/s",
                               "cores": 1, "kind": "port",
                               "sample": f"oracle/replay.cpp on this host, map {args.c5_cpu_map} + tree-reduce "
                                         f"({len(ref['pl_task'])} placements) x {args.c5_workers} workers; the "
                                         "rootish scan is O(W) per root, so the ratio reflects that scan"}
    # the 1-core port on the FULL graph (tools/c5_cpu_full.py, minutes: run once per round on
    # the GPU box's host and committed under profiles/), reported beside the sample
    import glob

    full = sorted(glob.glob(os.path.join(REPO, "profiles", "*_c5_cpu_full.json")))
    if full and rank == 0:
        f = json.load(open(full[-1]))
        leg["cpu_baseline_full"] = {"value": f["placements_per_s"], "unit": "placements/s", "cores": 1, "kind": "port",
                                    "seconds": f["seconds"], "digest_matches_gpu_pin": f["digest_matches_gpu_pin"],
                                    "source": os.path.relpath(full[-1], REPO)}
    return leg


REF_PY_C2 = 22_615.0  # reference placement-only throughput at C2, 1 core


def ref_python_summary(value):
    """The committed timings of the reference's own Python (profiles/ref_python_*.json)."""
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
    out = {"baseline_md_placements_per_s": REF_PY_C2, "multiple_of_baseline_md": round(value / REF_PY_C2, 2)}
    for cfg in ("c2", "c3", "c4"):
        f = os.path.join(here, f"ref_python_{cfg}.json")
        if not os.path.exists(f):
            continue
        r = json.load(open(f))
        keep = {k: r[k] for k in ("placements", "placement_only_s", "replay_s", "balance_s", "steal_requests", "cores",
                                  "python", "dask") if k in r}
        if "placement_only_s" in r:
            keep["placements_per_placement_only_s"] = round(r["placements"] / r["placement_only_s"], 1)
        out[cfg] = keep
    if "c2" in out and "placements_per_placement_only_s" in out["c2"]:
        out["multiple_of_measured_c2"] = round(value / out["c2"]["placements_per_placement_only_s"], 2)
    out["source"] = "tools/ref_python_time.py (build container, /root/reference under python3.9, 1 core)"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tasks", type=int, default=1_000_000)
    ap.add_argument("--workers", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-steal", action="store_true", help="skip the WorkStealing.balance leg")
    ap.add_argument("--steal-tasks", type=int, default=500_000)
    ap.add_argument("--steal-workers", type=int, default=4096)
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 (P2P shuffle, 200k x 512) leg")
    ap.add_argument("--c3-partitions", type=int, default=66_666)
    ap.add_argument("--c3-workers", type=int, default=512)
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 (10M x 16k) leg")
    ap.add_argument("--no-service", action="store_true", help="skip the service-mode (dgp_tasks_finished) leg")
    ap.add_argument("--no-variants", action="store_true", help="skip the 16-prefix C2 / restricted C3 legs")
    ap.add_argument("--svc-tasks", type=int, default=20_000)
    ap.add_argument("--svc-window-us", type=float, default=50.0,
                    help="host work between post and wait in the overlapped service leg (the extension's "
                         "window before its first decision: tests/ext_driver.py us_overlap_window)")
    ap.add_argument("--c5-map", type=int, default=8_750_000)
    ap.add_argument("--c5-workers", type=int, default=16_384)
    ap.add_argument("--c5-cpu-map", type=int, default=200_000, help="map tasks of the C5 CPU-baseline sample")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"))
    ap.add_argument("--no-latency", action="store_true", help="skip the link-latency chain and the latency bound")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        # one GPU per rank; --dist-backend gloo rehearses the protocol with ranks sharing
        # the GPUs there are (RCCL needs a GPU of its own per rank)
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend)

    from distributed_amd import graphs
    from distributed_amd.engine import PlacementEngine

    g = graphs.random_dag(args.tasks, args.workers, seed=rank)  # one scheduler per GPU, its own graph
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

    # placements made by update_graph (the initial wave) precede the replay kernel's
    eng.reset()
    eng.update_graph()
    n_ug = eng.num_placements()
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
    elapsed = reduce_max(elapsed, dist)
    total_placements = reduce_sum(placements, dist) * args.steps  # the distinct work of all ranks
    value = total_placements / elapsed

    out = eng.placements()
    agree = None
    if dist is not None and not args.no_cpu_baseline:
        # every rank checks its own replay against the oracle (its own graph); all must agree
        from oracle import oracle

        ref = oracle.replay(g, CONFIG, snapshots=False)
        ok = all(np.array_equal(out[k], ref[k]) for k in ("pl_task", "pl_worker", "pl_comm", "pl_start",
                                                           "pl_wsnbytes", "pl_route"))
        agree = reduce_sum(1.0 if ok else 0.0, dist) == world
    steal = None
    if not args.no_steal:  # every rank takes part (sharded thief rows)
        steal = steal_leg(eng, args, world, dist, barrier)
    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "placements/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int64+f64",
        "data": "synthetic",
        "config": {"workload": "C2: random DAG, fan-in<=4 (window 4W), lognormal(10,2) nbytes, roots N/10, "
                               "workers x 1 thread, worker-saturation 1.1; full replay per step",
                   "n_tasks": args.tasks, "n_workers": args.workers,
                   "parallelism": f"{world} independent schedulers, one per GPU (rank k: seed k)" if world > 1
                   else "single", "placements_per_step": placements},
    }
    if world > 1:
        result["per_rank_value"] = round(placements * args.steps / elapsed, 1)
    if rank == 0:
        n_waves = eng.stats()["rounds"]
        # bytes of the placements each kernel makes: update_graph's initial wave, then the replay
        ab = {"update_graph": algorithmic_bytes(g, out["pl_task"][:n_ug], 1),
              "replay": algorithmic_bytes(g, out["pl_task"][n_ug:], max(n_waves - 1, 0))}
        kernels = {}
        for name, nbytes in ab.items():
            ms, n = kt_total.get(name, (0.0, 0))
            if n == 0:
                continue
            per_launch_bytes = nbytes / (n / args.steps)  # every launch of a step shares its placements
            avg_ms = ms / n
            kernels[name] = {"total_ms_per_step": ms / args.steps, "launches_per_step": n // args.steps,
                             "avg_us": 1e3 * avg_ms, "bytes_per_launch": per_launch_bytes,
                             "achieved_GBs": per_launch_bytes / (avg_ms * 1e-3) / 1e9}
        dom = max(kernels, key=lambda k: kernels[k]["total_ms_per_step"])
        ach = kernels[dom]["achieved_GBs"]
        # the replay is bound by its ordered chain of stimuli (latency_bound below), not by
        # HBM: achieved / peak is the fraction of the HBM roofline the ordered replay reaches
        result["roofline"] = {"kernel": dom, "bound": "latency", "roofline_axis": "hbm", "achieved": round(ach, 4),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 8),
                              "traffic": None}
        # HBM bytes per launch of the replay kernel, from the committed rocprofv3 --pmc passes
        # (tools/pmc_traffic.py); only reported for the workload they were measured on
        tf = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "hbm_traffic.json")
        if dom == "replay" and os.path.exists(tf):
            t = json.load(open(tf))
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
            from pmc_traffic import engine_source_hash

            if (t.get("n_tasks"), t.get("n_workers")) != (args.tasks, args.workers):
                pass
            elif t.get("src_sha256") != engine_source_hash():  # measured on other engine sources
                result["roofline"]["traffic_source"] = f"stale ({t.get('source')}): engine sources changed since"
            else:
                result["roofline"]["traffic"] = round(t["traffic_bytes_per_launch"], 1)
                result["roofline"]["traffic_source"] = t.get("source")
        # a measured copy peak beside the 8 TB/s datasheet figure: a 2 GiB
        # device-to-device copy, read + written bytes over its event-timed duration
        try:
            import torch

            src = torch.empty(1 << 31, dtype=torch.uint8, device=f"cuda:{local}")
            dst = torch.empty_like(src)
            dst.copy_(src)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = None
            for _ in range(5):
                e0.record()
                dst.copy_(src)
                e1.record()
                torch.cuda.synchronize()
                ms_c = e0.elapsed_time(e1)
                best = ms_c if best is None else min(best, ms_c)
            result["roofline"]["copy_peak_measured"] = round(2 * src.numel() / (best * 1e-3) / 1e9, 1)
            del src, dst
            torch.cuda.empty_cache()
        except Exception as ex:  # reported, never fatal
            result["roofline"]["copy_peak_measured"] = f"unavailable: {ex}"
        if not args.no_latency:
            link_us = link_latency_us(PlacementEngine, local)
            result["latency_bound"] = latency_bound(g, out, link_us, 1e3 * elapsed / args.steps)
        result["kernels"] = {k: {kk: round(vv, 3) for kk, vv in v.items()} for k, v in kernels.items()}
        result["config"]["waves"] = int(n_waves)
        result["config"]["stream_window"] = eng.get_window()  # the stream-kernel build that ran (32 / 64)
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
        # the reference's own Python (22,615 placements/s placement-only, C2, one
        # core) is the north_star's "reference CPU placement throughput": vs_baseline is the
        # multiple of it; profiles/ref_python_*.json are this container's own timings of the
        # reference (tools/ref_python_time.py: it never travels to the GPU box)
        result["vs_baseline"] = round(value / REF_PY_C2, 2)
        result["reference_python"] = ref_python_summary(value)
        if agree is not None:
            result["parity_all_ranks"] = agree
        if steal is not None:
            result["steal"] = steal
    eng.close()
    if rank == 0 and not args.no_c3:
        result["c3"] = c3_leg(PlacementEngine, local, args, result.get("latency_bound", {}).get("link_us"))
    if rank == 0 and not args.no_variants:
        result.update(variant_legs(PlacementEngine, local, args))
    if rank == 0 and not args.no_service:
        result["service"] = service_leg(PlacementEngine, local, args)
    if not args.no_c5:  # every rank takes part (barriers, max over ranks)
        c5 = c5_leg(PlacementEngine, local, args, dist, barrier)
        if rank == 0:
            result["c5"] = c5
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
