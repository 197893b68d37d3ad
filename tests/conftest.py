import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP engine parity / smoke)")
    config.addinivalue_line("markers", "slow: long CPU test")


def golden_files():
    """Placement replay fixtures (tests/golden/gen_golden.py, gen_service.py)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.endswith(".npz")
                  and not f.startswith(("steal_", "svc_steal_", "svcaddw_", "svcgraph_", "svcgdep_", "svcev_",
                                            "svcrs_", "svcrt_", "svcwl_", "svcp2p_", "svcgrst_", "svcgprio_", "svcpfx_",
                                            "svcgrec_", "svcrel_", "svccan_", "svcretry_")))


def svc_second_graph_files():
    """Service-mode message streams with a second graph submitted (gen_service.py second-graph)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcgraph_") and f.endswith(".npz"))


def svc_dep_graph_files():
    """Service-mode streams with a later graph that depends on earlier tasks (gen_service.py
    second-graph svcgdep_*; svcgrec_*: some of them released, recomputed by that stimulus)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith(("svcgdep_", "svcgrec_")) and f.endswith(".npz"))


def svc_restr_graph_files():
    """Service-mode streams with a later graph carrying worker restrictions (gen_service.py
    second-graph svcgrst_*): appended deferred, the scheduler's stimulus, resync + rows."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcgrst_") and f.endswith(".npz"))


def svc_prio_graph_files():
    """Service-mode streams with a later graph whose user priority outranks the earlier tasks
    (gen_service.py second-graph svcgprio_*): appended deferred, re-ranked, resynced."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcgprio_") and f.endswith(".npz"))


def second_graph(g, z, with_results=False):
    """A ``svcgraph_*`` fixture's second graph over the engine-wide tables: priorities after
    the first graph's, its groups after the first graph's groups, the same prefixes; with
    ``with_results`` also its tasks' completion reports (from the message stream)."""
    import numpy as np

    G1 = len(g["group_prefix"])
    h = dict(dep_ptr=z["g2_dep_ptr"], dep_idx=z["g2_dep_idx"], prio=z["g2_prio"] + int(g["prio"].max()) + 1,
             prefix_id=z["g2_prefix_id"], group_id=z["g2_group_id"] + G1, wanted=z["g2_wanted"],
             rootish_override=z["g2_rootish_override"], prefix_default_dur=g["prefix_default_dur"],
             group_prefix=np.concatenate([g["group_prefix"], g["group_prefix"]]))
    if with_results:
        n1, n2 = g["n_tasks"], len(h["prio"])
        nb, a, b = np.zeros(n2, np.int64), np.zeros(n2), np.zeros(n2)
        for t, x, s0, s1 in zip(z["msg_task"], z["msg_nbytes"], z["msg_start"], z["msg_stop"]):
            if t >= n1:
                nb[t - n1], a[t - n1], b[t - n1] = x, s0, s1
        h.update(nbytes=nb, start=a, stop=b)
    return h


def svc_add_worker_files():
    """Service-mode message streams with workers joining (tests/golden/gen_service.py add-workers)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcaddw_") and f.endswith(".npz"))


def svc_event_files():
    """Service-mode streams with the other worker stimuli interleaved (gen_service.py events)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcev_") and f.endswith(".npz"))


def svc_resync_files():
    """Service streams with stimuli the scheduler decides itself, then resyncs (gen_service.py resync)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcrs_") and f.endswith(".npz"))


def svc_retire_files():
    """Service streams where drained workers retire, followed on the device (gen_service.py resync svcrt_*)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcrt_") and f.endswith(".npz"))


def svc_release_files():
    """Service streams where clients release results in memory (gen_service.py resync svcrel_*)
    and wanted tasks in any state: cancelled work with what it releases and forgets (svccan_*)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith(("svcrel_", "svccan_")) and f.endswith(".npz"))


def svc_retry_files():
    """Service streams with task-erred reports that do not err -- retries and stale runs,
    re-placed by the engine (gen_service.py resync svcretry_*)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcretry_") and f.endswith(".npz"))


def svc_loss_files():
    """Service streams where workers with processing tasks / sole replicas are lost, decided
    on the device (gen_service.py resync svcwl_*)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcwl_") and f.endswith(".npz"))


def svc_p2p_files():
    """The P2P shuffle's scheduler-side lifecycle (gen_service.py p2p)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svcp2p_") and f.endswith(".npz"))


def svc_steal_files():
    """Service-mode message streams with confirmed steals (tests/golden/gen_service.py)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("svc_steal_") and f.endswith(".npz"))


def steal_files():
    """WorkStealing balance fixtures (tests/golden/gen_steal.py)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("steal_") and f.endswith(".npz")
                  and f != STEAL_REFTESTS)


# the reference's own balance unit scenarios, many problems in one file (gen_steal_ref.py)
STEAL_REFTESTS = "steal_reftests.npz"


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
