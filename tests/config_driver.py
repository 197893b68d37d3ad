"""distributed.scheduler.gpu-placement.* in a real reference ``Scheduler`` (python3.9 + the
reference via tests/golden/_refshim.py; build container only). Called by tests/test_ext.py.
Prints one JSON line per case: which extensions / plugins the started scheduler holds."""
from __future__ import annotations

import asyncio
import json
import os
import sys
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.dirname(HERE))
warnings.filterwarnings("ignore")
import _refshim  # noqa: E402

_refshim.install()
import dask  # noqa: E402
from distributed.scheduler import Scheduler  # noqa: E402

from distributed_amd import config as C  # noqa: E402


def describe(s) -> dict:
    st = s.extensions.get("stealing")
    return dict(extensions=sorted(s.extensions), stealing=type(st).__name__ if st is not None else None,
                placement=type(s.extensions.get("gpu-placement")).__name__,
                plugins=sorted(type(p).__name__ for p in s.plugins.values()),
                steal_handler=getattr(s.stream_handlers.get("steal-response"), "__self__", None) is st if st else None,
                stealing_callback="stealing" in s.periodic_callbacks,
                task_finished=getattr(s.stream_handlers.get("task-finished"), "__qualname__", ""))


async def run(case: str) -> dict:
    kw = dict(dashboard_address=None, dashboard=False, host="127.0.0.1", port=0)
    cfg = {"distributed.scheduler.gpu-placement.enabled": case != "default",
           "distributed.scheduler.work-stealing": case != "no_stealing"}
    with dask.config.set(cfg):
        if case == "extensions":
            s = Scheduler(extensions=C.scheduler_extensions(), **kw)
        else:
            s = Scheduler(preload=["distributed_amd.preload"], **kw)
        await s
        out = describe(s)
        await s.close()
    out["case"] = case
    return out


if __name__ == "__main__":
    for c in sys.argv[1:] or ("default", "preload", "no_stealing", "extensions"):
        print(json.dumps(asyncio.run(run(c))), flush=True)
