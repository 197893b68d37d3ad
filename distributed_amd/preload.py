"""``distributed.scheduler.preload: [distributed_amd.preload]`` (distributed.yaml): installs
the drop-ins configured under ``distributed.scheduler.gpu-placement`` on the scheduler
before it starts (config.install)."""
from __future__ import annotations


def dask_setup(scheduler) -> None:
    from .config import install

    install(scheduler)
