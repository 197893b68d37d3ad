"""The drop-ins from dask.config (``distributed.scheduler.gpu-placement.*``).

The reference picks its scheduler extensions from ``DEFAULT_EXTENSIONS`` and drops
``"stealing"`` when ``distributed.scheduler.work-stealing`` is off (scheduler.py:178-193,
:3890-3897). The same rule with the GPU drop-ins:

* ``scheduler_extensions()`` -- the ``extensions=`` mapping for ``Scheduler(...)``:
  ``DEFAULT_EXTENSIONS`` plus ``"gpu-placement"`` when ``gpu-placement.enabled``, and
  ``GPUWorkStealing`` as ``"stealing"`` when ``gpu-placement.stealing`` and
  ``work-stealing`` are on;
* ``install(scheduler)`` -- the same on a constructed scheduler before it starts (what the
  ``distributed_amd.preload`` module does from ``distributed.scheduler.preload``).

Defaults: ``gpu-placement.yaml`` beside this file, merged into dask.config at import.
"""
from __future__ import annotations

import functools
import os

KEY = "distributed.scheduler.gpu-placement"
DEFAULTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gpu-placement.yaml")


def _dask_config():
    import dask
    import yaml

    with open(DEFAULTS) as f:
        dask.config.update_defaults(yaml.safe_load(f))
    return dask.config


def settings() -> dict:
    """``distributed.scheduler.gpu-placement.*`` and ``work-stealing`` as read now."""
    cfg = _dask_config()
    return dict(enabled=bool(cfg.get(f"{KEY}.enabled")), stealing=bool(cfg.get(f"{KEY}.stealing")),
                device=int(cfg.get(f"{KEY}.device")), validate=bool(cfg.get(f"{KEY}.validate")),
                work_stealing=bool(cfg.get("distributed.scheduler.work-stealing")))


def scheduler_extensions(base: dict | None = None) -> dict:
    """The ``extensions=`` mapping of ``Scheduler`` under the current config (the reference's
    ``DEFAULT_EXTENSIONS`` rule, scheduler.py:3890-3894, with the GPU drop-ins)."""
    st = settings()
    if base is None:
        from distributed.scheduler import DEFAULT_EXTENSIONS

        base = DEFAULT_EXTENSIONS
    ext = dict(base)
    if not st["work_stealing"]:
        ext.pop("stealing", None)
    if st["enabled"]:
        from .ext import GPUPlacementExtension
        from .stealing import GPUWorkStealing

        if st["stealing"] and st["work_stealing"]:
            ext["stealing"] = functools.partial(GPUWorkStealing, device=st["device"], validate=st["validate"])
        ext["gpu-placement"] = functools.partial(GPUPlacementExtension, device=st["device"], validate=st["validate"])
    return ext


def install(scheduler) -> dict:
    """Install the configured drop-ins on ``scheduler`` (constructed, not yet started:
    the preload hook). A reference ``WorkStealing`` already installed is replaced by
    ``GPUWorkStealing`` (its plugin entry, ``steal-response`` handler and events log are
    re-registered by the new one; its periodic callback starts with the plugins, after the
    preloads, scheduler.py:4099-4109). Returns what was installed."""
    st = settings()
    done = {}
    if not st["enabled"]:
        return done
    from .ext import GPUPlacementExtension
    from .stealing import GPUWorkStealing

    exts = scheduler.extensions
    old = exts.get("stealing")
    if st["stealing"] and st["work_stealing"] and old is not None and not isinstance(old, GPUWorkStealing):
        if "stealing" in scheduler.periodic_callbacks:
            raise RuntimeError("gpu-placement: the scheduler's work stealing has already started")
        for name, plugin in list(scheduler.plugins.items()):
            if plugin is old:
                del scheduler.plugins[name]
        exts["stealing"] = done["stealing"] = GPUWorkStealing(scheduler, device=st["device"], validate=st["validate"])
    if not isinstance(exts.get("gpu-placement"), GPUPlacementExtension):
        exts["gpu-placement"] = done["gpu-placement"] = GPUPlacementExtension(
            scheduler, device=st["device"], validate=st["validate"])
    return done
