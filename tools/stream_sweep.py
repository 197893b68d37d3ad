"""Replay throughput of the stream engine under env-var knobs (diagnostic, GPU).

    python tools/stream_sweep.py VAR v1 v2 ... [--tasks N]
Each value runs in its own child process (the knob is read at engine setup).
"""
import os
import subprocess
import sys

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import time
    from distributed_amd import graphs
    from distributed_amd.engine import PlacementEngine
    n = int(sys.argv[2])
    g = graphs.random_dag(n, 1024, seed=0)
    e = PlacementEngine(0)
    e.load(g, {"saturation": 1.1})
    best = 1e9
    for it in range(3):
        e.reset(); e.update_graph(); t = time.time(); e.run_rounds(-1); best = min(best, time.time() - t)
    st = e.stats()
    print(f"  {os.environ.get('SWEEP_TAG')}: {best:.3f}s {e.num_placements() / best / 1e6:.3f} M/s  REG busy/stim {st['wave_phase3'] / n:.0f}"
          f" A {st['cyc_local_steps'] / n:.0f} B {st['cyc_global'] / n:.0f} win-full {st['stall0'] / n:.0f} exe {st['wave_phase5'] / n:.0f}"
          f" batches {st['stall3']} | fetch {st['cyc_setup'] / n:.0f} masks {st['cyc_reserve'] / n:.0f} sumloop {st['cyc_max_step'] / n:.0f}", flush=True)
    sys.exit(0)
var, vals = sys.argv[1], [v for v in sys.argv[2:] if not v.startswith("--")]
n = 1_000_000
for v in vals:
    env = dict(os.environ, **{var: v, "SWEEP_TAG": f"{var}={v}"})
    rc = subprocess.call([sys.executable, os.path.abspath(__file__), "--child", str(n)], env=env)
    if rc:
        sys.exit(rc)
