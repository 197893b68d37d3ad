"""Per-message host cost of the drop-in against the reference's own handler (build container
only: needs /root/reference and python3.9, as tests/test_ext.py).

Runs tests/ext_driver.py on each fixture: the unmodified reference with a SchedulerPlugin
registered (``--plain --plugin``) and GPUPlacementExtension (overlapped engine call, the
stand-in engine's time subtracted) side by side in two processes at the same time (this
machine is shared: back-to-back runs differ by up to 2x), ``--reps`` pairs, and prints
min / median of each with the extension's overlap window (post -> first decision). The
composed cost on the box is the extension's host cost plus bench.py's
``service.per_message_overlap_ext.exposed_us_per_call``.

    python tools/dropin_cost.py [--reps 3] [--cpu] [fixture.npz ...]
"""
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY39 = "/opt/conda/bin/python3.9"


def start(fixture, *flags, core=None):
    env = dict(os.environ, PYTHONHASHSEED="0")
    env.pop("PYTHONPATH", None)
    pin = ["taskset", "-c", str(core)] if core is not None else []  # one core each: no migrations
    return subprocess.Popen([*pin, PY39, os.path.join(REPO, "tests", "ext_driver.py"), *flags, fixture],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=REPO)


def result(proc):
    out, err = proc.communicate(timeout=1200)
    assert proc.returncode == 0, err[-2000:]
    return json.loads([x for x in out.splitlines() if x.startswith("{")][-1])


def main():
    args = sys.argv[1:]
    reps = 3
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    key = "us_per_message"
    if "--cpu" in args:  # process CPU time: what other tenants of the machine do not move
        args.remove("--cpu")
        key = "cpu_us_per_message"
    fixtures = args or ["c5mini_sat1.1.npz", "c2var_sat1.1.npz"]
    res = {}
    for fx in fixtures:
        plain, ext, win, p10 = [], [], [], []
        for _ in range(reps):
            # the pair runs at the same time: whatever else loads the machine loads both
            pp, pe = start(fx, "--plain", "--plugin", core=2), start(fx, "--novalidate", core=5)
            plain.append(result(pp)[key])
            r = result(pe)
            ext.append(r[key.replace("message", "message_host")])
            win.append(r["us_overlap_window"])
            p10.append(r["us_overlap_window_p10_p50"][0])
        res[fx] = dict(reference_us=dict(min=min(plain), median=statistics.median(plain)),
                       extension_host_us=dict(min=min(ext), median=statistics.median(ext)),
                       overlap_window_us=dict(mean=statistics.median(win), p10=statistics.median(p10)),
                       reps=reps, messages=r["messages"], clock=key)
        print(json.dumps({fx: res[fx]}), flush=True)
    return res


if __name__ == "__main__":
    main()
