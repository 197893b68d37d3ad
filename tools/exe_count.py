"""C2 replay wall time vs executor count (GPU; DGP_STREAM_DEBUG bits 8..11 = executors):
python tools/exe_count.py [n_tasks] [counts...]"""
import os, subprocess, sys
n = sys.argv[1] if len(sys.argv) > 1 else "1000000"
counts = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8, 11]
code = ("import sys,time;sys.path.insert(0,'.');from distributed_amd import graphs;"
        "from distributed_amd.engine import PlacementEngine as PE;g=graphs.random_dag(%s,1024,seed=0);"
        "e=PE(0,window=32);e.load(g,{'saturation':1.1});ts=[]\n"
        "for i in range(2):\n e.reset();e.update_graph();t=time.time();e.run_rounds(-1);ts.append(time.time()-t)\n"
        "print(f'{min(ts):.4f} {e.num_placements()/min(ts)/1e6:.3f}')" % n)
for c in counts:
    env = dict(os.environ, DGP_STREAM_DEBUG=str(c << 8))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    print(f"executors {c:2d}: {out.stdout.strip()} {out.stderr.strip()[-200:] if out.returncode else ''}", flush=True)
