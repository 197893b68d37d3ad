import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_amd.engine import PlacementEngine
from oracle import oracle
g, cfg, exp, meta = oracle.load_fixture(os.path.join("tests/golden", sys.argv[1]))
with PlacementEngine(0) as e:
    e.load(g, cfg)
    try:
        e.replay()
        print("no error")
    except Exception as ex:
        print(ex)
    buf = np.zeros(64 * 8)
    e.lib.dgp_debug_buf.argtypes = [C.c_void_p, C.c_void_p]
    e.lib.dgp_debug_buf(e.h, buf.ctypes.data_as(C.c_void_p))
b = buf.reshape(64, 8)
print("r", b[0, 5], "eb_first", b[0, 6], "pre", b[0, 7])
for i in range(20):
    print(i, b[i, :5].astype(np.int64))
