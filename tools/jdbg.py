"""Debug: one join call of the C4 workload (used with an experiment build via GF_LIB_PATH)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import spatialflink_amd as sf  # noqa: E402
from spatialflink_amd import _lib  # noqa: E402

BEIJING = (115.50000, 117.60000, 39.60000, 41.10000)
no, nq = 10_000_000, 1_000_000
g = sf.UniformGrid(1000, *BEIJING)
x, y = sf.synthetic_uniform(11, no, *BEIJING)
qx, qy = sf.synthetic_uniform(21, nq, *BEIJING)
import numpy as np  # noqa: E402
wo = sf.PointWindow.from_numpy(x, y, np.arange(no, dtype=np.int64), device=0)
wq = sf.PointWindow.from_numpy(qx, qy, np.arange(nq, dtype=np.int64), device=0)
ctx = _lib.context(0)
cap = 4 * (no + nq)
pairs = torch.empty(2 * cap, dtype=torch.int32, device="cuda")
n = C.c_int64()
po, pq = wo.c_struct(), wq.c_struct()
st = _lib.lib().gf_join_pp(ctx.handle, C.byref(g.c_grid), C.byref(g.c_grid), C.byref(po), C.byref(pq), 0.001, 0, 0,
                           pairs.data_ptr(), cap, C.byref(n))
torch.cuda.synchronize()
print("status", st, "pairs", n.value, flush=True)
