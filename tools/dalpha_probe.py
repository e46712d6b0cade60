"""Diagnostic: the distribution of |delta|, how far an RK45 stage input's angle difference
(alpha_1 - alpha_0, alpha_2 - alpha_0) lies from the attempt's start state (tools/dalpha_probe.c,
the CPU oracle with a stage hook), on env-trajectory joints.  A stage's sin/cos reached from the
trig of y by a rotation through delta needs a kernel for |delta| of this size.
usage: python tools/dalpha_probe.py [n_envs]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import oracle  # noqa: E402
from sim_sched import trajectory_joints  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
q = np.ascontiguousarray(trajectory_joints(n, 12), dtype=np.float32)
L = ctypes.CDLL(os.path.join(ROOT, "tools", "libdalpha_probe.so"))
P = ctypes.c_void_p
ci = ctypes.c_int
L.dalpha_hist.argtypes = [P]
L.oracle_fk_ex.argtypes = [P, P, ctypes.c_int64, P, ci, ci, ci, P, P, P, P, P]
systems = oracle.make_systems()
tip = np.zeros((n, 3))
cnt = [np.zeros(n, np.int32) for _ in range(4)]
L.dalpha_reset()
L.oracle_fk_ex(q.ctypes.data, None, n, ctypes.cast(systems, P), 0, 0, 0, tip.ctypes.data, *[c.ctypes.data for c in cnt])
h = np.zeros(80, np.int64)
L.dalpha_hist(h.ctypes.data)
h = h.reshape(2, 40)
for k, name in enumerate(("a1 - a0", "a2 - a0")):
    tot = h[k].sum()
    cum = np.cumsum(h[k])
    print("%s: %d stage inputs" % (name, tot))
    for b in range(0, 14):
        print("   |delta| >= 2^-%-2d  %.4f" % (b + 1, cum[b] / tot))
