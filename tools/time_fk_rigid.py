"""Diagnostic: latency of configs[1]'s FK outside k_step (rigid model, RK4 at 100 steps/m): ctr_fk
(one lane per FK, fk_lane_rk4 -- what k_refill and k_reset run) on freshly sampled joints, for a
refill-sized batch (1 212 FKs = 606 resets) and a full one, timed with HIP events behind a busy
kernel (no launch latency in the number).  Also the pool refill of 606 queued resets.
usage: python tools/time_fk_rigid.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

n = 4096
env = CtrReachVecEnv(n, device="cuda", seed=0, refill_interval=1000, pool_depth=16, integrator="rk4",
                     rk4_steps_per_m=100, model="rigid")
env.reset()
torch.cuda.synchronize()
q = torch.cat([env.pool_qd.reshape(-1, 6), env.pool_q0.reshape(-1, 6)])      # fresh samples


def timed(fn, reps=10):
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(200000)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for m in (64, 1212, 16384, 65536):
    qm = q[:m].contiguous()
    out = env.forward_kinematics(qm)
    print("ctr_fk rigid RK4, %6d fresh joints: %.1f us" % (m, timed(lambda: env.forward_kinematics(qm))), flush=True)
