"""Diagnostic: how much would grouping environments with similar RK45 work into the same wave
shorten the FK launch?  Times k_fk (HIP events) on 65 536 env-trajectory joints in their natural
order and sorted by the oracle's per-segment attempt signature (fresh, i.e. an upper bound for a
sort made from the previous step's counts)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

n = 65536
env = CtrReachVecEnv(n, device="cuda", seed=0)
env.reset()
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
for k in range(20):
    env.step(((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous())
hist = []
for k in range(17):
    hist.append(env.joints.cpu().numpy().copy())
    env.step(((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous())
q = env.joints.cpu().numpy()


def key_orders(qq, tag):
    att = oracle.fk_segattempts(qq)
    tot = att.sum(1)
    nseg = (att > 0).sum(1)
    keys = [tuple(np.cumsum(a[a > 0])) for a in att]
    return {
        tag + " signature": np.array(sorted(range(n), key=lambda i: (len(keys[i]), keys[i]))),
        tag + " total": np.argsort(tot, kind="stable"),
        tag + " nseg,total": np.argsort(nseg * 64 + tot, kind="stable"),
        tag + " nseg,first2": np.argsort((nseg * 64 + att[:, 0]) * 64 + att[:, 0] + att[:, 1], kind="stable"),
    }


orders = {"natural": np.arange(n)}
orders.update(key_orders(q, "fresh"))
for lag in (1, 4, 16):
    orders.update(key_orders(hist[-lag], "lag%d" % lag))


def time_fk(qq, reps=20):
    qt = torch.tensor(qq, device="cuda")
    env.forward_kinematics(qt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        env.forward_kinematics(qt)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, o in orders.items():
    print("%-15s k_fk %.1f us" % (name, time_fk(q[o])))
