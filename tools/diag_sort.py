"""Diagnostic: how much would grouping environments with similar RK45 work into the same wave
shorten the FK launch?  Times k_fk (HIP events) on 65 536 env-trajectory joints in their natural
order and sorted by the oracle's per-segment attempt signature (fresh, i.e. an upper bound for a
sort made from the previous step's counts), globally and inside blocks of 256 / 1024 envs.

usage: python tools/diag_sort.py [steady]"""
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
# "steady": the bench's batch (episode clocks staggered over [0, 150), 300 steps: resets at their
# natural rate, most configurations drifted); default: 20 steps after reset() (fresh samples)
steady = len(sys.argv) > 1 and sys.argv[1] == "steady"
if steady:
    env.t.copy_(torch.randint(0, env.max_steps_per_episode, (n,), generator=torch.Generator().manual_seed(17),
                              dtype=torch.int32))
for k in range(300 if steady else 20):
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


def in_blocks(o_key, b):
    """The same key order applied inside each block of b consecutive envs (a workgroup's rows)."""
    rank = np.empty(n, np.int64)
    rank[o_key] = np.arange(n)
    return np.concatenate([b0 + np.argsort(rank[b0:b0 + b], kind="stable") for b0 in range(0, n, b)])


for name in ("lag1 signature", "lag1 total", "lag1 nseg,total", "lag16 signature"):
    for b in (256, 1024):
        orders["%s /%d" % (name, b)] = in_blocks(orders[name], b)


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


time_fk(q, reps=400)                    # sustained-load clocks first (the first launches run slower)
orders["natural (again, last)"] = orders["natural"]
for name, o in orders.items():
    print("%-26s k_fk %.1f us" % (name, time_fk(q[o])))
