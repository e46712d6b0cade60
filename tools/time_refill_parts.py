"""Diagnostic: k_refill's fixed cost vs its work, for the library named by CTR_REACH_AMD_LIB.
After 20 steady-state steps the queue holds the resets they took; the refill of that queue is timed
(HIP events), then a refill of the now empty queue (launch + table staging + the ticket only).
usage: python tools/time_refill_parts.py [n_envs] [rigid]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv, _abi  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
kw = {}
if len(sys.argv) > 2 and sys.argv[2] == "rigid":
    kw = dict(integrator="rk4", rk4_steps_per_m=100, model="rigid")
env = CtrReachVecEnv(n, device="cuda", seed=0, refill_interval=1000, pool_depth=32, **kw)
env.reset()
g0 = torch.Generator(device="cpu")
g0.manual_seed(2)
env.t.copy_(torch.randint(0, 150, (n,), generator=g0, dtype=torch.int32))
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
acts = [((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
sp = _abi.stream_ptr()


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


refill = lambda: _abi.check(env.lib.ctr_pool_refill(env.cfg, env._batch, sp), "ctr_pool_refill")  # noqa: E731
for i in range(200):
    env.step_raw(acts[i % 8])
    if i % 20 == 19:
        refill()
full, empty, counts = [], [], []
for rep in range(8):
    for i in range(20):
        env.step_raw(acts[i % 8])
    torch.cuda.synchronize()
    counts.append(int(env.refill[0].item()))
    full.append(timed(refill))
    empty.append(timed(refill))
print("%d envs%s: k_refill %.1f us for %d queued resets; %.1f us with the queue empty"
      % (n, " rigid" if kw else "", sum(full) / len(full), sum(counts) // len(counts), sum(empty) / len(empty)))
