"""Diagnostic: k_refill time (HIP events) for the queue 20 steady-state steps leave (~10 k resets at
65 536 envs), averaged over 8 refills, for the library named by CTR_REACH_AMD_LIB."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
kw = {}
if len(sys.argv) > 2 and sys.argv[2] == "rigid":      # configs[1]: rigid model, RK4 at 100 steps/m
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
for i in range(200):
    env.step_raw(acts[i % 8])
    if i % 20 == 19:
        env.refill_pool()
ts, counts = [], []
for rep in range(8):
    for i in range(20):
        env.step_raw(acts[i % 8])
    torch.cuda.synchronize()
    counts.append(int(env.refill[0].item()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    env.refill_pool()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) * 1e3)
print("k_refill %.1f us (queue %d entries on average)" % (sum(ts) / len(ts), sum(counts) // len(counts)))
