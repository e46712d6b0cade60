"""Diagnostic: k_refill time (HIP events) against the resumable refill's budget, in the steady
state of the headline (65 536 envs, staggered episode clocks, refill every 20 steps, pool depth
64): per refill, the time and the resets it left suspended, averaged over 8 refills after 30
untimed periods.  Budget 0 = every FK runs to its end in the refill that starts it.
usage: python tools/time_refill_budget.py [n_envs] [budgets, comma-separated]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
budgets = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "0,6,8,10,12,16").split(",")]
R = 20
for budget in budgets:
    env = CtrReachVecEnv(n, device="cuda", seed=0, refill_interval=R, pool_depth=64, refill_budget=budget,
                         record_info=False)
    env.reset()
    g0 = torch.Generator(device="cpu")
    g0.manual_seed(2)
    env.t.copy_(torch.randint(0, 150, (n,), generator=g0, dtype=torch.int32))
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    hi = torch.tensor(env.action_space.high, device="cuda")
    acts = [((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
    for i in range(30 * R):
        env.step_raw(acts[i % 8])
    ts, queued, carried = [], [], []
    for rep in range(8):
        for i in range(R - 1):
            env.step_raw(acts[i % 8])
        torch.cuda.synchronize()
        # the period's last step, then its refill, timed alone
        env._steps_since_refill = 0          # keep step_raw from refilling; refill_pool below does
        env.step_raw(acts[R % 8])
        torch.cuda.synchronize()
        queued.append(int(env.refill[0].item()))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        env.refill_pool()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
        carried.append(sum(env.carried()))
    print("budget %2d (carry %s): k_refill %.1f us (min %.1f), queue %d, suspended after %d" %
          (budget, "on" if env.carry is not None else "off", sum(ts) / len(ts), min(ts),
           sum(queued) // len(queued), sum(carried) // len(carried)), flush=True)
    del env
    torch.cuda.empty_cache()
