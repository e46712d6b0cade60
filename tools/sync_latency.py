"""Diagnostic: the fixed host cost of a timed window (sync, clock, work, sync, clock) on this box,
for an empty kernel and for configs[1]'s captured 20-step graph, ending the window with
  block  torch.cuda.synchronize()
  poll   an event recorded after the work, polled with event.query() until it completes, then
         torch.cuda.synchronize() (which then returns at once)
Medians of 200 (empty) / 30 (graph) windows.  usage: python tools/sync_latency.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402


def end_block():
    torch.cuda.synchronize()


def end_poll():
    ev = torch.cuda.Event()
    ev.record()
    while not ev.query():
        pass
    torch.cuda.synchronize()


def window(fn, end):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    end()
    return (time.perf_counter() - t0) * 1e6


def med(fn, end, reps):
    ts = sorted(window(fn, end) for _ in range(reps))
    return ts[len(ts) // 2]


x = torch.zeros(1, device="cuda")
n, R = 4096, 20
env = CtrReachVecEnv(n, device="cuda", seed=0, refill_interval=R, integrator="rk4", rk4_steps_per_m=100, model="rigid")
env.reset()
g0 = torch.Generator(device="cpu")
g0.manual_seed(2)
env.t.copy_(torch.randint(0, 150, (n,), generator=g0, dtype=torch.int32))
hi = torch.tensor(env.action_space.high, device="cuda")
acts = [((torch.rand((n, 6), device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
for i in range(25 * R):
    env.step_raw(acts[i % 8])
torch.cuda.synchronize()
graph = env.capture_steps([acts[i % 8] for i in range(R)])
for _ in range(3):
    graph.replay()
for rep in range(3):
    print("empty kernel: block %.1f us, poll %.1f us   configs[1] 20-step graph: block %.1f us, poll %.1f us" %
          (med(lambda: x.add_(1.0), end_block, 200), med(lambda: x.add_(1.0), end_poll, 200),
           med(graph.replay, end_block, 30), med(graph.replay, end_poll, 30)), flush=True)
