"""Diagnostic: what the bench's host-timed window adds to the steps it contains.

bench.py times K steps between two device syncs with the host clock.  This splits such a window
(65 536 envs, one refill period of R = 20 steps + the refill, steady state) into
  - the GPU's own time: HIP events recorded on the stream right before and after the work,
    enqueued behind a short spin kernel so the first event is not stamped before the host has
    submitted the work;
  - the host window as bench.py reads it (sync, clock, launches, sync, clock);
  - the empty round trip: sync, clock, one empty launch, sync, clock;
for the captured HIP graph (bench.py's default) and for eager launches, interleaved.
usage: python tools/window_overhead.py [reps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n, R = 65536, 20
env = CtrReachVecEnv(n, device="cuda", seed=0, refill_interval=R)
env.reset()
g0 = torch.Generator(device="cpu")
g0.manual_seed(2)
env.t.copy_(torch.randint(0, 150, (n,), generator=g0, dtype=torch.int32))
g = torch.Generator(device="cuda")
g.manual_seed(1)
hi = torch.tensor(env.action_space.high, device="cuda")
acts = [((torch.rand((n, 6), generator=g, device="cuda") * 2 - 1) * hi).contiguous() for _ in range(8)]
for i in range(25 * R):
    env.step_raw(acts[i % 8])
torch.cuda.synchronize()
graph = env.capture_steps([acts[i % 8] for i in range(R)])
for _ in range(3):
    graph.replay()
torch.cuda.synchronize()
sink = torch.zeros(1, device="cuda")


def eager():
    for i in range(R):
        env.step_raw(acts[i % 8])


def window(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e6


def gpu_time(fn):
    # a ~200 us busy kernel first, so both events are stamped by the GPU in stream order after
    # the host has enqueued everything
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(400000)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


def empty():
    sink.add_(1.0)


for rep in range(reps):
    row = []
    for name, fn in (("graph", graph.replay), ("eager", eager)):
        w = window(fn)
        gt = gpu_time(fn)
        row.append("%s: host window %.1f us, GPU %.1f us (+%.1f)" % (name, w, gt, w - gt))
    row.append("empty round trip %.1f us" % window(empty))
    print("   ".join(row), flush=True)
