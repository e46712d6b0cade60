"""Diagnostic: does an RCCL-sized gather kernel, issued after every step on its own stream,
slow the steps down on one GPU?  Stand-in for configs[3]'s per-step all-gather (which needs 8
GPUs): tools/fake_gather.hip holds workgroups with RCCL's footprint (256 VGPRs, 37.7 KB LDS)
resident for a fixed time.  The dependency pattern is bench.py's: the gather of step t waits for
step t, and step t+2 waits for the gather of step t (two pack buffers).

Prints us per step for: no gather; the gather overlapping the next step with the env on a
normal-priority stream, and on a high-priority one; the gather serialised between the steps
(step t+1 waits for the gather of step t).  The gather alone is timed
first.
usage: python tools/gather_interference.py [gather_us] [blocks]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv  # noqa: E402

target_us = float(sys.argv[1]) if len(sys.argv) > 1 else 35.0
blocks = int(sys.argv[2]) if len(sys.argv) > 2 else 32
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libfake_gather.so"))
lib.fake_gather_launch.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda", 0)
sink = torch.zeros(1, dtype=torch.int32, device=dev)


def launch(cycles, stream):
    rc = lib.fake_gather_launch(blocks, cycles, sink.data_ptr(), ctypes.c_void_p(stream.cuda_stream))
    assert rc == 0, rc


def time_alone(cycles):
    s = torch.cuda.Stream(device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        for _ in range(5):
            launch(cycles, s)
        e0.record(s)
        for _ in range(20):
            launch(cycles, s)
        e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 20 * 1e3


# calibrate the s_memtime count that keeps the workgroups resident for target_us
c = 100000
us = time_alone(c)
c = max(1, int(c * target_us / max(us, 1e-3)))
us = time_alone(c)
print("fake gather alone: %d workgroups, %.1f us" % (blocks, us), flush=True)

n = 65536
env = CtrReachVecEnv(n, device=dev, seed=0, refill_interval=20)
env.reset()
g = torch.Generator(device="cpu")
g.manual_seed(17)
env.t.copy_(torch.randint(0, 150, (n,), generator=g, dtype=torch.int32))
gd = torch.Generator(device=dev)
gd.manual_seed(1)
hi = torch.tensor(env.action_space.high, device=dev)
acts = [((torch.rand((n, 6), generator=gd, device=dev) * 2 - 1) * hi).contiguous() for _ in range(8)]
torch.cuda.synchronize()


def run(gather, prio, steps=200, warm=200, serial=False):
    comp = torch.cuda.Stream(device=dev, priority=-1 if prio else 0)
    side = torch.cuda.Stream(device=dev, priority=0)
    comp.wait_stream(torch.cuda.current_stream())
    done = [None, None]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(comp):
        for i in range(warm + steps):
            if i == warm:
                e0.record(comp)
            k = i & 1
            if gather and done[k] is not None:
                comp.wait_event(done[k])
            if serial and done[k ^ 1] is not None:
                comp.wait_event(done[k ^ 1])          # the previous step's gather, before this step
            env.step_raw(acts[i % 8])
            if gather:
                ev = torch.cuda.Event()
                ev.record(comp)
                side.wait_event(ev)
                launch(c, side)
                d = torch.cuda.Event()
                d.record(side)
                done[k] = d
        e1.record(comp)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e3


for rep in range(2):
    print("no gather                    %.1f us/step" % run(False, False), flush=True)
    print("gather, env normal priority  %.1f us/step" % run(True, False), flush=True)
    print("gather, env high priority    %.1f us/step" % run(True, True), flush=True)
    print("gather serialised (in order) %.1f us/step" % run(True, False, serial=True), flush=True)
