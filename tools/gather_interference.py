"""Diagnostic: what does a per-step gather cost the step on one GPU?  Stand-in for configs[3]'s
all-gather (which needs 8 GPUs), with bench.py's dependency pattern: the gather of step t waits
for step t, and step t + 2 waits for the gather of step t (two pack buffers).

Gathers:
  fused  the fused push (bench.py's default): k_step itself stores every env's row into `peers`
         destination blocks (uncached memory, as the receive rings) and the next launch
         publishes the sequence words -- distributed.PushGather's "fused" engine with local
         destinations in place of the peers' IPC-mapped rings
  push   the standalone push kernel (ctr_gather_push) after every step: the
         step's packed block stored into `peers` destination blocks (uncached memory, as the
         receive rings) + the sequence words, `workgroups` workgroups, on a side stream
  sdma   the copy-engine backend's traffic on one device: after every step, the step's packed
         block (n x 16 B) is copied into `peers` destination blocks of a receive ring, plus a
         4-B sequence word after each, with hipMemcpyDeviceToDeviceNoCU (ctr_copy_list) spread
         over `streams` copy streams -- the same copy list CopyEngineGather runs, with the
         peers' rings replaced by local buffers (no xGMI here)
  fake   tools/fake_gather.hip: workgroups with RCCL's footprint (256 VGPRs, 37.7 KB LDS)
         resident for a set time (round 2's measurement)

Prints us per step with no gather, and with the gather overlapping the next step.  Also the
host time per ctr_copy_list call and the copies' own duration.
usage: python tools/gather_interference.py fused [peers] [wait]
       python tools/gather_interference.py push [peers] [workgroups]
       python tools/gather_interference.py sdma [peers] [streams]
       python tools/gather_interference.py fake [gather_us] [blocks]"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
from ctr_reach_amd import CtrReachVecEnv, _abi  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "sdma"
dev = torch.device("cuda", 0)
n = 65536
env = CtrReachVecEnv(n, device=dev, seed=0, refill_interval=20, pack_outputs=True)
env.reset()
g = torch.Generator(device="cpu")
g.manual_seed(17)
env.t.copy_(torch.randint(0, 150, (n,), generator=g, dtype=torch.int32))
gd = torch.Generator(device=dev)
gd.manual_seed(1)
hi = torch.tensor(env.action_space.high, device=dev)
acts = [((torch.rand((n, 6), generator=gd, device=dev) * 2 - 1) * hi).contiguous() for _ in range(8)]
lib = env.lib
torch.cuda.synchronize()

if mode == "fused":
    from ctr_reach_amd.distributed import HipCopyOps
    peers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    wait_prev = len(sys.argv) > 3 and sys.argv[3] == "wait"
    D = 3
    block = n * 16
    ops = HipCopyOps(dev)
    ring = ops.alloc_shared(D * peers * block + 4096)
    seqw = ring + D * peers * block                # [D][peers] words, then [peers] release words
    relw = seqw + 4 * D * peers
    gerr = torch.zeros(1, dtype=torch.int32, device=dev)

    class LocalFused(object):
        """PushGather's fused engine (depth 3) with `peers` local destination blocks per slot and
        the flow control's release words local too (this rank releases for every 'peer')."""
        engine = "fused"
        depth = D

        def __init__(self):
            flow = {"relw": [relw + 4 * i for i in range(peers)], "rel": relw,
                    "wait_seqw": [seqw + 4 * peers * ((s - 1) % D) for s in range(D)],
                    "err": gerr.data_ptr(), "depth": D, "wait_us": 10_000_000,
                    "poisonw": [seqw + 3072 + 4 * i for i in range(peers)], "poison": seqw + 3072}
            self.keep, self.desc = ops.upload_descriptors(
                [[(ring + (s * peers + i) * block, seqw + 4 * (s * peers + i)) for i in range(peers)] for s in range(D)],
                n, seqw + 2048, flow)
            self.pending = 0
            self.wait_prev = wait_prev

        def step_args(self, seq):
            prev = self.pending
            return self.desc[seq % D], (self.desc[prev % D] if prev else None), prev

        def stepped(self, seq):
            self.pending = seq

        def wait_pushed(self, parity, stream):
            pass

    fused = LocalFused()
    host_us = []

    def gather_after_step(comp):
        pass

    def wait_before_step(comp):
        pass
    label = "fused push into %d blocks%s" % (peers, " + fused wait" if wait_prev else "")
elif mode == "push":
    peers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    wg = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    block = n * 16
    ring_p = ctypes.c_void_p()
    _abi.check(lib.ctr_seqw_alloc(2 * peers * block + 4096, ctypes.byref(ring_p)), "alloc")
    ring = ring_p.value
    seqw, ticket = ring + 2 * peers * block, ring + 2 * peers * block + 2048
    side = torch.cuda.Stream(device=dev, priority=int(os.environ.get("SIDE_PRIO", "0")))
    done = [torch.cuda.Event(), torch.cuda.Event()]
    for e in done:
        e.record(side)
    structs = []
    for k in range(2):
        gp = _abi.CtrGatherPush()
        gp.src, gp.n, gp.world, gp.ticket = env.packed_bufs[k].data_ptr(), n, peers, ticket
        for i in range(peers):
            gp.dst[i], gp.seqw[i] = ring + (k * peers + i) * block, seqw + 4 * (k * peers + i)
        structs.append(gp)
    ready = torch.cuda.Event()
    host_us = []
    seqc = [0]

    def gather_after_step(comp):
        k = env._packed_k
        ready.record(comp)
        side.wait_event(ready)
        seqc[0] += 1
        t0 = time.perf_counter()
        _abi.check(lib.ctr_gather_push(structs[k], seqc[0], wg, side.cuda_stream), "ctr_gather_push")
        host_us.append((time.perf_counter() - t0) * 1e6)
        done[k].record(side)

    def wait_before_step(comp):
        comp.wait_event(done[env._packed_k ^ 1])

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(3):
        torch.cuda.synchronize()
        e0.record(side)
        for _ in range(20):
            seqc[0] += 1
            _abi.check(lib.ctr_gather_push(structs[1], seqc[0], wg, side.cuda_stream), "ctr_gather_push")
        e1.record(side)
        torch.cuda.synchronize()
        print("push kernel alone: %d x %d KB, %d workgroups: %.1f us" % (peers, block // 1024, wg,
                                                                         e0.elapsed_time(e1) * 1e3 / 20), flush=True)
    label = "push %d peers / %d workgroups" % (peers, wg)
elif mode == "sdma":
    peers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    S = int(sys.argv[3]) if len(sys.argv) > 3 else peers
    block = n * 16
    ring = torch.zeros((2, peers, n + 1, 4), dtype=torch.float32, device=dev)     # destination blocks
    seqw = torch.zeros((2, peers, 4), dtype=torch.int32, device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]
    sp = (ctypes.c_void_p * S)(*[s.cuda_stream for s in streams])
    done = [[torch.cuda.Event() for _ in range(S)] for _ in range(2)]
    for evs in done:
        for e in evs:
            e.record(streams[0])
    dps = [(ctypes.c_void_p * S)(*[e.cuda_event for e in evs]) for evs in done]
    plans = {}

    def plan(k):
        if k not in plans:
            src = env.packed_bufs[k].data_ptr()
            arr = (_abi.CtrCopy * (2 * peers))()
            for i in range(peers):
                arr[2 * i].dst, arr[2 * i].src, arr[2 * i].bytes, arr[2 * i].stream = ring[k, i].data_ptr(), src, block, i % S
                arr[2 * i + 1].dst, arr[2 * i + 1].src, arr[2 * i + 1].bytes = seqw[k, i].data_ptr(), src + block, 4
                arr[2 * i + 1].stream = i % S
            plans[k] = arr
        return plans[k]

    ready = torch.cuda.Event()
    host_us = []

    def gather_after_step(comp):
        k = env._packed_k
        ready.record(comp)
        t0 = time.perf_counter()
        rc = lib.ctr_copy_list(plan(k), 2 * peers, sp, S, ready.cuda_event, dps[k])
        host_us.append((time.perf_counter() - t0) * 1e6)
        _abi.check(rc, "ctr_copy_list")

    def wait_before_step(comp):
        for e in done[env._packed_k ^ 1]:
            comp.wait_event(e)

    # the copies alone: one step's list, timed on the copy streams
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(3):
        torch.cuda.synchronize()
        e0.record(streams[0])
        for s in streams[1:]:
            s.wait_event(e0)
        rc = lib.ctr_copy_list(plan(1), 2 * peers, sp, S, None, dps[1])
        for e in done[1]:
            streams[0].wait_event(e)
        e1.record(streams[0])
        torch.cuda.synchronize()
        print("copies alone: %d x %d KB + seq words on %d streams: %.1f us" % (peers, block // 1024, S,
                                                                                e0.elapsed_time(e1) * 1e3), flush=True)
    label = "sdma %d peers / %d streams" % (peers, S)
else:
    assert mode == "fake", mode
    target_us = float(sys.argv[2]) if len(sys.argv) > 2 else 35.0
    blocks = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    fl = ctypes.CDLL(os.path.join(ROOT, "tools", "libfake_gather.so"))
    fl.fake_gather_launch.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    side = torch.cuda.Stream(device=dev, priority=0)
    fdone = [None, None]

    def launch(cycles, stream):
        assert fl.fake_gather_launch(blocks, cycles, sink.data_ptr(), ctypes.c_void_p(stream.cuda_stream)) == 0

    def time_alone(cycles):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            launch(cycles, side)
        e0.record(side)
        for _ in range(20):
            launch(cycles, side)
        e1.record(side)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 20 * 1e3

    c = 100000
    c = max(1, int(c * target_us / max(time_alone(c), 1e-3)))
    print("fake gather alone: %d workgroups, %.1f us" % (blocks, time_alone(c)), flush=True)
    host_us = []

    def gather_after_step(comp):
        ev = torch.cuda.Event()
        ev.record(comp)
        side.wait_event(ev)
        launch(c, side)
        d = torch.cuda.Event()
        d.record(side)
        fdone[env._packed_k] = d

    def wait_before_step(comp):
        d = fdone[env._packed_k ^ 1]
        if d is not None:
            comp.wait_event(d)
    label = "fake RCCL-footprint gather"


def run(gather, prio=False, steps=200, warm=200):
    if mode == "fused":
        env._push_gather = fused if gather else None
    comp = torch.cuda.Stream(device=dev, priority=-1 if prio else 0)
    comp.wait_stream(torch.cuda.current_stream())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(comp):
        for i in range(warm + steps):
            if i == warm:
                e0.record(comp)
            if gather:
                wait_before_step(comp)
            env.step_raw(acts[i % 8], comp)
            if gather:
                gather_after_step(comp)
        e1.record(comp)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps * 1e3


for rep in range(3):
    a = run(False)
    b = run(True)
    line = "no gather %.1f us/step   %s overlapped %.1f us/step   (+%.1f)" % (a, label, b, b - a)
    c2 = run(True, prio=True)
    line += "   env high priority %.1f" % c2
    if host_us:
        hs = sorted(host_us[-200:])
        line += "   host per gather call: median %.1f us" % hs[len(hs) // 2]
    if mode == "fused":
        line += "   err %d" % int(gerr.item())
    print(line, flush=True)
