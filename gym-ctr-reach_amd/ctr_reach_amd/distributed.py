"""Multi-GPU helpers: one process per GPU, environments sharded by global id.

Environments are independent, so the step itself has no exchange: rank r owns the contiguous
global ids [r * n, (r + 1) * n) (``env_base``) and every random draw is keyed by the global id,
which makes results independent of the number of GPUs.  The only collective is OPTIONAL and off
the data path: ``all_gather_outputs`` packs (tip x/y/z, done | success << 1 | (reward = -1) << 2)
into 16 B per env and all-gathers it over RCCL (backend "nccl" on ROCm, xGMI between the GPUs of a node) for a
single-process trainer that wants every shard's outputs.
"""
import os

PACK_WIDTH = 4   # float32 words per env: tip x, y, z, flags (done | success << 1 | (reward = -1) << 2)


def world():
    """(rank, world_size, local_rank) from the torchrun environment (1 process if unset)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(num_envs_per_rank, rank):
    """Global id of this rank's first environment."""
    return int(num_envs_per_rank) * int(rank)


def pack_step_outputs(achieved_goal, reward, done, success, out=None):
    """[n, 4] float32 tensor: tip (3, f64 -> f32), done | success << 1 | (reward = -1) << 2.
    The env's reward is sparse, -1 or 0 (ctr_reach_env.py:160-170), so one bit carries it."""
    import torch
    n = achieved_goal.shape[0]
    if out is None:
        out = torch.empty((n, PACK_WIDTH), dtype=torch.float32, device=achieved_goal.device)
    out[:, 0:3] = achieved_goal
    out[:, 3] = done.to(torch.float32) + 2.0 * success.to(torch.float32) + 4.0 * (reward < 0).to(torch.float32)
    return out


def unpack_step_outputs(packed):
    """(tip [n, 3] f32, reward [n] f32, done [n] bool, success [n] bool) of packed rows."""
    import torch
    flags = packed[:, 3].round().to(torch.int32)
    reward = ((flags >> 2) & 1).to(torch.float32).neg_().add_(0.0)     # -1 or +0 (not -0)
    return packed[:, 0:3], reward, (flags & 1).bool(), (flags & 2).bool()


def all_gather_outputs(packed, group=None, async_op=False):
    """All-gather every rank's packed [n, 4] block into [world * n, 4] (rank-major = global id
    order).  Uses all_gather_into_tensor: one RCCL ring/tree call for the whole step.

    async_op=True returns (out, work): the collective runs on RCCL's own stream, ordered after
    the packing on the current stream, so the next ctr_step overlaps it; ``work.wait()`` before
    reading ``out``, and keep ``packed`` unchanged until then."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    if packed.is_cuda and dist.get_backend(group) == "gloo":
        # gloo rehearsal of the RCCL path (several ranks on one GPU): gather host copies
        host = packed.cpu()
        out = torch.empty((ws * packed.shape[0], packed.shape[1]), dtype=packed.dtype)
        dist.all_gather_into_tensor(out, host, group=group)
        out = out.to(packed.device)
        return (out, _DoneWork()) if async_op else out
    out = torch.empty((ws * packed.shape[0], packed.shape[1]), dtype=packed.dtype, device=packed.device)
    work = dist.all_gather_into_tensor(out, packed.contiguous(), group=group, async_op=async_op)
    return (out, work) if async_op else out


class _DoneWork(object):
    """A completed collective (the synchronous gloo rehearsal path)."""

    def wait(self):
        return True

    def is_completed(self):
        return True


def max_over_ranks(value, device=None, group=None):
    """Max of a python float over ranks (bench timing); identity without a process group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


# ---------------------------------------------------------------------------------------------
# Push all-gather (configs[3] without RCCL's CU-holding kernels)
#
# RCCL's all-gather runs as kernels whose workgroups (248-256 VGPRs per lane) cannot share a SIMD
# with a k_step wave, so the gather of step t holds CUs that step t + 1 needs (DESIGN.md section
# 6).  PushGather moves the same bytes without them: every rank maps every rank's receive ring once
# (IPC handles exchanged over the process group), and each step's rows go into slot `seq % depth`
# of every ring, followed by the step's sequence word.  Engines:
#   "fused"  k_step itself stores each env's row into every rank's slot (ctr_step_out_t.gather:
#            8 extra 16-B stores per lane at the end of the step, then a system-scope release
#            fence per wave), and the NEXT k_step launch publishes the sequence words (its
#            predecessor has completed, so the rows are performed at system scope); a consumer
#            that waits before the next step publishes them itself (ctr_gather_publish).  No
#            extra launch, no cross-stream dependency per step.
#   "sdma"   ctr_copy_list after the step: copy-engine copies (no CU at all) of the packed rows;
#            measured host-synchronous per copy in this runtime (~25 us each), so it cannot keep
#            up with a step; kept selectable
# (A standalone push kernel on a side stream, ctr_gather_push, overlaps the step but each step
# then waits on a cross-stream event: ~10 us per hop, measured)
# Layout of a rank's shared memory: the receive ring [depth][world][n][4] float32 (a slot is the
# rank-major = global-id-ordered [world * n, 4] gather), and a control block of sequence words
# [depth][world] uint32 (word [slot][r] = the last step rank r published into that slot), release
# words [world] uint32 (word [c] = the last step whose slot consumer c released, written by c) and
# the push kernel's ticket.  Both are uncached device memory: other GPUs write them, so this
# GPU's L2 must not serve stale lines.
#
# Reuse rule (flow control, fused engine): slot s % depth is rewritten by step s + depth.  A rank
# releases its slot of step s when it launches step s + depth - 1 (the launch's first lanes write
# the release words of every producer), so a gathered view of step s is valid until this rank
# launches step s + depth - 1; k_step(t) stores its rows only once every rank has released step
# t - depth.  With wait_prev (depth >= 3) k_step(t) also waits until every rank's rows of step
# t - 1 are in this rank's ring, so that slot is readable after the launch (the consumer wait
# fused into the step).  The sdma engine and ctr_gather_push leave the pacing to the caller
# (ctr_gather_wait flags a slot overwritten before it was consumed).

class HipCopyOps(object):
    """The device side of PushGather: libctr_reach_amd.so's IPC, uncached memory, descriptor,
    publish, copy-list and wait entry points (include/ctr_reach_amd.h)."""

    def __init__(self, device):
        from . import _abi
        self._abi = _abi
        self.lib = _abi.load()
        self.device = device
        self._arrays = {}

    def alloc_shared(self, nbytes):
        import ctypes
        p = ctypes.c_void_p()
        self._abi.check(self.lib.ctr_seqw_alloc(int(nbytes), ctypes.byref(p)), "ctr_seqw_alloc")
        return p.value

    def free_shared(self, ptr):
        self.lib.ctr_seqw_free(ptr)

    def handle(self, ptr):
        import ctypes
        buf = ctypes.create_string_buffer(self._abi.CTR_IPC_HANDLE_BYTES)
        self._abi.check(self.lib.ctr_ipc_get_handle(ptr, buf), "ctr_ipc_get_handle")
        return buf.raw

    def open(self, handle):
        import ctypes
        p = ctypes.c_void_p()
        self._abi.check(self.lib.ctr_ipc_open(handle, ctypes.byref(p)), "ctr_ipc_open")
        return p.value

    def close(self, ptr):
        self.lib.ctr_ipc_close(ptr)

    def make_streams(self, k):
        import torch
        return [torch.cuda.Stream(device=self.device) for _ in range(k)]

    def make_event(self):
        import torch
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))      # created now, not lazily
        return ev

    def upload_descriptors(self, targets, n, ticket_ptr, flow):
        """Per-slot ctr_gather_push_t descriptors in device memory (the fused push reads them):
        targets[slot] = [(row block dst, sequence word), ...] per rank; flow = the flow-control
        fields (relw: this rank's release word in every rank, rel, wait_seqw per slot, err, depth,
        wait_us, poisonw: this rank's poison word in every rank, poison).  Returns (keep-alive,
        device pointer per slot)."""
        import ctypes
        import torch
        size = ctypes.sizeof(self._abi.CtrGatherPush)
        raw = bytearray()
        for slot, tg in enumerate(targets):
            g = self._abi.CtrGatherPush()
            g.n, g.world, g.ticket = n, len(tg), ticket_ptr
            for k, (dst, sw) in enumerate(tg):
                g.dst[k], g.seqw[k] = dst, sw
            for k, rw in enumerate(flow["relw"]):
                g.relw[k] = rw
            g.rel, g.wait_seqw, g.err = flow["rel"], flow["wait_seqw"][slot], flow["err"]
            g.depth, g.wait_us = flow["depth"], flow["wait_us"]
            for k, pw in enumerate(flow["poisonw"]):
                g.poisonw[k] = pw
            g.poison = flow["poison"]
            raw += bytes(g)
        dev = torch.frombuffer(raw, dtype=torch.uint8).to(self.device)
        return dev, [dev.data_ptr() + i * size for i in range(len(targets))]

    def publish(self, desc_ptr, seq, stream):
        self._abi.check(self.lib.ctr_gather_publish(desc_ptr, seq & 0xFFFFFFFF, stream.cuda_stream),
                        "ctr_gather_publish")

    def native_plan(self, copies):
        arr = (self._abi.CtrCopy * max(1, len(copies)))()
        for i, (dst, src, nbytes, s) in enumerate(copies):
            arr[i].dst, arr[i].src, arr[i].bytes, arr[i].stream = dst, src, nbytes, s
        return arr, len(copies)

    def copy_list(self, plan, streams, ready_event, done_events):
        import ctypes
        arr, n = plan["native"]
        key = (id(streams), id(done_events))
        if key not in self._arrays:      # the streams and per-parity event lists live as long as the gather
            self._arrays[key] = ((ctypes.c_void_p * len(streams))(*[s.cuda_stream for s in streams]),
                                 (ctypes.c_void_p * len(done_events))(*[e.cuda_event for e in done_events]))
        sp, dp = self._arrays[key]
        rc = self.lib.ctr_copy_list(arr, n, sp, len(streams), ready_event.cuda_event if ready_event else None, dp)
        self._abi.check(rc, "ctr_copy_list")

    def wait(self, seqw_ptr, n, seq, wait_us, err, stream):
        rc = self.lib.ctr_gather_wait(seqw_ptr, n, seq & 0xFFFFFFFF, wait_us, err.data_ptr(), stream.cuda_stream)
        self._abi.check(rc, "ctr_gather_wait")

    def view(self, ptr, shape, dtype):
        """A torch tensor over device memory this object allocated (CUDA array interface)."""
        import torch
        typestr = {torch.float32: "<f4", torch.int32: "<i4"}[dtype]

        class _Iface(object):
            __cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(ptr), False),
                                        "version": 2, "strides": None, "stream": None}
        t = torch.as_tensor(_Iface(), device=self.device)
        assert t.data_ptr() == ptr and tuple(t.shape) == tuple(shape) and t.dtype == dtype
        return t


class PushWork(object):
    """Handle of one push gather (the async_op result of gather_outputs(backend="push"/"sdma"))."""

    def __init__(self, gather, seq):
        self.gather, self.seq = gather, seq

    def wait(self, stream=None):
        """Enqueue the wait for every rank's block of this step on `stream` (default: current);
        returns the gathered rows."""
        import torch
        return self.gather.wait(self.seq, stream if stream is not None else torch.cuda.current_stream())

    def is_completed(self):
        return False


class PushGather(object):
    """All-gather of every rank's packed step rows ([n, 4] float32: tip, done | success << 1 |
    (reward = -1) << 2) by pushes into IPC-mapped receive rings (see the section comment).

    fused engine (the env drives it around each ctr_step):
      step_args(seq)           (descriptor of seq's slot, descriptor to publish, its seq) for
                               ctr_step_out_t.gather / gather_prev / gather_prev_seq
      stepped(seq)             the step launch with seq was enqueued (its words are pending)
      wait_prev                ctr_step_out_t.gather_wait_prev for every step (depth >= 3)
    sdma engine:
      push(packed, seq, ready_event, parity)   copy-engine copies of packed ([n + 1, 4]: row n is
                               the sequence row k_step writes with ctr_step_out_t.packed_seq)
      wait_pushed(parity, stream)  before a step rewrites pack buffer `parity`
    both:
      wait(seq, stream)        enqueue the consumer wait for step seq (publishing it first if no
                               later step did) and return the gathered [world * n, 4] rows
    Step numbers are Python ints from 1 (slot = seq % depth); the device sees them modulo 2^32.
    ``ops`` is the device backend (HipCopyOps; tests pass a CPU stand-in)."""

    def __init__(self, n, group=None, depth=3, engine="fused", n_streams=None, device=None, ops=None,
                 wait_us=10_000_000, wait_prev=False):
        import torch
        import torch.distributed as dist
        if engine not in ("fused", "sdma"):
            raise ValueError("engine must be 'fused' or 'sdma'")
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.n, self.depth, self.engine = int(n), int(depth), engine
        if self.depth < 2:
            raise ValueError("depth must be >= 2 (a slot is rewritten depth steps later)")
        if wait_prev and self.depth < 3:
            raise ValueError("wait_prev needs depth >= 3 (the view of step t - 1 is read after step t)")
        if self.world > 16:
            raise ValueError("at most 16 ranks (CTR_GATHER_MAX_RANKS)")
        self.wait_prev = bool(wait_prev)
        self.ops = ops if ops is not None else HipCopyOps(device)
        if not 0 < int(wait_us) < 1 << 32:
            raise ValueError("wait_us must fit a uint32 (microseconds)")
        self.wait_us = int(wait_us)
        W, n4 = self.world, self.n * PACK_WIDTH * 4
        self.block_bytes = n4
        self.rel_off = self.depth * W * 4                 # release words, then the push ticket
        ticket_off = self.rel_off + W * 4
        self.poison_off = ticket_off + 64                 # poison words, after the ticket
        # every rank takes part in both exchanges even after a local failure, and all raise
        # together: a rank that gave up alone would leave the others blocked in a collective
        mine, err = None, None
        try:
            self.recv_ptr = self.ops.alloc_shared(self.depth * W * n4)
            self.seqw_ptr = self.ops.alloc_shared(self.poison_off + W * 4)
            mine = (self.ops.handle(self.recv_ptr), self.ops.handle(self.seqw_ptr))
        except Exception as ex:            # noqa: BLE001 -- re-raised below, on every rank
            err = "rank %d: %s" % (self.rank, ex)
        allh = [None] * W
        dist.all_gather_object(allh, (mine, err), group=group)
        errs = [e for _, e in allh if e]
        if errs:
            raise RuntimeError("PushGather setup failed: " + "; ".join(errs))
        self.ticket_ptr = self.seqw_ptr + ticket_off
        self.peer_recv, self.peer_seqw = [None] * W, [None] * W
        try:
            for p in range(W):
                self.peer_recv[p] = self.recv_ptr if p == self.rank else self.ops.open(allh[p][0][0])
                self.peer_seqw[p] = self.seqw_ptr if p == self.rank else self.ops.open(allh[p][0][1])
        except Exception as ex:            # noqa: BLE001
            err = "rank %d: %s" % (self.rank, ex)
        oks = [None] * W
        dist.all_gather_object(oks, err, group=group)
        errs = [e for e in oks if e]
        if errs:
            raise RuntimeError("PushGather peer mapping failed: " + "; ".join(errs))
        self.recv = self.ops.view(self.recv_ptr, (self.depth, W, self.n, PACK_WIDTH), torch.float32)
        self.seqw = self.ops.view(self.seqw_ptr, (self.depth, W), torch.int32)
        self.rel = self.ops.view(self.seqw_ptr + self.rel_off, (W,), torch.int32)
        self.poison = self.ops.view(self.seqw_ptr + self.poison_off, (W,), torch.int32)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.pending = 0          # fused: the last pushed step whose words are not yet published
        if engine == "fused":
            flow = {"relw": [self.peer_seqw[p] + self.rel_off + 4 * self.rank for p in range(W)],
                    "rel": self.seqw_ptr + self.rel_off,
                    "wait_seqw": [self.seqw_ptr + ((s - 1) % self.depth) * W * 4 for s in range(self.depth)],
                    "err": self.err.data_ptr(), "depth": self.depth, "wait_us": self.wait_us,
                    "poisonw": [self.peer_seqw[p] + self.poison_off + 4 * self.rank for p in range(W)],
                    "poison": self.seqw_ptr + self.poison_off}
            self._desc_keep, self.desc = self.ops.upload_descriptors(
                [self.targets(s) for s in range(self.depth)], self.n, self.ticket_ptr, flow)
            self.n_streams = 0
        else:
            # the copies to peer (rank + 1 + i) % world go on stream i % n_streams (different engines)
            self.n_streams = max(1, min(int(n_streams or W), W))
            self.streams = self.ops.make_streams(self.n_streams)
            self.done = [[self.ops.make_event() for _ in range(self.n_streams)] for _ in range(2)]
            self._plans = {}

    def targets(self, slot):
        """(row block destination, sequence word) in every rank for this rank's block of `slot`:
        rank-major offsets, starting at the next rank (so the ranks write to different peers at a
        time) and ending with this rank's own ring."""
        W, r = self.world, self.rank
        off = (slot * W + r) * self.block_bytes
        woff = (slot * W + r) * 4
        return [(self.peer_recv[(r + 1 + i) % W] + off, self.peer_seqw[(r + 1 + i) % W] + woff) for i in range(W)]

    # ---- fused engine
    def step_args(self, seq):
        prev = self.pending
        return self.desc[seq % self.depth], (self.desc[prev % self.depth] if prev else None), prev

    def stepped(self, seq):
        self.pending = seq

    # ---- sdma engine
    def plan(self, src_ptr, slot):
        key = (src_ptr, slot)
        if key not in self._plans:
            copies = []
            for i, (dst, sw) in enumerate(self.targets(slot)):
                s = i % self.n_streams
                copies.append((dst, src_ptr, self.block_bytes, s))
                copies.append((sw, src_ptr + self.block_bytes, 4, s))
            self._plans[key] = {"copies": copies, "native": self.ops.native_plan(copies)}
        return self._plans[key]

    def push(self, packed, seq, ready_event, parity=None):
        """packed: [n + 1, 4] float32 whose row n holds seq (k_step with packed_seq = seq)."""
        if self.engine != "sdma":
            raise RuntimeError("push() is the sdma engine's; the fused push runs inside the step")
        if packed.shape[0] != self.n + 1:
            raise ValueError("packed must hold n + 1 rows (the sequence row)")
        parity = (seq & 1) if parity is None else parity
        self.ops.copy_list(self.plan(packed.data_ptr(), seq % self.depth), self.streams, ready_event,
                           self.done[parity])

    def wait_pushed(self, parity, stream):
        if self.engine == "sdma":
            for ev in self.done[parity & 1]:
                stream.wait_event(ev)

    # ---- consumer
    def wait(self, seq, stream):
        slot = seq % self.depth
        if self.engine == "fused" and self.pending == seq:
            self.ops.publish(self.desc[slot], seq, stream)     # no later step has published it
            self.pending = 0
        self.ops.wait(self.seqw_ptr + slot * self.world * 4, self.world, seq, self.wait_us, self.err, stream)
        return self.slot_view(seq)

    def err_bits(self):
        """This rank's CTR_GATHER_E_* bits, with a producer's overrun of a slot this rank had not
        released (its poison word, fused engine) as CTR_GATHER_E_RELEASE_TIMEOUT.  Synchronises.
        Read after a view's readers have run, it covers every overwrite that reached that view
        (the producer's poison store is performed before its first row store)."""
        import torch
        if torch.is_tensor(self.err) and self.err.is_cuda:
            torch.cuda.synchronize(self.err.device)
        e = int(self.err.reshape(-1)[0].item()) & 0xFFFFFFFF
        if self.engine == "fused" and bool((self.poison != 0).any()):
            e |= 4                                           # CTR_GATHER_E_RELEASE_TIMEOUT
        return e

    def flush(self, stream):
        """Publish the last pushed step's sequence words now (fused engine: a step's words are
        otherwise published by the next step's launch) -- for a rank that stops stepping while
        others still wait for its last step."""
        if self.engine == "fused" and self.pending:
            self.ops.publish(self.desc[self.pending % self.depth], self.pending, stream)
            self.pending = 0

    def slot_view(self, seq):
        """The gathered [world * n, 4] rows of step seq's slot (valid once its wait has run)."""
        return self.recv[seq % self.depth].reshape(self.world * self.n, PACK_WIDTH)

    def close(self):
        for p in range(self.world):
            if p != self.rank:
                self.ops.close(self.peer_recv[p])
                self.ops.close(self.peer_seqw[p])
        self.ops.free_shared(self.recv_ptr)
        self.ops.free_shared(self.seqw_ptr)


def verify_gathered(out, mine, err, group=None):
    """Bit-compare a gathered slot `out` ([world * n, 4]) with a process-group all_gather of every
    rank's own rows `mine` ([n, 4]) -- the reference copy -- and agree on the verdict over every
    rank (MAX all_reduce).  Returns (ok on every rank, report).  Used by bench.py's untimed check of
    the push gather before any window runs with it."""
    import torch
    import torch.distributed as dist
    ws = dist.get_world_size(group)
    gloo = dist.get_backend(group) == "gloo"
    src = mine.cpu() if gloo else mine
    blocks = [torch.empty_like(src) for _ in range(ws)]
    dist.all_gather(blocks, src, group=group)
    ref = torch.cat(blocks)
    got = out.cpu() if gloo else out
    bad_rows = int((got != ref).any(dim=1).sum().item())
    # err: the error word, or a callable returning the bits (PushGather.err_bits), read after the rows
    e = err() if callable(err) else (int(err.item()) if hasattr(err, "item") else int(err))
    flags = torch.tensor([1 if bad_rows else 0, e, bad_rows], dtype=torch.int64,
                         device="cpu" if gloo else out.device)
    dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)
    ok = int(flags[0]) == 0 and int(flags[1]) == 0
    return ok, {"rows_equal_all_ranks": int(flags[0]) == 0, "err_bits_max": int(flags[1]),
                "mismatched_rows_max": int(flags[2])}


def check_push_steps(step, gather, mine, steps, stream=None, group=None):
    """bench.py's check of the fused push before any timing: `steps` times, run step(i) (one env
    step that pushes), wait for its slot and verify_gathered it against the process-group copy of
    mine() (this rank's own rows of that step).  Stops at the first failure.  Returns the report
    (``passed``, ``steps_checked``, and on a failure ``failed_at_step`` with verify_gathered's
    fields); every rank gets the same verdict."""
    rep = {"steps_checked": 0}
    for i in range(steps):
        seq = step(i)
        ok, r = verify_gathered(gather.wait(seq, stream), mine(), gather.err_bits, group=group)
        rep["steps_checked"] += 1
        if not ok:
            rep.update(r, failed_at_step=i)
            break
    rep["passed"] = "failed_at_step" not in rep
    return rep
