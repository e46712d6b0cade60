"""The push all-gather of packed step rows (CtrReachVecEnv.gather_outputs(backend="push" | "sdma"),
distributed.PushGather: the slim push kernel and the copy-engine copies) on the GPU: one rank,
and two processes on the same GPU that map each other's receive rings through IPC handles (the
8-GPU path minus xGMI).

Bars: the gathered rows equal every rank's own packed rows bit for bit (rank-major = global id
order), the sequence words equal the step numbers, and the consumer wait reports no error."""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _acts(env, rng):
    import torch
    return torch.tensor((rng.uniform(-1, 1, (env.num_envs, 6)) * env.action_space.high).astype(np.float32),
                        device=env.device)


@pytest.mark.parametrize("backend", ["push", "sdma"])
def test_gather_outputs_push_one_rank(cuda, backend):
    import torch
    import torch.distributed as dist
    from ctr_reach_amd import CtrReachVecEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        n = 4096
        env = CtrReachVecEnv(n, device=cuda, seed=9, pack_outputs=True, max_steps_per_episode=2)
        env.reset()
        env.enable_gather(backend)
        rng = np.random.default_rng(3)
        for i in range(5):
            env.step(_acts(env, rng))
            want = env.packed_outputs().clone()
            seq = env.packed_seq
            out, work = env.gather_outputs(backend=backend, async_op=True)
            env.step(_acts(env, rng))          # writes the other pack buffer while the push runs
            work.wait()
            torch.cuda.synchronize()
            assert torch.equal(out, want), i
            g = env._push_gather
            assert int(g.err.item()) == 0
            assert int(g.seqw[seq % g.depth, 0].item()) == seq
        # fused: a wait after later steps finds the words published by those steps' launches
        if backend == "push":
            env.step(_acts(env, rng))
            seq = env.gather_seq
            want = env.packed_outputs().clone()
            for _ in range(1):
                env.step(_acts(env, rng))      # publishes seq; its rows stay in the other slot
            out = g.wait(seq, torch.cuda.current_stream())
            torch.cuda.synchronize()
            assert torch.equal(out, want) and int(g.err.item()) == 0
        # the synchronous form
        full = env.gather_outputs(backend=backend)
        torch.cuda.synchronize()
        assert torch.equal(full, env.packed_outputs())
        env._push_gather.close()
    finally:
        dist.destroy_process_group()


def _two_rank_worker(rank, world, port, n, backend, q):
    sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ctr_reach_amd import CtrReachVecEnv
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        env = CtrReachVecEnv(n, device=dev, seed=5, env_base=rank * n, pack_outputs=True, max_steps_per_episode=3)
        env.reset()
        env.enable_gather(backend)
        rng = np.random.default_rng(10 + rank)
        errs = []
        for i in range(6):
            env.step(_acts(env, rng))
            mine = env.packed_outputs().cpu()
            blocks = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(blocks, mine)                  # the reference: every rank's rows over gloo
            out, work = env.gather_outputs(backend=backend, async_op=True)
            env.step(_acts(env, rng))
            work.wait()
            torch.cuda.synchronize()
            got = out.cpu()
            errs.append((i, bool(torch.equal(got, torch.cat(blocks))), int(env._push_gather.err.item())))
            dist.barrier()                                 # nobody pushes into a slot before it was read
        if rank == 0:
            q.put(errs)
        dist.barrier()
        env._push_gather.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("backend,world", [("push", 2), ("push", 8), ("sdma", 2)])
def test_push_gather_two_processes_one_gpu(cuda, backend, world):
    """`world` ranks on cuda:0, each mapping every other rank's receive ring, sequence words and
    release words (IPC): the 8-peer ring layout and handle exchange of configs[3] minus xGMI."""
    import torch.multiprocessing as mp
    n = 2048
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_rank_worker, args=(r, world, port, n, backend, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        errs = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    for i, equal, err in errs:
        assert equal and err == 0, (i, equal, err)


def _free_worker(rank, world, port, n, steps, q):
    sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import time
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ctr_reach_amd import CtrReachVecEnv
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        env = CtrReachVecEnv(n, device=dev, seed=5, env_base=rank * n, pack_outputs=True, max_steps_per_episode=3)
        env.reset()
        g = env.enable_gather("push", depth=3, wait_prev=True)
        rng = np.random.default_rng(20 + rank)
        own, views = [], []
        for i in range(steps):
            if rank == world - 1:
                time.sleep(0.01)               # one slow rank; no barrier anywhere in the loop
            env.step(_acts(env, rng))
            own.append(env.packed_outputs().clone())
            if i >= 1:
                # k_step(seq)'s fused wait completed every rank's rows of seq - 1 in this ring; the
                # view stays valid until this rank launches seq + 1 (depth 3): copy it now
                views.append(g.slot_view(env.gather_seq - 1).clone())
        g.flush(torch.cuda.current_stream())
        torch.cuda.synchronize()
        res = []
        for s in range(steps - 1):
            blocks = [torch.empty_like(own[s].cpu()) for _ in range(world)]
            dist.all_gather(blocks, own[s].cpu())
            res.append(bool(torch.equal(views[s].cpu(), torch.cat(blocks))))
        if rank == 0:
            q.put((res, int(g.err.item())))
        dist.barrier()
        g.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_push_gather_free_running_ranks_one_gpu(cuda, world):
    """The fused push as bench.py runs it (depth 3, the fused consumer wait, slot releases) with
    ranks on cuda:0 that never synchronise in the step loop, one of them slow: after every step
    the previous step's slot holds every rank's rows bit for bit, and no wait or release times
    out."""
    import torch.multiprocessing as mp
    n, steps = 2048, 10
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_free_worker, args=(r, world, port, n, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res, err = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    assert err == 0 and all(res), (res, err)


def _stalled_worker(rank, world, port, n, q):
    sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ctr_reach_amd import CtrReachVecEnv
        from ctr_reach_amd import _abi
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        env = CtrReachVecEnv(n, device=dev, seed=5, env_base=rank * n, pack_outputs=True)
        env.reset()
        g = env.enable_gather("push", depth=3, wait_us=2000)
        errs = []
        if rank == 0:
            # rank 1 never steps: it never releases a slot, so from step depth + 1 on this rank's
            # k_step waits for the release, gives up after wait_us (2 ms), and flags it
            rng = np.random.default_rng(4)
            for _ in range(5):
                env.step(_acts(env, rng))
                torch.cuda.synchronize()
                errs.append(int(g.err.item()))
            q.put((0, errs))
        dist.barrier()
        if rank == 1:
            # the overrun consumer learns it from its own error bits (the producer's poison
            # stores into its memory), without any cross-rank reduction
            q.put((1, g.err_bits()))
        assert _abi.CTR_GATHER_E_RELEASE_TIMEOUT == 4
        g.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_push_gather_unreleased_slot_times_out_without_hanging(cuda):
    """A consumer that never steps never releases its slots: the producer's k_step stores after a
    bounded wait and sets CTR_GATHER_E_RELEASE_TIMEOUT (steps 1-3 need no release: depth 3), and
    the overrun consumer's own err_bits() carry it too (poison words, ABI 14)."""
    import torch.multiprocessing as mp
    world, n = 2, 1024
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_stalled_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    errs = got[0]
    assert errs[:3] == [0, 0, 0], errs
    assert errs[3] & 4 and errs[4] & 4, errs
    assert got[1] & 4, got
