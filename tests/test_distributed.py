"""Multi-process (world_size 2, gloo, CPU) coverage of the sharded path: disjoint contiguous
env-id shards, shard-invariant reset draws and steps (checked with the oracle standing in for
the GPU kernel), the optional all-gather of packed step outputs, and max-over-ranks timing."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        from ctr_reach_amd import distributed as D
        base = D.shard(n, rank)
        # reset draws keyed by global id (stand-in for k_reset on this rank's shard)
        qd, _ = oracle.sample_joints(n, seed=99, stream=0, epoch=1, env_base=base)
        q0, _ = oracle.sample_joints(n, seed=99, stream=1, epoch=1, env_base=base)
        dg = oracle.fk(qd)["tip"]
        rng = np.random.default_rng(1000 + base)
        a = (rng.uniform(-1, 1, (n, 6)) * np.array([1e-3] * 3 + [0.087] * 3)).astype(np.float32)
        r = oracle.step(q0, a, dg, 0, 0.05)
        packed = D.pack_step_outputs(torch.tensor(r["achieved_goal"]), torch.tensor(r["reward"], dtype=torch.float32),
                                     torch.tensor(r["done"]), torch.tensor(r["is_success"]))
        full = D.all_gather_outputs(packed)
        full_async, work = D.all_gather_outputs(packed, async_op=True)     # overlapped form
        work.wait()
        assert torch.equal(full, full_async)
        t = D.max_over_ranks(0.5 + rank)
        if rank == 0:
            q.put((full.numpy(), t))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_match_single_process():
    import oracle
    world, n = 2, 64
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 1.5                         # max over ranks
    from ctr_reach_amd import distributed as D
    assert full.shape == (world * n, D.PACK_WIDTH)
    # the same global envs stepped in ONE process
    N = world * n
    qd, _ = oracle.sample_joints(N, seed=99, stream=0, epoch=1, env_base=0)
    q0, _ = oracle.sample_joints(N, seed=99, stream=1, epoch=1, env_base=0)
    dg = oracle.fk(qd)["tip"]
    acts = []
    for r in range(world):
        rng = np.random.default_rng(1000 + r * n)
        acts.append((rng.uniform(-1, 1, (n, 6)) * np.array([1e-3] * 3 + [0.087] * 3)).astype(np.float32))
    ref = oracle.step(q0, np.concatenate(acts), dg, 0, 0.05)
    np.testing.assert_allclose(full[:, :3], ref["achieved_goal"].astype(np.float32))
    _, rew, _, _ = D.unpack_step_outputs(torch.tensor(full))
    np.testing.assert_array_equal(rew.numpy(), ref["reward"].astype(np.float32))
    flags = full[:, 3].astype(int)
    np.testing.assert_array_equal(flags & 1, ref["done"].astype(int))
    np.testing.assert_array_equal((flags >> 1) & 1, ref["is_success"].astype(int))


def test_shard_ranges_are_contiguous_and_disjoint():
    from ctr_reach_amd import distributed as D
    n, world = 65536, 8
    bases = [D.shard(n, r) for r in range(world)]
    assert bases == [r * n for r in range(world)]
    assert bases[-1] + n == world * n


def test_pack_roundtrip():
    from ctr_reach_amd import distributed as D
    ag = torch.randn(10, 3, dtype=torch.float64)
    rew = -torch.randint(0, 2, (10,)).float()
    done = torch.randint(0, 2, (10,)).bool()
    succ = torch.randint(0, 2, (10,)).bool()
    p = D.pack_step_outputs(ag, rew, done, succ)
    a2, r2, d2, s2 = D.unpack_step_outputs(p)
    assert torch.equal(d2, done) and torch.equal(s2, succ) and torch.equal(r2, rew)
    assert torch.allclose(a2, ag.float())


def _run_bench(args, env=None, timeout=240):
    import json
    import subprocess
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True, text=True,
                       timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


def test_bench_gpus_n_self_launches_ranks():
    """bench.py --gpus 2 without a launcher starts two ranks itself; they form one process group."""
    r, out = _run_bench(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert out == dict(out, dry_run=True, n_gpus=2, ranks_reporting=2, backend="gloo")


def test_bench_refuses_rank_count_mismatch():
    r, out = _run_bench(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and out is None
    assert "--gpus 4" in (r.stderr + r.stdout)


def test_refill_interval_tiles_the_window():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.refill_interval_for(20) == 20
    assert bench.refill_interval_for(128) == 64
    assert bench.refill_interval_for(100) == 50
    assert bench.refill_interval_for(7) == 7
    for k in range(1, 300):
        ri = bench.refill_interval_for(k)
        assert k % ri == 0 and 1 <= ri <= 64
