"""Soak of the fused push gather's flow control on one GPU: W processes (ranks on cuda:0, gloo for
the host side), each stepping its own 1 024-env shard `steps` times with random host delays and
NO synchronisation in the step loop, the fused consumer wait on (depth 3, as bench.py runs it).
After every step each rank copies the previous step's slot; at the end every copy is compared
bit for bit with a gloo all_gather of the ranks' own packed rows of that step, and every rank's
error word must be 0.  Prints one line per rank and TOTAL BAD <n>.

usage: python tools/push_soak.py [world] [steps]"""
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, n, steps, q):
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
        env = CtrReachVecEnv(n, device=dev, seed=11, env_base=rank * n, pack_outputs=True)
        env.reset()
        g = env.enable_gather("push", depth=3, wait_prev=True)
        rng = np.random.default_rng(100 + rank)
        hi = torch.tensor(env.action_space.high, device=dev)
        own, views = [], []
        for i in range(steps):
            if rng.random() < 0.3:
                time.sleep(float(rng.uniform(0, 0.004)))
            a = ((torch.rand((n, 6), device=dev) * 2 - 1) * hi).contiguous()
            env.step_raw(a)
            own.append(env.packed_outputs().clone())
            if i >= 1:
                views.append(g.slot_view(env.gather_seq - 1).clone())
        g.flush(torch.cuda.current_stream())
        torch.cuda.synchronize()
        bad = 0
        for s in range(steps - 1):
            blocks = [torch.empty_like(own[s].cpu()) for _ in range(world)]
            dist.all_gather(blocks, own[s].cpu())
            bad += int(not torch.equal(views[s].cpu(), torch.cat(blocks)))
        q.put((rank, bad, int(g.err.item())))
        dist.barrier()
        g.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, 1024, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    total = 0
    for rank, bad, err in res:
        print("rank %d: %d of %d gathered steps differ, error word %d" % (rank, bad, steps - 1, err), flush=True)
        total += bad + (err != 0)
    print("world %d, %d steps, TOTAL BAD %d" % (world, steps, total), flush=True)
    sys.exit(1 if total or any(p.exitcode != 0 for p in procs) else 0)
