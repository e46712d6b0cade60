"""The optional RCCL all-gather of packed step outputs (CtrReachVecEnv.gather_outputs) on the GPU,
in a one-rank process group (the multi-rank logic is covered with gloo in test_distributed.py):
synchronous and overlapped (async_op) forms, and a step launched while the gather is in flight.

Bars: the gathered block equals the env's own (tip as float32, done | success << 1 |
(reward = -1) << 2) bit for bit, and unpacks to the env's reward / done / success."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _want(env, tip):
    """The packed rows of the env's last step (distributed.PACK_WIDTH), checked against unpack."""
    import torch
    from ctr_reach_amd import distributed as D
    flags = env.done.float() + 2 * env.success.float() + 4 * (env.reward < 0).float()
    want = torch.cat([tip, flags[:, None]], 1)
    t, r, d, sc = D.unpack_step_outputs(want)
    assert torch.equal(r, env.reward) and torch.equal(d, env.done.bool()) and torch.equal(sc, env.success.bool())
    return want


def test_gather_outputs_over_rccl(cuda):
    import torch
    import torch.distributed as dist
    from ctr_reach_amd import CtrReachVecEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=cuda)
    try:
        n = 1024
        env = CtrReachVecEnv(n, device=cuda, seed=4)
        env.reset()
        g = torch.Generator(device=cuda)
        g.manual_seed(2)
        hi = torch.tensor(env.action_space.high, device=cuda)
        act = lambda: ((torch.rand((n, 6), generator=g, device=cuda) * 2 - 1) * hi).contiguous()  # noqa: E731
        env.step(act())
        full = env.gather_outputs()
        d = env.done.bool()
        tip = torch.where(d[:, None], env.terminal_achieved, env.achieved_goal).float()
        want = _want(env, tip)
        assert torch.equal(full, want)
        # overlapped: the gather of step k runs while step k + 1 is launched
        out, work = env.gather_outputs(async_op=True)
        want = want.clone()
        env.step(act())
        work.wait()
        torch.cuda.synchronize()
        assert torch.equal(out, want)
    finally:
        dist.destroy_process_group()


def test_gather_of_kernel_packed_rows_over_rccl(cuda):
    """pack_outputs=True: k_step writes the gather rows itself (alternating buffers); the RCCL
    gather of step k, left in flight while step k + 1 runs, returns step k's rows."""
    import torch
    import torch.distributed as dist
    from ctr_reach_amd import CtrReachVecEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=cuda)
    try:
        n = 4096
        env = CtrReachVecEnv(n, device=cuda, seed=9, pack_outputs=True, max_steps_per_episode=2)
        env.reset()
        rng = np.random.default_rng(3)
        for _ in range(4):
            act = torch.tensor((rng.uniform(-1, 1, (n, 6)) * env.action_space.high).astype(np.float32), device=cuda)
            env.step(act)
            d = env.done.bool()
            tip = torch.where(d[:, None], env.terminal_achieved, env.achieved_goal).float()
            want = _want(env, tip)
            out, work = env.gather_outputs(async_op=True)
            env.step(act)                      # writes the other pack buffer while the gather runs
            work.wait()
            torch.cuda.synchronize()
            assert torch.equal(out, want)
    finally:
        dist.destroy_process_group()
