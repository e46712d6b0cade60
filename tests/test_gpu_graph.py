"""Captured step sequences (CtrReachVecEnv.capture_steps, one HIP graph per refill period) replay
the same trajectory as stepping from Python: joints, goals, episode clocks, reset numbers,
observations, rewards, done flags and the reset pool bit-exact after several replays with
auto-resets and refills inside them (compliant scipy-RK45, the rigid 8-lane group path and
configs[4]'s lane-pair step)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEYS = ("joints", "desired_goal", "achieved_goal", "t", "epoch", "system", "obs", "reward", "done", "success",
        "terminal_obs", "pool_r", "pool_q0", "pool_dg")


@pytest.mark.parametrize("n,kw", [(2048, {}), (1024, dict(integrator="rk4", rk4_steps_per_m=100, model="rigid")),
                                  (1500, dict(integrator="rk4", rk4_steps_per_m=400, model="compliant"))])
def test_graph_replay_matches_eager_steps(cuda, n, kw):
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    R = 4
    mk = lambda: CtrReachVecEnv(n, device=cuda, seed=7, max_steps_per_episode=5, refill_interval=R,  # noqa: E731
                                select_systems=[0, 1, 2, 3], **kw)
    a, b = mk(), mk()
    for e in (a, b):
        e.goal_tolerance.current_tol = 0.03
        e.reset()
    rng = np.random.default_rng(4)
    acts = [torch.tensor((rng.uniform(-1, 1, (n, 6)) * a.action_space.high).astype(np.float32), device=cuda)
            for _ in range(R)]
    g = b.capture_steps(acts)
    for rep in range(3):
        for i in range(R):
            a.step_raw(acts[i])
        g.replay()
        torch.cuda.synchronize()
        for k in KEYS:
            assert torch.equal(getattr(a, k), getattr(b, k)), (rep, k)
    assert int((a.epoch - 1).sum().item()) > n        # resets inside the replays
    assert a.refills == b.refills


def test_capture_refuses_a_sequence_that_does_not_close(cuda):
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    env = CtrReachVecEnv(256, device=cuda, seed=1, refill_interval=4)
    env.reset()
    acts = [torch.zeros((256, 6), device=cuda)] * 3
    with pytest.raises(RuntimeError):
        env.capture_steps(acts)                        # not a multiple of the refill interval
    env.step_raw(acts[0])
    with pytest.raises(RuntimeError):
        env.capture_steps(acts + acts[:1])             # not on a refill boundary
