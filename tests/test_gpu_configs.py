"""GPU runs of the BASELINE.json configurations that the other tests size down, and of bench.py.

* configs[3] (524 288 envs sharded over 8 GPUs + all-gather of tip/reward/done): on one GPU the
  eight env_base shards of 65 536 envs are stepped next to ONE 524 288-env batch.  Bars: joints,
  goals, t, epoch, obs bit-exact (every draw is keyed by the global env id); the shards' packed
  gather rows concatenated equal the big batch's, bit for bit, and equal the step outputs.
* configs[4] (65 536 envs, compliant, RK4 at 400 steps/m) at full size: joint constraints and
  step outputs hold for the whole batch, and a 4 096-env subset of the last step matches the
  oracle (tips <= 1e-11 m, joints / reward bit-exact).
* bench.py's steady-state window (staggered episodes, refills inside the window) and its
  two-rank entry point (gloo rehearsal on one GPU).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _acts(rng, n, hi):
    return (rng.uniform(-1, 1, (n, 6)) * hi).astype(np.float32)


def _packed_want(env):
    import torch
    d = env.done.bool()
    tip = torch.where(d[:, None], env.terminal_achieved, env.achieved_goal).float()
    flags = env.done.float() + 2 * env.success.float() + 4 * (env.reward < 0).float()
    return torch.cat([tip, flags[:, None]], 1)


def test_configs3_eight_shards_match_one_batch(cuda):
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    shards, n = 8, 65536
    N = shards * n
    kw = dict(device=cuda, seed=42, max_steps_per_episode=3, pack_outputs=True)   # time-limit resets every 3 steps
    full = CtrReachVecEnv(N, **kw)
    full.goal_tolerance.current_tol = 0.03                                          # and early successes
    parts = [CtrReachVecEnv(n, env_base=r * n, **kw) for r in range(shards)]
    for p in parts:
        p.goal_tolerance.current_tol = 0.03
    full.reset()
    for p in parts:
        p.reset()
    rng = np.random.default_rng(8)
    resets0 = int(full.epoch.sum().item())
    for _ in range(7):
        act = torch.tensor(_acts(rng, N, full.action_space.high), device=cuda)
        full.step(act)
        for r, p in enumerate(parts):
            p.step(act[r * n:(r + 1) * n].contiguous())
        torch.cuda.synchronize()
        got = torch.cat([p.packed_outputs() for p in parts])
        assert torch.equal(got, full.packed_outputs())
        assert torch.equal(full.packed_outputs(), _packed_want(full))
    assert int(full.epoch.sum().item()) - resets0 > N      # every env reset at least once in the window
    for k in ("joints", "achieved_goal", "desired_goal", "t", "epoch", "system", "obs"):
        np.testing.assert_array_equal(getattr(full, k).cpu().numpy(),
                                      np.concatenate([getattr(p, k).cpu().numpy() for p in parts]), err_msg=k)


def test_configs4_full_size_rk4_fine(cuda, oracle_mod):
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    n, spm = 65536, 400
    env = CtrReachVecEnv(n, device=cuda, seed=12, integrator="rk4", rk4_steps_per_m=spm, model="compliant")
    env.reset()
    rng = np.random.default_rng(6)
    L = np.array([0.431, 0.332, 0.174])
    for _ in range(6):
        a = _acts(rng, n, env.action_space.high)
        q_before = env.joints.cpu().numpy().copy()
        dg_before = env.desired_goal.cpu().numpy().copy()
        t_before = env.t.cpu().numpy().copy()
        obs, rew, done, info = env.step(torch.tensor(a, device=cuda))
        torch.cuda.synchronize()
    q = env.joints.cpu().numpy()
    assert (q[:, :3] <= 0).all() and (q[:, :3] >= np.float32(-L + 1e-3) - 1e-7).all()
    assert (info["status"].cpu().numpy() == 0).all()
    ag = env.achieved_goal.cpu().numpy()
    assert np.isfinite(ag).all() and np.isfinite(env.obs.cpu().numpy()).all()
    err = info["error"].cpu().numpy()
    d = done.cpu().numpy()
    idx = np.where(~d)[0][:4096]
    # reward / error consistent with the goal distance for the whole batch (non-reset envs)
    dist = np.linalg.norm(ag[~d] - env.desired_goal.cpu().numpy()[~d], axis=1)
    np.testing.assert_allclose(err[~d], dist.astype(np.float32), rtol=1e-6)
    ref = oracle_mod.step(q_before[idx], a[idx], dg_before[idx], t_before[idx], env.get_goal_tolerance(),
                          integrator="rk4", steps_per_m=spm, model="compliant")
    np.testing.assert_array_equal(q[idx], ref["joints"])
    assert np.abs(ag[idx] - ref["achieved_goal"]).max() < 1e-11
    np.testing.assert_array_equal(rew.cpu().numpy()[idx], ref["reward"].astype(np.float32))


def _bench(args, env=None, timeout=300):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args, env=e, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_window_holds_steady_state_resets(cuda):
    n, steps = 8192, 10
    out = _bench(["--envs", str(n), "--steps", str(steps), "--warmup", "2", "--no-cpu-baseline"])
    ss = out["config"]["steady_state"]
    assert out["n_gpus"] == 1 and out["steps"] == steps
    assert ss["refills_in_window"] == 1 and out["config"]["reset_pool"]["refill_interval"] == steps
    # staggered clocks: about n / 150 time-limit resets per step, plus early successes
    expect = n * steps / 150.0
    assert 0.6 * expect < ss["resets_in_window"] < 3.0 * expect, ss


def test_bench_two_ranks_gloo_rehearsal(cuda):
    """bench.py --gpus 2 launches its own two ranks (gloo, both on cuda:0 here) with the
    per-step gather on; the line reports both ranks' envs."""
    out = _bench(["--gpus", "2", "--envs", "2048", "--steps", "4", "--warmup", "1", "--gather", "on"],
                 env={"CTR_BENCH_BACKEND": "gloo", "CTR_BENCH_SAME_DEVICE": "1"})
    assert out["n_gpus"] == 2 and out["config"]["global_envs"] == 4096
    assert out["config"]["process_group"] == {"backend": "gloo", "world_size": 2}
    assert out["config"]["all_gather"]["bytes_per_env"] == 16
    assert out["config"]["steady_state"]["refills_in_window"] == 2


@pytest.mark.parametrize("systems,rand", [([0], 0.0), ([0, 1, 2, 3], 0.0), ([0, 1, 2, 3], 0.05)])
def test_configs4_pair_step_matches_one_lane_fk(cuda, systems, rand):
    """configs[4]'s k_step runs each env on a lane pair (fk_pair_rk4, work-ranked inside 512-lane
    workgroups); the FK operator (ctr_fk) runs one env per lane (fk_lane_rk4).  Same ODE and step
    plan, the twist rounded in another order: the step's tips equal the operator's on the post-step
    joints to rounding (<= 1e-12 m; mixed systems, domain-randomised tables, a ragged batch), and
    the RHS counts are equal."""
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    n = 65536 - 77
    env = CtrReachVecEnv(n, device=cuda, seed=4, integrator="rk4", rk4_steps_per_m=400, model="compliant",
                         select_systems=systems, domain_rand=rand, autoreset=False)
    env.reset()
    rng = np.random.default_rng(8)
    for _ in range(2):
        env.step(torch.tensor(_acts(rng, n, env.action_space.high), device=cuda))
    torch.cuda.synchronize()
    tables = env.domain_parameters()["table"] if rand else None
    tip, st = env.forward_kinematics(env.joints, None if rand else env.system, tables=tables, return_stats=True)
    torch.cuda.synchronize()
    assert np.abs(env.achieved_goal.cpu().numpy() - tip.cpu().numpy()).max() < 1e-12
    env.enable_nfev()
    env.step(torch.zeros((n, 6), device=cuda))
    tip, st = env.forward_kinematics(env.joints, None if rand else env.system, tables=tables, return_stats=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(env.nfev.cpu().numpy(), st["nfev"].cpu().numpy())
    assert np.abs(env.achieved_goal.cpu().numpy() - tip.cpu().numpy()).max() < 1e-12
