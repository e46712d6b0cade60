"""Evaluation-mode outputs: the facade's evaluation=True info dict (ctr_reach_env.py:144-153) on
the reference's own evaluation episodes (tests/golden/eval_info.npz, from make_golden.py), and
the batched env's record_info buffers (desired_joints, starting_joints, starting_position) after
auto-resets.

Bars: q_achieved / q_desired / q_starting / system_idx / tolerances / is_success exact;
errors_pos, achieved_goal and starting_position within TIP_TOL of the reference (1e-10 m);
the record_info tips equal the FK of the recorded joints (device FK, 1e-12 m; oracle TIP_TOL)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TIP_TOL = 1e-10


def test_facade_evaluation_info_vs_reference(golden_dir, cuda):
    import torch
    from ctr_reach_amd import make
    d = np.load(os.path.join(golden_dir, "eval_info.npz"))
    select = [int(s) for s in d["select_systems"]]
    env = make("CTR-Reach-v0", device=cuda, select_systems=select, evaluation=True, constrain_alpha=False)
    n_ep = len(d["reset_system"])
    checked = 0
    for ep in range(n_ep):
        rows = np.nonzero(d["episode"] == ep)[0]
        sysi = int(d["reset_system"][ep])
        env.goal_tolerance.current_tol = float(d["tol"][rows[0]])
        # the reference's reset: goal and system given; the start joints replace the sampled ones
        env.reset(goal=d["reset_desired_goal"][ep], system=sysi)
        q0 = d["reset_starting_joints"][ep]
        env.vec.joints.copy_(torch.tensor(q0[None]))
        sp = env.model.forward_kinematics(q0, sysi)           # the start FK, on the GPU
        assert np.abs(sp - d["reset_starting_position"][ep]).max() < TIP_TOL
        env.vec.achieved_goal.copy_(torch.tensor(sp[None]))
        env.starting_position, env.starting_joints = sp, q0.copy()
        env.desired_joints = d["reset_desired_joints"][ep].copy()
        dg = env.model.forward_kinematics(env.desired_joints, sysi)   # the goal FK, on the GPU
        assert np.abs(dg - d["reset_desired_goal"][ep]).max() < TIP_TOL
        for i in rows:
            obs, reward, done, info = env.step(d["action"][i])
            assert reward == d["reward"][i] and done == bool(d["done"][i])
            assert info["is_success"] == bool(d["is_success"][i])
            assert abs(info["errors_pos"] - d["errors_pos"][i]) < TIP_TOL
            assert info["errors_orient"] == d["errors_orient"][i] == 0
            assert info["orientation_tolerance"] == d["orientation_tolerance"][i] == 0
            assert info["system_idx"] == d["system_idx"][i] == select[sysi]
            assert info["position_tolerance"] == d["position_tolerance"][i]
            np.testing.assert_array_equal(np.asarray(info["q_achieved"], np.float64), d["q_achieved"][i])
            np.testing.assert_array_equal(np.asarray(info["q_desired"], np.float64), d["q_desired"][i])
            np.testing.assert_array_equal(np.asarray(info["q_starting"], np.float64), d["q_starting"][i])
            assert np.abs(info["achieved_goal"] - d["achieved_goal"][i]).max() < TIP_TOL
            np.testing.assert_array_equal(info["desired_goal"], d["desired_goal"][i])
            assert np.abs(info["starting_position"] - d["starting_position"][i]).max() < TIP_TOL
            assert np.abs(obs["observation"] - d["observation"][i]).max() < 1e-7
            checked += 1
    assert checked == len(d["t"]) and checked > 200


def test_record_info_after_autoresets(cuda, oracle_mod):
    """CtrReachVecEnv(record_info=True): after pooled auto-resets, every env's desired_goal is the
    FK of desired_joints, starting_position the FK of starting_joints (the episode's first
    achieved goal), and an env reset in this step holds its starting joints."""
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    n = 2048
    env = CtrReachVecEnv(n, device=cuda, seed=13, max_steps_per_episode=3, select_systems=[0, 1, 2, 3],
                         refill_interval=2)
    env.goal_tolerance.current_tol = 0.03
    env.reset()
    rng = np.random.default_rng(8)
    for _ in range(7):
        act = torch.tensor((rng.uniform(-1, 1, (n, 6)) * env.action_space.high).astype(np.float32), device=cuda)
        env.step(act)
    torch.cuda.synchronize()
    assert int(env.epoch.min().item()) >= 3                  # every env auto-reset at least twice
    sysid = env.system.cpu().numpy()
    qd, q0 = env.desired_joints.cpu().numpy(), env.starting_joints.cpu().numpy()
    dg, sp = env.desired_goal.cpu().numpy(), env.starting_position.cpu().numpy()
    assert np.abs(env.forward_kinematics(env.desired_joints, env.system).cpu().numpy() - dg).max() < 1e-12
    assert np.abs(env.forward_kinematics(env.starting_joints, env.system).cpu().numpy() - sp).max() < 1e-12
    systems = oracle_mod.make_systems(select=[0, 1, 2, 3])
    assert np.abs(oracle_mod.fk(qd, sysid, systems=systems)["tip"] - dg).max() < TIP_TOL
    assert np.abs(oracle_mod.fk(q0, sysid, systems=systems)["tip"] - sp).max() < TIP_TOL
    fresh = env.t.cpu().numpy() == 0
    assert fresh.any()
    np.testing.assert_array_equal(env.joints.cpu().numpy()[fresh], q0[fresh])
    np.testing.assert_array_equal(env.achieved_goal.cpu().numpy()[fresh], sp[fresh])
