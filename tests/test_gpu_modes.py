"""GPU parity for the build's extra solver modes (BASELINE.json configs 2 and 5): fixed-step
RK4 and the torsionally-rigid model, through the C ABI, against the oracle restatement
(oracle/ctr_oracle.c rk4_span / rhs with rigid=1).  These modes have no reference
counterpart; their gap to the reference is pinned on the CPU side (test_oracle_modes.py).

Bars: tips within 1e-11 m of the oracle (fp64 both sides; the kernel contracts to FMA, the
oracle does not), RHS-evaluation counts identical, joints / reward / done bit-exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MODES = [("rk4", 100, "compliant"), ("rk4", 400, "compliant"), ("rk4", 100, "rigid"),
         ("rk45_scipy", 100, "rigid")]


def _joints(oracle_mod, n, seed):
    rng = np.random.default_rng(seed)
    sysid = rng.integers(0, 4, n).astype(np.int32)
    q = np.zeros((n, 6), np.float32)
    for s in range(4):
        m = sysid == s
        q[m], _ = oracle_mod.sample_joints(int(m.sum()), seed=seed + s, system=np.full(int(m.sum()), s))
    q[:, 3:] += rng.uniform(-10, 10, (n, 3)).astype(np.float32)
    return q, sysid


@pytest.mark.parametrize("integrator,spm,model", MODES)
def test_fk_modes_vs_oracle(cuda, oracle_mod, integrator, spm, model):
    from ctr_reach_amd import CtrReachVecEnv
    q, sysid = _joints(oracle_mod, 16384, 21)
    env = CtrReachVecEnv(1, device=cuda, select_systems=[0, 1, 2, 3], integrator=integrator,
                         rk4_steps_per_m=spm, model=model)
    tip, st = env.forward_kinematics(q, sysid, return_stats=True)
    ref = oracle_mod.fk(q, sysid, integrator=integrator, steps_per_m=spm, model=model)
    err = np.linalg.norm(tip.cpu().numpy() - ref["tip"], axis=1)
    assert err.max() < 1e-11, err.max()
    nfev = st["nfev"].cpu().numpy()
    if integrator == "rk4":
        np.testing.assert_array_equal(nfev, ref["nfev"])
        # the packed stats[2] is decoded: no rejections, the mapped segments apart
        assert (st["nrej"].cpu().numpy() == 0).all()
        maps = st["maps"].cpu().numpy()
        assert (maps <= st["nseg"].cpu().numpy()).all() and (st["compositions"].cpu().numpy() >= 0).all()
        if model == "rigid":
            assert (maps > 0).all()
    else:
        assert (nfev == ref["nfev"]).mean() > 0.999
    assert (st["status"].cpu().numpy() == 0).all()


@pytest.mark.parametrize("name", ["fk_random.npz", "fk_edge.npz", "csv_known.npz"])
def test_configs4_rk4_400_vs_reference_fixtures(cuda, golden_dir, name):
    """configs[4]'s GPU FK (compliant, RK4 at 400 steps/m) straight against the REFERENCE's tips
    (scipy RK45, model.py:141-151) on its own fixtures: the north_star bar (<= 1e-4 m) with the
    per-system bars of test_oracle_modes.RK4_400_BARS, and p99.9 <= 1e-4 m per system."""
    import os
    from ctr_reach_amd import CtrReachVecEnv
    from test_oracle_modes import RK4_400_BARS
    d = np.load(os.path.join(golden_dir, name))
    ref = d["tip"] if "tip" in d.files else d["tip_reference"]
    sysid = d["system"].astype(np.int32)
    env = CtrReachVecEnv(1, device=cuda, select_systems=[0, 1, 2, 3], integrator="rk4",
                         rk4_steps_per_m=400, model="compliant")
    tip = env.forward_kinematics(d["joints"].astype(np.float32), sysid).cpu().numpy()
    err = np.linalg.norm(tip - ref, axis=1)
    for s, bar in RK4_400_BARS.items():
        e = err[sysid == s]
        if e.size:
            assert e.max() < bar, (s, e.max())
            assert np.quantile(e, 0.999) <= 1e-4, (s, np.quantile(e, 0.999))
    assert (err <= 1e-4).mean() >= 0.999


@pytest.mark.parametrize("integrator,spm,model", MODES[:3])
def test_step_modes_vs_oracle(cuda, oracle_mod, integrator, spm, model):
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    n = 4096
    env = CtrReachVecEnv(n, device=cuda, seed=5, select_systems=[0, 1, 2, 3], autoreset=False,
                         integrator=integrator, rk4_steps_per_m=spm, model=model)
    env.enable_nfev()
    env.reset()
    rng = np.random.default_rng(3)
    hi = env.action_space.high
    for _ in range(3):
        q = env.joints.cpu().numpy()
        dg = env.desired_goal.cpu().numpy()
        t = env.t.cpu().numpy()
        sysid = env.system.cpu().numpy()
        a = ((rng.random((n, 6)) * 2 - 1) * hi).astype(np.float32)
        obs, rew, done, info = env.step(torch.tensor(a, device=cuda))
        torch.cuda.synchronize()
        ref = oracle_mod.step(q, a, dg, t, env.goal_tolerance.get_tol(), system=sysid, multi=True,
                              integrator=integrator, steps_per_m=spm, model=model)
        np.testing.assert_array_equal(env.joints.cpu().numpy(), ref["joints"])
        assert np.abs(env.achieved_goal.cpu().numpy() - ref["achieved_goal"]).max() < 1e-11
        np.testing.assert_array_equal(rew.cpu().numpy(), ref["reward"].astype(np.float32))
        np.testing.assert_array_equal(done.cpu().numpy(), ref["done"])
        assert np.abs(obs["observation"].cpu().numpy() - ref["observation"]).max() < 1e-6
        # RHS counts (rigid RK4: the lane group's summed 4 n per segment)
        assert (env.nfev.cpu().numpy() == ref["nfev"]).mean() > 0.999
        if done.any():
            break


def test_rigid_group_step_edge_joints(cuda, oracle_mod, golden_dir):
    """configs[1]'s step runs one env on 8 lanes, which rank the 10 segment points between them
    (seg_build_group) instead of sorting them each.  Edge joints (fk_edge.npz: ties, limits,
    reversed sub-um spans) under zero, +max, -max and mixed-sign max actions, which drive joints
    onto the action-box limits (ties with 0 and between tubes): joints, reward and done
    bit-exact, tips within 1e-11 m of the oracle, equal RHS counts."""
    import os
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    d = np.load(os.path.join(golden_dir, "fk_edge.npz"))
    q0, s0 = d["joints"], d["system"].astype(np.int32)
    m = len(q0)
    env0 = CtrReachVecEnv(1, device=cuda)
    hi = env0.action_space.high
    signs = np.array([[0, 0, 0, 0, 0, 0], [1, 1, 1, 1, 1, 1], [-1, -1, -1, -1, -1, -1],
                      [1, -1, 1, -1, 1, -1], [-1, 1, -1, 1, -1, 1]], np.float32)
    q = np.tile(q0, (len(signs), 1))
    sysid = np.tile(s0, len(signs))
    a = (np.repeat(signs, m, axis=0) * hi).astype(np.float32)
    n = len(q)
    env = CtrReachVecEnv(n, device=cuda, seed=9, select_systems=[0, 1, 2, 3], autoreset=False,
                         integrator="rk4", rk4_steps_per_m=100, model="rigid")
    env.enable_nfev()
    env.reset()
    env.joints.copy_(torch.tensor(q, device=cuda))
    env.system.copy_(torch.tensor(sysid, device=cuda))
    for _ in range(3):
        qi = env.joints.cpu().numpy()
        dg = env.desired_goal.cpu().numpy()
        t = env.t.cpu().numpy()
        obs, rew, done, info = env.step(torch.tensor(a, device=cuda))
        torch.cuda.synchronize()
        ref = oracle_mod.step(qi, a, dg, t, env.goal_tolerance.get_tol(), system=sysid, multi=True,
                              integrator="rk4", steps_per_m=100, model="rigid")
        np.testing.assert_array_equal(env.joints.cpu().numpy(), ref["joints"])
        assert np.abs(env.achieved_goal.cpu().numpy() - ref["achieved_goal"]).max() < 1e-11
        np.testing.assert_array_equal(rew.cpu().numpy(), ref["reward"].astype(np.float32))
        np.testing.assert_array_equal(done.cpu().numpy(), ref["done"])
        np.testing.assert_array_equal(env.nfev.cpu().numpy(), ref["nfev"])


def test_reset_goals_follow_mode(cuda, oracle_mod):
    """Reset goals are the FK of the drawn joints under the env's own solver mode."""
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    n = 2048
    env = CtrReachVecEnv(n, device=cuda, seed=8, select_systems=[0, 1, 2, 3], integrator="rk4",
                         rk4_steps_per_m=100, model="rigid")
    env.reset()
    torch.cuda.synchronize()
    sysid = env.system.cpu().numpy()
    dg = oracle_mod.fk(env.desired_joints.cpu().numpy(), sysid, integrator="rk4", steps_per_m=100,
                       model="rigid")["tip"]
    assert np.abs(env.desired_goal.cpu().numpy() - dg).max() < 1e-11


def test_tube_gap_nan_status(cuda):
    """A tube gap (joints outside the nesting constraints) gives a NaN tip and CTR_STATUS_NAN
    (the reference never returns there; see test_oracle_modes.py)."""
    from ctr_reach_amd import CtrReachVecEnv
    from test_oracle_modes import GAP_JOINTS
    env = CtrReachVecEnv(1, device=cuda)
    tip, st = env.forward_kinematics(np.array([GAP_JOINTS], np.float32), return_stats=True)
    assert np.isnan(tip.cpu().numpy()).all()
    assert st["status"].cpu().numpy()[0] & 4


def test_fk_huge_angles_vs_oracle(cuda, oracle_mod):
    """Joint angles of magnitude >= 2^18 (e.g. alpha accumulated over many episodes without
    resampling) take the wave-uniform careful path: exact large-argument sin/cos for any angle
    difference >= 2^20.  Mixed with ordinary waves; tips vs the oracle (libm sin/cos)."""
    from ctr_reach_amd import CtrReachVecEnv
    n = 4096
    q, sysid = _joints(oracle_mod, n, 31)
    rng = np.random.default_rng(2)
    big = np.zeros(n, bool)
    big[:64] = True                           # the first wave: every lane huge
    big[64 * 5 + 3] = True                    # one lane of another wave
    big[64 * 9:64 * 9 + 32] = True            # half a wave
    q[big, 3:] = (rng.choice([-1, 1], (big.sum(), 3)) * rng.uniform(3e5, 3e6, (big.sum(), 3))).astype(np.float32)
    env = CtrReachVecEnv(1, device=cuda, select_systems=[0, 1, 2, 3])
    tip, st = env.forward_kinematics(q, sysid, return_stats=True)
    ref = oracle_mod.fk(q, sysid)
    err = np.linalg.norm(tip.cpu().numpy() - ref["tip"], axis=1)
    # at |alpha| ~ 1e6 one ulp of an angle is ~1e-10 rad: FMA vs separately rounded stage angles
    # move the tip by up to ~1e-8 m; ordinary lanes keep the usual agreement
    assert err[big].max() < 1e-6, err[big].max()
    assert err[~big].max() < 1e-10, err[~big].max()
    assert np.isfinite(tip.cpu().numpy()).all()


@pytest.mark.parametrize("integrator,spm,model", [("rk45_scipy", 100, "compliant"), ("rk4", 100, "compliant"),
                                                  ("rk4", 100, "rigid")])
def test_nan_and_far_joints_terminate(cuda, integrator, spm, model):
    """FK inputs the reference cannot integrate end with a status flag instead of a hang: NaN
    angles (scipy would loop on a NaN step size) -> NAN / STEP_UNDERFLOW; a fixed-step RK4
    segment of more than 2^20 steps -> TOO_LONG with a NaN tip.  The env's own step (the 8-lane
    group path for the rigid model) is bounded the same way."""
    import torch
    from ctr_reach_amd import CtrReachVecEnv, _abi
    q = np.array([[-0.1, -0.05, -0.02, np.nan, 0.2, 0.3],
                  [-0.1, -0.05, -0.02, 0.1, np.nan, 0.3],
                  [np.nan, -0.05, -0.02, 0.1, 0.2, 0.3],
                  [5e4, -0.05, -0.02, 0.1, 0.2, 0.3]], np.float32)
    env = CtrReachVecEnv(4, device=cuda, seed=1, integrator=integrator, rk4_steps_per_m=spm, model=model)
    tip, st = env.forward_kinematics(torch.tensor(q, device=cuda), return_stats=True)
    torch.cuda.synchronize()
    status = st["status"].cpu().numpy()
    assert (status[:2] & (_abi.CTR_STATUS_NAN | _abi.CTR_STATUS_STEP_UNDERFLOW)).all()
    if integrator == "rk4":
        assert status[3] & _abi.CTR_STATUS_TOO_LONG and np.isnan(tip.cpu().numpy()[3]).all()
    else:
        assert status[3] & _abi.CTR_STATUS_NAN                      # the tube gap [0, 5e4]
    env.reset()
    env.joints.copy_(torch.tensor(q, device=cuda))
    env.step(torch.zeros((4, 6), device=cuda))
    torch.cuda.synchronize()


@pytest.mark.parametrize("integrator,spm,model", MODES + [("rk45_scipy", 100, "compliant")])
def test_fk_is_independent_of_wave_composition(cuda, oracle_mod, integrator, spm, model):
    """A lane's FK must not depend on which envs share its wave: the kernels pick a code path per
    wave (tube levels, the careful trig, the RK4 step level), so every path must give a lane the
    same bits -- the property the shard test, pooled-vs-synchronous resets and the refill's
    arbitrary lane pairing rest on.  The same joints in a permuted order (other wave mates) give
    bit-identical tips, RHS counts and status words; systems mixed, angles up to +-10 rad."""
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    q, sysid = _joints(oracle_mod, 16384, 33)
    env = CtrReachVecEnv(1, device=cuda, select_systems=[0, 1, 2, 3], integrator=integrator,
                         rk4_steps_per_m=spm, model=model)
    tip, st = env.forward_kinematics(q, sysid, return_stats=True)
    perm = np.random.default_rng(5).permutation(q.shape[0])
    tip_p, st_p = env.forward_kinematics(q[perm], sysid[perm], return_stats=True)
    inv = np.argsort(perm)
    np.testing.assert_array_equal(tip_p.cpu().numpy()[inv], tip.cpu().numpy())
    for k in st:                      # nfev nstep nrej nseg status (+ RK4's maps, compositions)
        np.testing.assert_array_equal(st_p[k].cpu().numpy()[inv], st[k].cpu().numpy(), err_msg=k)
    torch.cuda.synchronize()
