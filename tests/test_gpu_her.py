"""GPU HER replay feed (ctr_her_open / ctr_her_record / ctr_her_sample) against the CPU restatement
of stable-baselines 2's HindsightExperienceReplayWrapper (oracle/her_oracle.py) fed with the same
per-step env outputs.

Bars: every sampled row (observation, action, reward, next observation, done) bit-equal to the
restatement's row with the same (env, reset number, t, j); stored episode lengths equal; the row
draws uniform over the stored rows (slot frequencies within 5 sigma of rows(L) / total).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GTP = {"inc_tol_obs": False, "final_tol": 0.001, "initial_tol": 0.05, "N_ts": 1000, "function": "constant",
       "set_tol": 0}


def _run(cuda, n=48, steps=60, t_max=12, slots=4, strategy="future", k=4, select_systems=(0,), fused=True, **envkw):
    import torch
    import her_oracle as H
    from ctr_reach_amd import CtrReachVecEnv
    env = CtrReachVecEnv(n, device=cuda, seed=5, max_steps_per_episode=t_max, goal_tolerance_parameters=GTP,
                         select_systems=list(select_systems), **envkw)
    her = env.enable_her(slots=slots, n_sampled_goal=k, goal_selection_strategy=strategy)
    her.fused = fused
    env.reset()
    tol = env.get_goal_tolerance()
    rec = H.EpisodeRecorder(n, k=k, strategy=strategy, seed=her.seed)

    def c(x):
        return x.cpu().numpy().copy()

    obs, ag, dg, ep = c(env.obs), c(env.achieved_goal), c(env.desired_goal), c(env.epoch)
    for e in range(n):
        rec.open(e, obs[e], ag[e], dg[e], ep[e])
    g = torch.Generator(device=cuda)
    g.manual_seed(9)
    hi = torch.tensor(env.action_space.high, device=cuda)
    for _ in range(steps):
        a = ((torch.rand((n, 6), generator=g, device=cuda) * 2 - 1) * hi * 3).contiguous()
        env.step(a)
        A, R, D = c(a), c(env.reward), c(env.done)
        obs, ag, dg, ep = c(env.obs), c(env.achieved_goal), c(env.desired_goal), c(env.epoch)
        tobs, tag = c(env.terminal_obs), c(env.terminal_achieved)
        for e in range(n):
            d = bool(D[e])
            rec.record(e, A[e], R[e], d, tobs[e] if d else obs[e], tag[e] if d else ag[e], tol)
            if d:
                rec.open(e, obs[e], ag[e], dg[e], ep[e])
    torch.cuda.synchronize()
    return env, her, rec


@pytest.mark.parametrize("strategy,systems,fused", [("future", (0,), True), ("final", (0, 1, 2, 3), True),
                                                    ("episode", (0,), True), ("future", (0,), False)])
def test_sampled_rows_match_restatement(cuda, oracle_mod, strategy, systems, fused):
    env, her, rec = _run(cuda, strategy=strategy, select_systems=systems, fused=fused)
    lens, eps = her.len.cpu().numpy(), her.epoch.cpu().numpy()
    stored = np.where(lens > 0)[0]
    assert len(stored) > 100
    for s in stored:                                  # the store holds finished episodes only
        key = (s // her.slots, int(eps[s]))
        assert key in rec.lengths and rec.lengths[key] == lens[s]
    assert len(her) == int(her.rows_per_episode(lens[stored]).sum())
    b = her.sample(8192, return_index=True)
    idx = b["index"].cpu().numpy()
    assert (idx[:, 0] >= 0).all()
    got = {k: b[k].cpu().numpy() for k in ("obs", "action", "reward", "next_obs", "done")}
    nrel = 0
    for i, (s, t, j) in enumerate(idx):
        row = rec.stored[(s // her.slots, int(eps[s]))][(t, j)]
        np.testing.assert_array_equal(got["obs"][i], row["obs"])
        np.testing.assert_array_equal(got["next_obs"][i], row["next_obs"])
        np.testing.assert_array_equal(got["action"][i], row["action"])
        assert got["reward"][i] == row["reward"] and got["done"][i] == row["done"]
        nrel += j > 0
    # k = 4 relabels per stored transition: about 4 in 5 rows are relabelled
    assert 0.7 < nrel / len(idx) < 0.85
    # relabelled rows with reward 0 exist (the next observation's own goal is a candidate)
    assert ((idx[:, 2] > 0) & (got["reward"] == 0)).any()


def test_sampling_is_uniform_over_rows(cuda, oracle_mod):
    env, her, rec = _run(cuda, n=32, steps=40)
    lens = her.len.cpu().numpy()
    rows = her.rows_per_episode(np.maximum(lens, 0)).astype(np.float64)
    B = 400000
    idx = her.sample(B, return_index=True)["index"].cpu().numpy()
    cnt = np.bincount(idx[:, 0], minlength=len(lens)).astype(np.float64)
    p = rows / rows.sum()
    sd = np.sqrt(B * p * (1 - p)) + 1e-9
    assert (np.abs(cnt - B * p) <= 5 * sd + 1e-9).all()
    assert cnt[rows == 0].sum() == 0
    # within an episode, transition t is drawn in proportion to its rows (k + 1, the last one 1)
    s0 = int(np.argmax(rows))
    ts = idx[idx[:, 0] == s0, 1]
    L = lens[s0]
    w = np.array([5.0] * (L - 1) + [1.0])
    ct = np.bincount(ts, minlength=L)
    exp = len(ts) * w / w.sum()
    assert (np.abs(ct - exp) <= 5 * np.sqrt(exp) + 1).all()


def test_reset_drops_unfinished_episodes(cuda, oracle_mod):
    env, her, rec = _run(cuda, n=16, steps=5, t_max=50)
    before = her.len.cpu().numpy().copy()
    assert (before == -1).sum() == 16                # one episode being recorded per env
    rows_before = len(her)                           # episodes that already ended (early success)
    env.reset()                                      # every env is mid-episode (t_max 50)
    lens = her.len.cpu().numpy()
    assert (lens == -1).sum() == 16                  # the new episodes; the unfinished ones dropped
    np.testing.assert_array_equal(lens[before > 0], before[before > 0])   # finished ones kept
    assert len(her) == rows_before


def test_empty_store_returns_flagged_rows(cuda):
    from ctr_reach_amd import CtrReachVecEnv
    env = CtrReachVecEnv(8, device=cuda, seed=1)
    her = env.enable_her()
    env.reset()
    b = her.sample(16, return_index=True)
    assert (b["index"][:, 0] == -1).all() and len(her) == 0


def test_one_step_episodes_never_miss(cuda):
    """Every episode ends at its first step (tolerance 1 m): one stored row per episode against the
    746 rows a 150-step episode holds.  The inverse-CDF draw still returns a stored row for every
    sample (a rejection sampler over (slot, row) would miss almost every draw here)."""
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    gtp = dict(GTP, initial_tol=1.0, final_tol=1.0)
    env = CtrReachVecEnv(64, device=cuda, seed=2, goal_tolerance_parameters=gtp)
    her = env.enable_her(slots=4)
    env.reset()
    for _ in range(3):
        env.step(torch.zeros((64, 6), device=cuda))
    lens = her.len.cpu().numpy()
    assert (lens > 0).sum() == 3 * 64 and (lens[lens > 0] == 1).all() and len(her) == 3 * 64
    idx = her.sample(65536, return_index=True)["index"].cpu().numpy()
    assert (idx[:, 0] >= 0).all() and (idx[:, 1] == 0).all() and (idx[:, 2] == 0).all()
    cnt = np.bincount(idx[:, 0], minlength=len(lens))
    assert (cnt[lens <= 0] == 0).all()
    exp = 65536 / (3 * 64)
    assert (np.abs(cnt[lens > 0] - exp) <= 5 * np.sqrt(exp)).all()


def test_rows_match_when_resets_miss_the_pool(cuda, oracle_mod):
    """A one-deep reset pool that is never refilled: from each env's second auto-reset on, the
    reset misses the pool and the sweep (k_reset) resets the env and opens its next HER episode.
    Rows stay bit-equal to the restatement's."""
    for fused in (True, False):
        _check_pool_misses(cuda, fused)


def _check_pool_misses(cuda, fused):
    env, her, rec = _run(cuda, n=32, steps=40, pool_depth=1, refill_interval=100000, fused=fused)
    lens, eps = her.len.cpu().numpy(), her.epoch.cpu().numpy()
    stored = np.where(lens > 0)[0]
    assert len(stored) > 64
    for s in stored:
        key = (s // her.slots, int(eps[s]))
        assert key in rec.lengths and rec.lengths[key] == lens[s]
    b = her.sample(4096, return_index=True)
    idx = b["index"].cpu().numpy()
    got = {k: b[k].cpu().numpy() for k in ("obs", "next_obs", "action", "reward")}
    for i, (s, t, j) in enumerate(idx):
        row = rec.stored[(s // her.slots, int(eps[s]))][(t, j)]
        np.testing.assert_array_equal(got["obs"][i], row["obs"])
        np.testing.assert_array_equal(got["next_obs"][i], row["next_obs"])
        assert got["reward"][i] == row["reward"]


def test_fused_and_unfused_recording_write_identical_stores(cuda, oracle_mod):
    """The same seeds and actions through ctr_step_her (recording inside k_step) and through
    ctr_step + ctr_her_record (a second launch reading the step outputs): every store buffer is
    byte-equal, pool misses (a one-deep pool, never refilled) included."""
    for envkw in ({}, dict(pool_depth=1, refill_interval=100000),
                  dict(integrator="rk4", rk4_steps_per_m=400, model="compliant")):   # the lane-pair step
        stores = []
        for fused in (True, False):
            env, her, rec = _run(cuda, n=40, steps=30, fused=fused, **envkw)
            stores.append({k: getattr(her, k).cpu().numpy().copy()
                           for k in ("state", "step_rows", "len", "epoch", "dg", "tol", "cur_t", "cur_epoch")})
        for k in stores[0]:
            np.testing.assert_array_equal(stores[0][k].view(np.uint8), stores[1][k].view(np.uint8), err_msg=k)


@pytest.mark.parametrize("fused", [True, False])
def test_reset_opens_episode_when_none_was_open(cuda, fused):
    """One rule on every path: every auto-reset opens the env's next episode, also for an env
    that had no open episode before the step (cur_t = -1), whether its reset comes from the
    pool (first reset after the refill) or from the miss sweep (the one-deep pool is empty)."""
    import torch
    from ctr_reach_amd import CtrReachVecEnv
    n = 128
    env = CtrReachVecEnv(n, device=cuda, seed=4, max_steps_per_episode=2, goal_tolerance_parameters=GTP,
                         pool_depth=1, refill_interval=100000)
    env.goal_tolerance.current_tol = 1e-12
    her = env.enable_her(slots=3)
    her.fused = fused
    env.reset()
    z = torch.zeros((n, 6), device=cuda)
    for cycle in range(2):                          # cycle 0: pooled reset; cycle 1: pool miss -> sweep
        env.step(z)
        her.cur_t[: n // 2] = -1                   # these envs have no open episode at the done step
        env.step(z)
        torch.cuda.synchronize()
        assert env.done.bool().all() and (env.t.cpu().numpy() == 0).all()
        assert (her.cur_t.cpu().numpy() == 0).all(), cycle
        np.testing.assert_array_equal(her.cur_epoch.cpu().numpy(), env.epoch.cpu().numpy().astype(np.uint32))
    assert env.sweeps > 0


def test_step_her_rejects_mismatched_store(cuda):
    from ctr_reach_amd import CtrReachVecEnv, _abi
    import torch
    env = CtrReachVecEnv(16, device=cuda, seed=1)
    her = env.enable_her()
    env.reset()
    a = torch.zeros((16, 6), device=cuda)
    her._h.t_max = env.max_steps_per_episode + 1
    rc = env.lib.ctr_step_her(env.cfg, env._batch, _abi.ptr(a), env._out, _abi.AUTORESET_POOLED, her._h,
                              _abi.stream_ptr())
    assert rc == -1 and b"t_max" in env.lib.ctr_last_error()
    her._h.t_max = env.max_steps_per_episode
    her._h.env_base = 5
    rc = env.lib.ctr_step_her(env.cfg, env._batch, _abi.ptr(a), env._out, _abi.AUTORESET_POOLED, her._h,
                              _abi.stream_ptr())
    assert rc == -1 and b"env_base" in env.lib.ctr_last_error()
