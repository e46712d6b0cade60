"""CPU checks of the HER replay restatement (oracle/her_oracle.py) against the stable-baselines 2
HindsightExperienceReplayWrapper semantics it restates (row order, future-goal ranges, relabelled
reward / done, unchanged 'observation' part).  stable-baselines is absent: parity unpinned."""
import numpy as np
import pytest


def _episode(L, seed=0):
    rng = np.random.default_rng(seed)
    dg = rng.normal(size=3)
    obs = [dict(observation=rng.normal(size=13).astype(np.float32), achieved_goal=rng.normal(size=3) * 0.01,
                desired_goal=dg) for _ in range(L + 1)]
    return [(obs[t], rng.normal(size=6).astype(np.float32), -1.0, obs[t + 1], t == L - 1) for t in range(L)]


@pytest.mark.parametrize("strategy", ["future", "final", "episode"])
def test_store_episode_order_and_relabels(oracle_mod, strategy):
    import her_oracle as H
    L, k = 6, 4
    tr = _episode(L)
    rows = H.store_episode(tr, k, strategy, tol=0.02, seed=7, genv=3, epoch=2)
    n_rel = L - 1 if strategy == "future" else L
    assert len(rows) == L + k * n_rel
    # _store_episode order: the real transition, then its k relabels
    labels = [(r["t"], r["j"]) for r in rows]
    want = []
    for t in range(L):
        want.append((t, 0))
        if not (strategy == "future" and t == L - 1):
            want += [(t, j) for j in range(1, k + 1)]
    assert labels == want
    for r in rows:
        t = r["t"]
        obs_t, a, rew, obs_tp1, done = tr[t]
        np.testing.assert_array_equal(r["obs"][:13], obs_t["observation"])     # 'observation' kept
        np.testing.assert_array_equal(r["action"], a)
        if r["j"] == 0:
            assert r["reward"] == rew and r["done"] == float(done)
            np.testing.assert_array_equal(r["obs"][16:], np.float32(obs_t["desired_goal"]))
            continue
        assert r["done"] == 0.0
        goal = r["obs"][16:]
        np.testing.assert_array_equal(goal, r["next_obs"][16:])
        cands = {"future": range(t + 1, L), "final": [L - 1], "episode": range(L)}[strategy]
        matches = [s for s in cands if np.array_equal(np.float32(tr[s][0]["achieved_goal"]), goal)]
        assert matches, (t, r["j"])
        s = matches[0]
        want_r = -float(np.linalg.norm(obs_tp1["achieved_goal"] - tr[s][0]["achieved_goal"]) > 0.02)
        assert r["reward"] == want_r


def test_future_draws_cover_the_range(oracle_mod):
    import her_oracle as H
    L = 9
    for t in range(L - 1):
        sels = [H.sel_index(11, 5, e, t, j, L) for e in range(60) for j in range(1, 5)]
        assert min(sels) >= t + 1 and max(sels) <= L - 1
        assert set(sels) == set(range(t + 1, L))      # every later transition reachable
    # the next observation's own goal (sel = t + 1) earns reward 0
    tr = _episode(3)
    rows = H.store_episode(tr, 4, "future", tol=1e-9, seed=1, genv=0, epoch=0)
    r1 = [r for r in rows if r["t"] == 1 and r["j"] > 0]
    assert all(r["reward"] == 0.0 for r in r1)        # only sel = 2 = t + 1 is possible
