"""CPU restatement of the HER replay feed's reference algorithm -- TEST INFRASTRUCTURE ONLY
(imported by tests/, never by the product package).

The reference trains with stable-baselines 2 HER (absent here and from /root/reference: an
external dependency of the reference's src/ scripts, `from stable_baselines import DDPG, HER`,
e.g. src/jacobian_controller.py:6; version unpinned, the saved models are stable-baselines 2.x
zips).  Its settings are in saved_policies/**/her/CTR-Generic-Reach-v0_1/CTR-Generic-Reach-v0/
config.yml: goal_selection_strategy future, n_sampled_goal 4, batch_size 256, buffer_size 500000.
This file restates the published algorithm of stable_baselines/her/replay_buffer.py
(HindsightExperienceReplayWrapper):

    add(obs_t, action, reward, obs_tp1, done, info):
        episode_transitions.append(...); if done: _store_episode(); episode_transitions = []
    _store_episode():
        for transition_idx, transition in enumerate(episode_transitions):
            replay_buffer.add(obs_t, action, reward, obs_tp1, done)
            if transition_idx == len(episode_transitions) - 1 and strategy == FUTURE: break
            for goal in [_sample_achieved_goal(episode_transitions, transition_idx) for _ in range(k)]:
                obs['desired_goal'] = next_obs['desired_goal'] = goal
                reward = env.compute_reward(next_obs['achieved_goal'], goal, info); done = False
                replay_buffer.add(obs, action, reward, next_obs, done)
    _sample_achieved_goal(episode_transitions, transition_idx):
        FUTURE: selected = episode_transitions[choice(arange(transition_idx + 1, L))]
        FINAL: selected = episode_transitions[-1];  EPISODE: selected = ...[choice(arange(L))]
        return convert_obs_to_dict(selected[0])['achieved_goal']       # obs_t of that transition

with HERGoalEnvWrapper.convert_dict_to_obs = concatenate([observation, achieved_goal,
desired_goal]) and CtrReachEnv.compute_reward (envs/ctr_reach_env.py:160-170).  The random
choice is the build's Philox draw (stream 4, keyed by seed, global env id, reset number, t, j),
so GPU rows can be checked bit for bit; against stable-baselines itself the relabelling is
"parity unpinned" (the library is absent and the reference holds no HER fixtures).
"""
import numpy as np

import oracle


def u53(a, b):
    return ((int(a) >> 5) * 67108864.0 + (int(b) >> 6)) * (1.0 / 9007199254740992.0)


def sel_index(seed, genv, epoch, t, j, L, strategy="future"):
    """The transition whose obs_t gives relabel j (1..k) of transition t (ctr_her.inc her_sel)."""
    if strategy == "final":
        return L - 1
    c = oracle.philox([t | (j << 16), epoch & 0xFFFFFFFF, genv & 0xFFFFFFFF, ((genv >> 32) ^ (4 << 24)) & 0xFFFFFFFF],
                      seed)
    u = u53(c[0], c[1])
    lo = t + 1 if strategy == "future" else 0
    return min(lo + int(u * (L - lo)), L - 1)


def compute_reward(ag, dg, tol):
    """CtrReachEnv.compute_reward (ctr_reach_env.py:160-170) for one pair."""
    d = np.linalg.norm(np.asarray(ag, np.float64) - np.asarray(dg, np.float64), axis=-1)
    return -(d > tol).astype(np.float64)


def flat(obs):
    """HERGoalEnvWrapper.convert_dict_to_obs, stored as float32 as the device batch is."""
    return np.concatenate([obs["observation"], obs["achieved_goal"], obs["desired_goal"]]).astype(np.float32)


def store_episode(transitions, k, strategy, tol, seed, genv, epoch):
    """_store_episode: returns the rows in the wrapper's order as dicts with keys obs, action,
    reward, next_obs, done (flat float32 observations) and (t, j) labels."""
    rows = []
    L = len(transitions)
    for t, (obs_t, action, reward, obs_tp1, done) in enumerate(transitions):
        rows.append(dict(t=t, j=0, obs=flat(obs_t), action=np.asarray(action, np.float32), reward=float(reward),
                         next_obs=flat(obs_tp1), done=float(done)))
        if t == L - 1 and strategy == "future":
            break
        for j in range(1, k + 1):
            sel = sel_index(seed, genv, epoch, t, j, L, strategy)
            goal = transitions[sel][0]["achieved_goal"]
            o = dict(obs_t, desired_goal=goal)
            no = dict(obs_tp1, desired_goal=goal)
            rows.append(dict(t=t, j=j, obs=flat(o), action=np.asarray(action, np.float32),
                             reward=float(compute_reward(no["achieved_goal"], goal, tol)), next_obs=flat(no),
                             done=0.0))
    return rows


class EpisodeRecorder(object):
    """HindsightExperienceReplayWrapper.add over a vectorised env with auto-reset: feeds the
    per-step outputs env by env and stores each finished episode (keyed by env, reset number)."""

    def __init__(self, n, k=4, strategy="future", seed=0, env_base=0):
        self.n, self.k, self.strategy, self.seed, self.env_base = n, k, strategy, seed, env_base
        self.cur = [None] * n
        self.stored = {}        # (env, epoch) -> {(t, j): row}
        self.lengths = {}

    def open(self, e, obs, ag, dg, epoch):
        self.cur[e] = dict(epoch=int(epoch), obs=dict(observation=np.asarray(obs, np.float32).copy(),
                                                      achieved_goal=np.asarray(ag, np.float64).copy(),
                                                      desired_goal=np.asarray(dg, np.float64).copy()), tr=[])

    def record(self, e, action, reward, done, next_obs, next_ag, tol):
        c = self.cur[e]
        if c is None:
            return
        nobs = dict(observation=np.asarray(next_obs, np.float32).copy(), achieved_goal=np.asarray(next_ag).copy(),
                    desired_goal=c["obs"]["desired_goal"])
        c["tr"].append((c["obs"], np.asarray(action, np.float32).copy(), float(reward), nobs, bool(done)))
        c["obs"] = nobs
        if done:
            rows = store_episode(c["tr"], self.k, self.strategy, tol, self.seed, self.env_base + e, c["epoch"])
            self.stored[(e, c["epoch"])] = {(r["t"], r["j"]): r for r in rows}
            self.lengths[(e, c["epoch"])] = len(c["tr"])
            self.cur[e] = None
