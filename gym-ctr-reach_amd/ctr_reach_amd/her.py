"""HerReplayBuffer -- the replay side of the reference's training pipeline, on the device.

The reference trains CTR-Reach with stable-baselines 2 HER + DDPG (goal_selection_strategy
'future', n_sampled_goal 4, batch_size 256, buffer_size 500000: saved_policies/**/her/
CTR-Generic-Reach-v0_1/CTR-Generic-Reach-v0/config.yml).  That wrapper keeps each episode's
transitions, and when the episode ends stores every transition plus, for all but the last one,
k copies whose desired goal is the achieved goal of a later observation of the same episode,
with the reward recomputed by ``env.compute_reward`` (envs/ctr_reach_env.py:160-170).
``ReplayBuffer.sample`` then draws rows uniformly.

Here the episodes are recorded where the environments run (``ctr_her_record`` after every
``ctr_step``; ``ctr_her_open`` after every ``ctr_reset``) and the relabelled rows are formed
when they are sampled (``ctr_her_sample``) from goal indices fixed per row, so a row costs no
HBM until it is drawn.  Sampled batches are device tensors in HERGoalEnvWrapper's flat layout
``[observation, achieved_goal, desired_goal]``.

Differences from stable-baselines (documented, not hidden):
  * capacity is in episodes: every env keeps its last ``slots - 1`` finished episodes (FIFO per
    env) instead of a global FIFO of rows;
  * the relabel draws come from Philox keyed (seed, global env id, reset number, t, j), not
    numpy's global RNG, so rows match the wrapper in distribution, not draw for draw.
"""
import numpy as np

from . import _abi

STRATEGIES = {"future": _abi.CTR_HER_FUTURE, "final": _abi.CTR_HER_FINAL, "episode": _abi.CTR_HER_EPISODE}


def _torch():
    import torch
    return torch


class HerReplayBuffer(object):
    def __init__(self, venv, slots=4, n_sampled_goal=4, goal_selection_strategy="future", seed=None):
        torch = _torch()
        if goal_selection_strategy not in STRATEGIES:
            raise ValueError("goal_selection_strategy must be one of %s" % sorted(STRATEGIES))
        if int(slots) < 2:
            raise ValueError("slots must be >= 2 (one episode is always being recorded)")
        if venv.obs_dtype != torch.float32:
            # ctr_her_open / ctr_her_record / the fused recording read the env's observation
            # rows as float32
            raise ValueError("the HER feed records float32 observations: build the env with obs_dtype='float32'")
        self.venv = venv
        self.lib = venv.lib
        self.n_sampled_goal = int(n_sampled_goal)
        self.strategy = goal_selection_strategy
        self.slots = int(slots)
        self.t_max = int(venv.max_steps_per_episode)
        self.obs_dim = venv.obs_dim
        self.seed = int(venv.seed_value if seed is None else seed) & 0xFFFFFFFFFFFFFFFF
        n, dev, T = venv.num_envs, venv.device, self.t_max
        E = n * self.slots
        f32, f64, i32 = torch.float32, torch.float64, torch.int32
        S = self.slots                     # env-minor 96-B / 32-B rows (include/ctr_reach_amd.h ctr_her_t)
        self.state = torch.zeros((S, T + 1, n, 24), dtype=f32, device=dev)
        self.step_rows = torch.zeros((S, T, n, 8), dtype=f32, device=dev)
        self.obs = self.state[..., :self.obs_dim]                       # views
        self.ag = self.state[..., 16:22].view(f64)
        self.action = self.step_rows[..., :6]
        self.reward = self.step_rows[..., 6]
        self.dg = torch.zeros((E, 3), dtype=f64, device=dev)
        self.tol = torch.zeros(E, dtype=f64, device=dev)
        self.len = torch.zeros(E, dtype=i32, device=dev)
        self.epoch = torch.zeros(E, dtype=i32, device=dev)
        self.cur_t = torch.full((n,), -1, dtype=i32, device=dev)
        self.cur_epoch = torch.zeros(n, dtype=i32, device=dev)
        tile = _abi.CTR_HER_SCAN_TILE        # sampler scratch: CTR_HER_CDF_LEN(E) prefix sums
        self.cdf = torch.zeros(E + (E + tile - 1) // tile + 1, dtype=torch.int64, device=dev)
        p = _abi.ptr
        h = self._h = _abi.CtrHer()
        h.obs_dim, h.t_max, h.n_sampled_goal, h.strategy = self.obs_dim, T, self.n_sampled_goal, STRATEGIES[self.strategy]
        h.n, h.env_base, h.slots, h.seed = n, venv.env_base, self.slots, self.seed
        h.state, h.step = p(self.state), p(self.step_rows)
        h.dg, h.tol, h.len, h.epoch = p(self.dg), p(self.tol), p(self.len), p(self.epoch)
        h.cur_t, h.cur_epoch, h.cdf = p(self.cur_t), p(self.cur_epoch), p(self.cdf)
        self._counter = 0
        self.fused = True        # record inside the step (ctr_step_her); False: ctr_her_record after it
        venv._her = self

    @property
    def nbytes(self):
        return sum(t.numel() * t.element_size() for t in (self.state, self.step_rows, self.dg, self.tol,
                                                           self.len, self.epoch, self.cur_t, self.cur_epoch,
                                                           self.cdf))

    # called by CtrReachVecEnv
    def _open(self, mask, stream):
        rc = self.lib.ctr_her_open(self._h, self.venv._batch, _abi.ptr(self.venv.obs), _abi.ptr(mask),
                                   _abi.stream_ptr(stream, self.venv.device.index))
        _abi.check(rc, "ctr_her_open")

    def _record(self, actions, stream):
        rc = self.lib.ctr_her_record(self._h, self.venv._batch, _abi.ptr(actions), self.venv._out,
                                     float(self.venv.cfg.tol), _abi.stream_ptr(stream, self.venv.device.index))
        _abi.check(rc, "ctr_her_record")

    def rows_per_episode(self, L):
        L = np.asarray(L, dtype=np.int64)
        if self.strategy == "future":
            return np.where(L > 0, L + self.n_sampled_goal * (L - 1), 0)
        return np.where(L > 0, L * (1 + self.n_sampled_goal), 0)

    def __len__(self):
        """Stored rows (len(ReplayBuffer) of the wrapper's buffer); synchronises."""
        return int(self.rows_per_episode(self.len.clamp(min=0).cpu().numpy()).sum())

    def sample(self, batch_size, seed=None, stream=None, return_index=False):
        """ReplayBuffer.sample(batch_size) on the device: dict of obs [B, d], action [B, 6],
        reward [B], next_obs [B, d], done [B] (d = obs_dim + 6) float32 tensors, plus index
        [B, 3] = (slot, t, j) with ``return_index``.  Asynchronous."""
        torch = _torch()
        B = int(batch_size)
        d = self.obs_dim + 6
        dev = self.venv.device
        out = dict(obs=torch.empty((B, d), dtype=torch.float32, device=dev),
                   action=torch.empty((B, 6), dtype=torch.float32, device=dev),
                   reward=torch.empty(B, dtype=torch.float32, device=dev),
                   next_obs=torch.empty((B, d), dtype=torch.float32, device=dev),
                   done=torch.empty(B, dtype=torch.float32, device=dev))
        idx = torch.empty((B, 3), dtype=torch.int32, device=dev) if return_index else None
        hb = _abi.CtrHerBatch()
        p = _abi.ptr
        hb.obs, hb.action, hb.reward, hb.next_obs, hb.done, hb.index = (p(out["obs"]), p(out["action"]),
                                                                        p(out["reward"]), p(out["next_obs"]),
                                                                        p(out["done"]), p(idx))
        s = (self.seed ^ 0x5DEECE66D) if seed is None else int(seed)
        rc = self.lib.ctr_her_sample(self._h, B, s & 0xFFFFFFFFFFFFFFFF, self._counter, hb, _abi.stream_ptr(stream, self.venv.device.index))
        _abi.check(rc, "ctr_her_sample")
        self._counter += 1
        if return_index:
            out["index"] = idx
        return out
