"""CtrReachVecEnv -- N concentric-tube-robot reach environments stepped in lockstep on one GPU.

Host side of the hot path.  State lives in device tensors (PyTorch is only the allocator and
stream provider); every step is ONE call into libctr_reach_amd.so (ctr_step), which enqueues
the fused step kernel (+ the compacted auto-reset kernel) on the current stream and returns
without synchronising.

Semantics per environment follow CtrReachEnv (envs/ctr_reach_env.py:13-210):
  * step        = n_substeps x Obs.set_action, forward kinematics, compute_reward,
                  done = reward == 0 or t >= max_steps, get_obs                  (:124-158)
  * reset       = system pick, sample_goal -> FK (desired goal), sample_goal -> FK (start)
                                                                                  (:70-114)
  * auto-reset  = VecEnv convention: a done environment is reset inside the same step call;
                  the returned observation is the new episode's, the terminal observation and
                  achieved goal are returned in ``info``.
Random draws come from a Philox4x32-10 stream keyed by (seed, global env id, reset number),
so results do not depend on how environments are sharded over GPUs.
"""
import numpy as np

from . import _abi
from . import distributed as D
from .goal_tolerance import GoalTolerance
from .spaces import Box, Dict
from .systems import default_kwargs, make_config, solver_codes, tubes_from_params

NUM_TUBES = 3
EXT_TOL = 1e-3    # obs.py:14
ZERO_TOL = 1e-4   # obs.py:16
RK4_REFILL_BUDGET = 32   # resumable refill, fixed-step RK4: RK4 steps per reset FK and refill


def _torch():
    import torch
    return torch


def _current_stream(stream, device):
    import torch
    return stream if stream is not None else torch.cuda.current_stream(device)


def joint_spaces(systems, constrain_alpha):
    """Obs.get_joint_space (obs.py:50-76): per-system (joint_space, joint_sample_space)."""
    js, jss = [], []
    for tubes in systems:
        L = np.array([t.L for t in tubes])
        jss.append(Box(low=np.concatenate((-L + EXT_TOL, np.full(NUM_TUBES, -np.pi))),
                       high=np.concatenate((np.full(NUM_TUBES, 0), np.full(NUM_TUBES, np.pi)))))
        lim = np.pi if constrain_alpha else np.inf
        js.append(Box(low=np.concatenate((-L + EXT_TOL, np.full(NUM_TUBES, -lim))),
                      high=np.concatenate((np.full(NUM_TUBES, 0), np.full(NUM_TUBES, lim)))))
    return js, jss


def observation_space(systems, goal_tolerance):
    """Obs.get_observation_space (obs.py:78-134)."""
    max_len = np.amax(np.array([[t.L for t in tubes] for tubes in systems]), axis=0)
    rep_low, rep_high = [], []
    for L in max_len:
        rep_low += [-1, -1, -L + ZERO_TOL]
        rep_high += [1, 1, 0]
    rep = Box(low=np.array(rep_low), high=np.array(rep_high), dtype="float32")
    if len(systems) == 1:
        lo = np.concatenate((rep.low, np.array([-0.2, -0.2, -0.2, goal_tolerance.final_tol])))
        hi = np.concatenate((rep.high, np.array([0.2, 0.2, 0.2, goal_tolerance.init_tol])))
    else:
        lo = np.concatenate((rep.low, np.array([-0.2, -0.2, -0.2, goal_tolerance.final_tol, 0])))
        hi = np.concatenate((rep.high, np.array([0.2, 0.2, 0.2, goal_tolerance.init_tol, len(systems) - 1])))
    return Dict(dict(
        desired_goal=Box(low=np.array([-0.1, -0.1, 0]), high=np.array([0.1, 0.1, 0.2]), dtype="float32"),
        achieved_goal=Box(low=np.array([-0.1, -0.1, 0]), high=np.array([0.1, 0.1, 0.2]), dtype="float32"),
        observation=Box(low=lo, high=hi, dtype="float32")))


def action_space(extension_action_limit, rotation_action_limit):
    """CtrReachEnv.__init__ :58-62."""
    b = np.full(NUM_TUBES, extension_action_limit)
    a = np.full(NUM_TUBES, np.deg2rad(rotation_action_limit))
    return Box(low=np.concatenate((-b, -a)), high=np.concatenate((b, a)), dtype="float32")


class CtrReachVecEnv(object):
    """Batched CTR-Reach on one GPU.  Constructor kwargs = the reference's (ctr_reach_env.py:14-17)
    plus ``num_envs``, ``device``, ``seed``, ``env_base`` (global id of env 0 for sharding),
    ``autoreset``.  Missing reference kwargs take the CTR-Reach-v0 registration defaults.

    Solver kwargs (build-specific): ``integrator`` "rk45_scipy" (default; the
    reference's solve_ivp RK45, bit-for-bit in its step sequence) or "rk4" (fixed step,
    ``rk4_steps_per_m`` equal steps per metre of each segment); ``model`` "compliant" (the
    reference's torsionally-compliant ODE, model.py:72-117) or "rigid" (GJ -> infinity).

    ``obs_dtype``: "float32" (default: what a trainer consumes) or "float64" (the reference's
    dtype, obs.py:153-156).  The observation is computed in float64 either way; float32 stores it
    rounded once.  The HER feed records float32 observations."""

    def __init__(self, num_envs, device="cuda", seed=0, env_base=0, autoreset=True, record_info=True,
                 pool_depth=None, refill_interval=64, integrator="rk45_scipy", rk4_steps_per_m=100,
                 model="compliant", pack_outputs=False, obs_dtype="float32", refill_budget=None, **kwargs):
        torch = _torch()
        kw = default_kwargs()
        kw.update(kwargs)
        if kw.get("length_based_sample"):
            raise NotImplementedError("length_based_sample: the reference branch is broken "
                                      "(reads the nonexistent self.system_parameters, ctr_reach_env.py:88)")
        assert kw["joint_representation"] in ("egocentric", "proprioceptive")
        self.kwargs = kw
        self.integrator, self.rk4_steps_per_m, self.model = integrator, int(rk4_steps_per_m), model
        solver = solver_codes(integrator, rk4_steps_per_m, model)
        self.lib = _abi.load()
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        self.env_base = int(env_base)
        self.autoreset = bool(autoreset)
        all_systems = tubes_from_params(kw["ctr_systems_parameters"])
        self.select_systems = list(kw["select_systems"])
        self.ctr_system_parameters = [all_systems[s] for s in self.select_systems]
        self.n_systems = len(self.ctr_system_parameters)
        self.goal_tolerance = GoalTolerance(kw["goal_tolerance_parameters"])
        self.max_steps_per_episode = kw["max_steps_per_episode"]
        self.n_substeps = kw["n_substeps"]
        self.constrain_alpha = kw["constrain_alpha"]
        self.joint_representation = kw["joint_representation"]
        self.resample_joints = kw["resample_joints"]
        self.evaluation = kw["evaluation"]
        self.noise_parameters = kw["noise_parameters"]   # stored, never applied (reference Q11)
        self.joint_spaces, self.joint_sample_spaces = joint_spaces(self.ctr_system_parameters, self.constrain_alpha)
        self.observation_space = observation_space(self.ctr_system_parameters, self.goal_tolerance)
        self.action_space = action_space(kw["extension_action_limit"], kw["rotation_action_limit"])
        self.obs_dim = 13 if self.n_systems == 1 else 14
        self.seed_value = int(seed)
        self.cfg = make_config(self.ctr_system_parameters, n_substeps=self.n_substeps,
                               max_steps=self.max_steps_per_episode, constrain_alpha=self.constrain_alpha,
                               egocentric=self.joint_representation == "egocentric",
                               resample_joints=self.resample_joints, tol=self.goal_tolerance.get_tol(),
                               seed=self.seed_value, integrator=solver[0], rk4_steps_per_m=solver[1],
                               model=solver[2], domain_rand=kw.get("domain_rand", 0.0))
        if obs_dtype not in ("float32", "float64", torch.float32, torch.float64):
            raise ValueError("obs_dtype must be float32 or float64")
        self.obs_dtype = torch.float64 if obs_dtype in ("float64", torch.float64) else torch.float32
        self.cfg.obs_f64 = int(self.obs_dtype == torch.float64)
        n, dev = self.num_envs, self.device
        f32, f64, i32 = torch.float32, torch.float64, torch.int32
        init = np.asarray(kw["initial_joints"], dtype=np.float64)
        self.joints = torch.tensor(np.tile(init, (n, 1)), dtype=f32, device=dev)
        self.desired_goal = torch.zeros((n, 3), dtype=f64, device=dev)
        self.achieved_goal = torch.zeros((n, 3), dtype=f64, device=dev)
        self.t = torch.zeros(n, dtype=i32, device=dev)
        self.system = torch.zeros(n, dtype=i32, device=dev)
        self.epoch = torch.zeros(n, dtype=i32, device=dev)
        self.work = torch.zeros(n + 2, dtype=i32, device=dev)
        self.desired_joints = torch.zeros((n, 6), dtype=f32, device=dev) if record_info else None
        self.starting_joints = torch.zeros((n, 6), dtype=f32, device=dev) if record_info else None
        self.starting_position = torch.zeros((n, 3), dtype=f64, device=dev) if record_info else None
        # outputs (persistent; step() returns views of these buffers)
        self.obs = torch.zeros((n, self.obs_dim), dtype=self.obs_dtype, device=dev)
        self.reward = torch.zeros(n, dtype=f32, device=dev)
        self.done = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.success = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.error = torch.zeros(n, dtype=f32, device=dev)
        self.terminal_obs = torch.zeros((n, self.obs_dim), dtype=self.obs_dtype, device=dev)
        self.terminal_achieved = torch.zeros((n, 3), dtype=f64, device=dev)
        self.status = torch.zeros(n, dtype=i32, device=dev)
        self.nfev = None
        # pack_outputs: k_step also writes each step's gather row ([n, 4] f32, distributed.PACK_WIDTH)
        # into one of two alternating buffers, so gather_outputs() needs no packing launch and one
        # gather may stay in flight while the next step writes the other buffer
        # (row n: the step's sequence word, for the copy-engine gather; see gather_outputs)
        self.packed_bufs = [torch.zeros((n + 1, D.PACK_WIDTH), dtype=f32, device=dev) for _ in range(2)] if pack_outputs else None
        self._packed_k = 0
        self.packed_seq = 0       # steps that wrote packed rows (the sequence word of the last one)
        self._push_gather = None  # distributed.PushGather (enable_gather)
        self.gather_seq = 0       # fused push: the last step pushed
        self.refills = 0          # ctr_pool_refill launches so far (bench accounting)
        self.sweeps = 0           # steps that launched the auto-reset miss sweep (CTR_AUTORESET_SWEEP)
        # reset pool: resets are a pure function of (seed, env id, reset number), so they are
        # precomputed in batches every `refill_interval` steps and consumed by a copy
        # depth >= the refill interval: every env then finds its next reset in the pool on every
        # step (CTR_AUTORESET_POOLED, no miss-sweep launch); 128 B per env and slot
        # resumable refill (scipy RK45, and fixed-step RK4 on the compliant model): a reset at least
        # one refill period ahead of its env runs at most refill_budget iterations (RK45 attempts,
        # RK4 steps) of each FK per refill; an unfinished one is
        # suspended and resumed (bit-identically) by the next refill, so a refill lasts about as
        # long as the budget instead of its slowest fresh sample's FK (ctr_batch_t.carry).  The
        # resets less than a period ahead always finish: none is due before it lands
        R = max(1, int(refill_interval))
        # the kernel's rule (ctr_kernels.hip refill_resumable): every mode but the rigid model's
        # fixed-step RK4, whose FKs run as segment maps on 8-lane groups
        resumable = not (integrator == "rk4" and model == "rigid")
        if refill_budget is None:
            refill_budget = (6 if integrator == "rk45_scipy" else RK4_REFILL_BUDGET) if resumable else 0
        if refill_budget and not resumable:
            raise ValueError("refill_budget is not available for the rigid model's fixed-step RK4 (its FKs run as "
                             "segment maps)")
        if pool_depth is None:
            # deep enough for the budget to apply over about two refills (queued resets are
            # P - R - 1 or more ahead); 64 slots cap the default ring (128 B per env and slot).
            # Deeper rings (up to CTR_POOL_MAX) work but measured slower: at R = 64 a 152-slot
            # ring with the budget ran the 128-step window at 78.4 against 78.0 us/step
            want = 2 * R + 24 if refill_budget else R
            pool_depth = max(8, min(64, want)) if (self.autoreset and self.resample_joints) else 0
        if pool_depth and not self.resample_joints:
            raise ValueError("the reset pool needs resample_joints=True")
        self.pool_depth = int(pool_depth)
        self.refill_interval = R
        # a reset queued in a period is at least P - R - 1 ahead at the refill: budgeted if P > 2R
        self.refill_budget = int(refill_budget) if (self.pool_depth > 2 * R) else 0
        self.refill_lead = R
        self._steps_since_refill = 0
        # True once a refill has followed a full (re)queue of every env and every refill period
        # since has taken at most pool_depth steps (pool_depth >= refill_interval)
        self._pool_full = False
        P = self.pool_depth
        if P:
            # [P][n] 128-B slots (ctr_pool_slot_t): a pooled reset reads one cache line.  The
            # per-field names are strided views of it (pool_r [P, n], pool_dg [P, n, 3], ...)
            self.pool = torch.zeros((P, n, _abi.POOL_SLOT_DWORDS), dtype=i32, device=dev)
            if self.pool.data_ptr() % 128:
                raise RuntimeError("reset pool not 128-B aligned")
            dt = {"f64": f64, "f32": f32}
            for k, (a, b_, kind) in _abi.POOL_SLOT_FIELDS.items():
                v = self.pool[..., a] if b_ is None else self.pool[..., a:b_].view(dt[kind])
                setattr(self, "pool_" + k, v)
            self.refill_cap = n * (P + self.refill_interval)
            self.refill = torch.zeros(2 + 2 * self.refill_cap, dtype=i32, device=dev)   # count, pairs, ticket
        else:
            self.pool = self.pool_qd = self.pool_dg = self.pool_q0 = self.pool_ag = None
            self.pool_sys = self.pool_r = self.pool_stat = self.refill = None
            self.refill_cap = 0
        self.carry, self.carry_cap = None, 0
        if P and self.refill_budget:
            # a steady-state period queues ~15 % of the envs (R = 20, 150-step episodes); a queue
            # longer than the list (reset(), requeue) runs without the budget.  640 B per reset
            self.carry_cap = max(256, 2 * n)
            nb = int(self.lib.ctr_refill_carry_bytes(self.carry_cap))
            self.carry = torch.zeros((nb + 15) // 16 * 16, dtype=torch.uint8, device=dev)
        self._batch = _abi.CtrBatch()
        self._out = _abi.CtrStepOut()
        self._her = None          # HerReplayBuffer bound by enable_her()
        self._fill_structs()

    # ------------------------------------------------------------------ plumbing
    def _fill_structs(self):
        p = _abi.ptr
        b = self._batch
        b.n, b.env_base = self.num_envs, self.env_base
        b.joints, b.desired_goal, b.achieved_goal = p(self.joints), p(self.desired_goal), p(self.achieved_goal)
        b.t, b.system, b.epoch, b.work = p(self.t), p(self.system), p(self.epoch), p(self.work)
        b.desired_joints, b.starting_joints = p(self.desired_joints), p(self.starting_joints)
        b.starting_position = p(self.starting_position)
        b.pool_depth = self.pool_depth
        b.pool = p(self.pool)
        b.refill, b.refill_cap = p(self.refill), self.refill_cap
        b.carry, b.carry_cap = p(self.carry), self.carry_cap
        b.refill_budget, b.refill_lead = self.refill_budget, self.refill_lead
        o = self._out
        o.obs, o.reward, o.done, o.success, o.error = (p(self.obs), p(self.reward), p(self.done), p(self.success),
                                                        p(self.error))
        o.terminal_obs, o.terminal_achieved, o.status = p(self.terminal_obs), p(self.terminal_achieved), p(self.status)
        o.nfev = p(self.nfev)
        o.packed = p(self.packed_bufs[self._packed_k]) if self.packed_bufs is not None else None

    def enable_nfev(self, on=True):
        """Record per-env RHS evaluation counts of the last step (diagnostics / roofline)."""
        torch = _torch()
        self.nfev = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device) if on else None
        self._fill_structs()

    def enable_her(self, slots=4, n_sampled_goal=4, goal_selection_strategy="future", seed=None):
        """Bind a device HER replay feed (ctr_reach_amd.her.HerReplayBuffer): every later reset /
        step records into it.  Call before reset()."""
        from .her import HerReplayBuffer
        return HerReplayBuffer(self, slots=slots, n_sampled_goal=n_sampled_goal,
                               goal_selection_strategy=goal_selection_strategy, seed=seed)

    def _obs_dict(self):
        return {"observation": self.obs, "achieved_goal": self.achieved_goal, "desired_goal": self.desired_goal}

    # ------------------------------------------------------------------ gym surface
    def seed(self, seed=None):
        if seed is not None:
            self.seed_value = int(seed)
            self.cfg.seed = self.seed_value & 0xFFFFFFFFFFFFFFFF
            if self.pool_depth:
                self.pool_r.zero_()          # precomputed resets belong to the old seed
                self._requeue_pool()
        return [self.seed_value]

    def _requeue_pool(self, stream=None):
        """Drop the refill queue and queue every env's next pool_depth resets the pool does not
        hold (ctr_pool_requeue), then refill: after a seed change or a checkpoint restore."""
        self.refill[0] = 0
        # (the requeue also empties the refill's suspended lists: it queues their resets again)
        rc = self.lib.ctr_pool_requeue(self.cfg, self._batch, _abi.stream_ptr(stream))
        _abi.check(rc, "ctr_pool_requeue")
        self._steps_since_refill = 0
        self.refill_pool(stream)
        self._pool_full = self._pooled_steps() >= self.refill_interval

    def _pooled_steps(self):
        # steps after a refill for which every env's next resets are in the pool: pool_depth, or
        # with the resumable refill the resets less than refill_lead ahead (the ones it finishes)
        return min(self.pool_depth, self.refill_lead) if self.carry is not None else self.pool_depth

    def carried(self):
        """Resets on the two suspended lists (resumable refill; diagnostics, synchronises)."""
        if self.carry is None:
            return (0, 0)
        c = self.carry[:512].view(_torch().int32).view(2, 64).sum(dim=1).tolist()   # CarryHdr.count[2][64]
        return (c[0], c[1])

    def refill_pool(self, stream=None):
        """Precompute the queued resets into the pool (ctr_pool_refill); asynchronous."""
        if self.pool_depth:
            rc = self.lib.ctr_pool_refill(self.cfg, self._batch, _abi.stream_ptr(stream))
            _abi.check(rc, "ctr_pool_refill")
            self.refills += 1
            if self._steps_since_refill > self._pooled_steps():
                self._pool_full = False      # a period longer than the pool: misses were swept
        self._steps_since_refill = 0

    def reset(self, goal=None, system=None, mask=None, stream=None):
        """CtrReachEnv.reset for all envs (or those with mask != 0).  goal: [N,3] f64 tensor or
        None (sample); system: [N] int tensor or None (uniform).  Returns the obs dict."""
        torch = _torch()
        self.cfg.tol = float(self.goal_tolerance.get_tol())
        g = None if goal is None else torch.as_tensor(goal, dtype=torch.float64, device=self.device).reshape(-1, 3).contiguous()
        s = None if system is None else torch.as_tensor(system, dtype=torch.int32, device=self.device).reshape(-1).contiguous()
        m = None if mask is None else torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        if g is not None and g.shape[0] == 1 and self.num_envs > 1:
            g = g.expand(self.num_envs, 3).contiguous()
        if s is not None and s.shape[0] == 1 and self.num_envs > 1:
            s = s.expand(self.num_envs).contiguous()
        if s is not None:
            bad = (s < 0) | (s >= self.n_systems)
            if bool(bad.any()):
                raise ValueError("system index out of range")
        self._keep = (g, s, m)   # keep alive until the kernel has consumed them
        if self.pool_depth and m is None:
            self.refill[0] = 0   # every env is reset and requeued: older queue entries are moot
        rc = self.lib.ctr_reset(self.cfg, self._batch, _abi.ptr(m), _abi.ptr(g), _abi.ptr(s), _abi.ptr(self.obs),
                                _abi.ptr(self.status), _abi.stream_ptr(stream))
        _abi.check(rc, "ctr_reset")
        if self._her is not None:
            self._her._open(m, stream)
        if self.pool_depth:
            # ctr_reset queued the P resets after each reset env's new one; a masked reset keeps
            # the other envs' pools (the refill below also takes their queued entries)
            steps = self._steps_since_refill
            self.refill_pool(stream)
            if m is None:
                self._pool_full = self._pooled_steps() >= self.refill_interval
            elif steps > self._pooled_steps():
                self._pool_full = False
        else:
            self._steps_since_refill = 0
        return self._obs_dict()

    def step(self, actions, stream=None):
        """One step of every env.  actions: [N,6] float32 device tensor.  Returns
        (obs dict, reward [N] f32, done [N] bool, info dict of tensors).  Returned tensors are
        views of persistent buffers, overwritten by the next call."""
        torch = _torch()
        if actions.dtype != torch.float32 or actions.device != self.device or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=torch.float32).contiguous()
        if actions.shape != (self.num_envs, 6):
            raise ValueError("actions must be [%d, 6]" % self.num_envs)
        self.cfg.tol = float(self.goal_tolerance.get_tol())
        self._last_actions = actions
        self.step_raw(actions, stream)
        info = {"is_success": self.success.bool(), "error": self.error,
                "terminal_observation": self.terminal_obs, "terminal_achieved_goal": self.terminal_achieved,
                "status": self.status}
        return self._obs_dict(), self.reward, self.done.bool(), info

    def step_raw(self, actions, stream=None):
        """step() without building Python return values (benchmark / graph capture)."""
        sp = _abi.stream_ptr(stream, self.device.index)
        her = self._her
        pb = self.packed_bufs
        if pb is not None:                     # this step writes the buffer the last gather did not
            self._packed_k ^= 1
            self._out.packed = pb[self._packed_k].data_ptr()
            # never 0 (no sequence row) and parity-preserving at the uint32 wrap (done events by parity)
            self.packed_seq = self.packed_seq + 1 if self.packed_seq < 0xFFFFFFFF else 2
            self._out.packed_seq = self.packed_seq
            if self._push_gather is not None:    # the copy engines have read this buffer's last rows
                self._push_gather.wait_pushed(self._packed_k, _current_stream(stream, self.device))
        g = self._push_gather
        fused = g is not None and g.engine == "fused"
        if fused:                              # this step also stores its rows into every rank's ring
            self.gather_seq += 1               # a Python int (slot = seq % depth); modulo 2^32 on the device
            cur, prev, prev_seq = g.step_args(self.gather_seq)
            o = self._out
            o.gather, o.gather_prev, o.gather_prev_seq = cur, prev, prev_seq & 0xFFFFFFFF
            o.gather_seq, o.gather_wait_prev = self.gather_seq & 0xFFFFFFFF, 1 if g.wait_prev else 0
        mode = _abi.AUTORESET_OFF
        if self.autoreset:
            # no done env can miss its pooled reset while at most pool_depth steps have run since
            # a refill that left every env's next pool_depth resets precomputed (one reset per env
            # and step): no miss-sweep launch then.  With pool_depth >= refill_interval that holds
            # on every step once reset() (or a requeue) has filled the pool.
            if self._pool_full and self._steps_since_refill < self._pooled_steps():
                mode = _abi.AUTORESET_POOLED
            else:
                mode = _abi.AUTORESET_SWEEP
                self.sweeps += 1
        if her is not None and her.fused:      # the step records itself into the HER store (ctr_step_her)
            rc = self.lib.ctr_step_her(self.cfg, self._batch, _abi.ptr(actions), self._out, mode, her._h, sp)
        else:
            rc = self.lib.ctr_step(self.cfg, self._batch, _abi.ptr(actions), self._out, mode, sp)
        if fused:
            o.gather = o.gather_prev = None    # only this launch pushes (other ctr_step users of _out do not)
            o.gather_wait_prev = 0
            if rc == 0:
                g.stepped(self.gather_seq)
        if rc:
            _abi.check(rc, "ctr_step")
        if her is not None and not her.fused:  # ctr_her_record from the step's outputs
            her._record(actions, stream)
        if self.autoreset:
            self._batch.work_parity ^= 1
        if self.pool_depth:
            self._steps_since_refill += 1
            if self._steps_since_refill >= self.refill_interval:
                self.refill_pool(stream)

    def capture_steps(self, actions, stream=None):
        """Capture len(actions) consecutive steps (step_raw, with the pool refills that fall due)
        into one HIP graph; ``StepGraph.replay()`` then runs them with a single launch, so a
        launch-bound batch (configs[1]: 4 096 envs, ~10 us kernels) is not paced by the host.

        The host side of a step (buffer parities, the refill schedule, the auto-reset mode) is
        fixed in the graph, so the sequence must bring it back to where it started: start right
        after a refill, a multiple of refill_interval steps, an even number of steps, the pool
        full (no miss sweeps).  Not with HER or the push gather (their sequence numbers change every
        step).  The goal tolerance and the action buffers are captured: re-capture after
        update_goal_tolerance, and write new actions into the captured buffers."""
        return StepGraph(self, actions, stream)

    def compute_reward(self, achieved_goal, desired_goal, info=None):
        """compute_reward (ctr_reach_env.py:160-170), batched over leading dims.  Device tensors
        run on the GPU (HER relabelling); numpy arrays follow the reference exactly."""
        torch = _torch()
        tol = float(self.goal_tolerance.get_tol())
        if isinstance(achieved_goal, torch.Tensor):
            assert achieved_goal.shape == desired_goal.shape
            shape = achieved_goal.shape[:-1]
            ag = achieved_goal.to(self.device, torch.float64).reshape(-1, 3).contiguous()
            dg = desired_goal.to(self.device, torch.float64).reshape(-1, 3).contiguous()
            out = torch.empty(ag.shape[0], dtype=torch.float32, device=self.device)
            rc = self.lib.ctr_compute_reward(_abi.ptr(ag), _abi.ptr(dg), ag.shape[0], tol, _abi.ptr(out),
                                             _abi.stream_ptr())
            _abi.check(rc, "ctr_compute_reward")
            return out.reshape(shape)
        achieved_goal = np.asarray(achieved_goal)
        desired_goal = np.asarray(desired_goal)
        assert achieved_goal.shape == desired_goal.shape
        d = np.linalg.norm(achieved_goal - desired_goal, axis=-1)
        return -(d > tol).astype(np.float64)

    def forward_kinematics(self, joints, system=None, stream=None, return_stats=False, tables=None):
        """Batched Model.forward_kinematics (model.py:30): joints [M,6] -> tip [M,3] f64 (device).
        ``system`` picks rows of the nominal tube tables; ``tables`` (a [M, 18] float64 device tensor
        in ctr_system_t order, e.g. ``domain_parameters()["table"]``) gives every row its own."""
        torch = _torch()
        q = torch.as_tensor(joints, dtype=torch.float32, device=self.device).reshape(-1, 6).contiguous()
        m = q.shape[0]
        s = None if system is None else torch.as_tensor(system, dtype=torch.int32, device=self.device).reshape(-1).expand(m).contiguous()
        tip = torch.empty((m, 3), dtype=torch.float64, device=self.device)
        stats = torch.zeros((m, 4), dtype=torch.int32, device=self.device) if return_stats else None
        status = torch.zeros(m, dtype=torch.int32, device=self.device)
        if tables is not None:
            tb = torch.as_tensor(tables, dtype=torch.float64, device=self.device).reshape(m, 18).contiguous()
            rc = self.lib.ctr_fk_tables(_abi.ptr(q), _abi.ptr(tb), m, self.cfg, _abi.ptr(tip), _abi.ptr(stats),
                                        _abi.ptr(status), _abi.stream_ptr(stream))
            _abi.check(rc, "ctr_fk_tables")
        else:
            rc = self.lib.ctr_fk(_abi.ptr(q), _abi.ptr(s), m, self.cfg, _abi.ptr(tip), _abi.ptr(stats),
                                 _abi.ptr(status), _abi.stream_ptr(stream))
            _abi.check(rc, "ctr_fk")
        if return_stats:
            if self.integrator == "rk4":
                # ctr_fk packs stats[2] for fixed-step RK4 (include/ctr_reach_amd.h): the segments run
                # as segment maps << 16 | their square-and-multiply compositions; RK4 rejects nothing.
                # nstep counts the RK4 steps taken stage by stage (nfev: 4 per step, mapped or not)
                packed = stats[:, 2]
                return tip, dict(nfev=stats[:, 0], nstep=stats[:, 1], nrej=torch.zeros_like(packed),
                                 maps=packed >> 16, compositions=packed & 0xFFFF, nseg=stats[:, 3], status=status)
            return tip, dict(nfev=stats[:, 0], nstep=stats[:, 1], nrej=stats[:, 2], nseg=stats[:, 3], status=status)
        return tip

    def forward_kinematics_shape(self, joints, system=None, tables=None, stream=None, cap=270):
        """Model.forward_kinematics with the backbone shape (model.py:66-68, 119-174) for joints
        [M, 6]: dict of device tensors tip [M, 3], r [M, cap, 3] and s [M, cap] (valid up to
        npts [M] = 30 x segments; the rest is NaN), status [M]."""
        torch = _torch()
        q = torch.as_tensor(joints, dtype=torch.float32, device=self.device).reshape(-1, 6).contiguous()
        m = q.shape[0]
        s = None if system is None else torch.as_tensor(system, dtype=torch.int32, device=self.device).reshape(-1).expand(m).contiguous()
        tb = None
        if tables is not None:
            tb = torch.as_tensor(tables, dtype=torch.float64, device=self.device).reshape(m, 18).contiguous()
        tip = torch.empty((m, 3), dtype=torch.float64, device=self.device)
        r = torch.full((m, cap, 3), float("nan"), dtype=torch.float64, device=self.device)
        sv = torch.full((m, cap), float("nan"), dtype=torch.float64, device=self.device)
        npts = torch.zeros(m, dtype=torch.int32, device=self.device)
        status = torch.zeros(m, dtype=torch.int32, device=self.device)
        rc = self.lib.ctr_fk_shape(_abi.ptr(q), _abi.ptr(s), _abi.ptr(tb), m, self.cfg, int(cap), _abi.ptr(tip),
                                   _abi.ptr(r), _abi.ptr(sv), _abi.ptr(npts), _abi.ptr(status), _abi.stream_ptr(stream))
        _abi.check(rc, "ctr_fk_shape")
        return dict(tip=tip, r=r, s=sv, npts=npts, status=status)

    def jacobian(self, joints, system=None, eps=1e-4, stream=None):
        """Forward-difference tip Jacobian (CTR_Model.jac scheme, CTR_Python/CTR_Model.py:251-262)
        of this env's FK over float64 joints [M, 6] -> (tip [M, 3], jac [M, 3, 6]) float64 (device)."""
        torch = _torch()
        q = torch.as_tensor(joints, dtype=torch.float64, device=self.device).reshape(-1, 6).contiguous()
        m = q.shape[0]
        s = None if system is None else torch.as_tensor(system, dtype=torch.int32, device=self.device).reshape(-1).expand(m).contiguous()
        tip = torch.empty((m, 3), dtype=torch.float64, device=self.device)
        jac = torch.empty((m, 3, 6), dtype=torch.float64, device=self.device)
        rc = self.lib.ctr_jacobian(_abi.ptr(q), _abi.ptr(s), m, self.cfg, float(eps), _abi.ptr(tip), _abi.ptr(jac),
                                   None, _abi.stream_ptr(stream))
        _abi.check(rc, "ctr_jacobian")
        return tip, jac

    def domain_parameters(self, stream=None):
        """Each env's current tube table (Model.current_sys_parameters after randomize_parameters,
        model.py:20-28): dict of [n, 3] float64 device tensors L, L_c, EI, GJ, U_x, U_y,
        diameter_inner, diameter_outer, E, G, plus "table" ([n, 18], the ctr_system_t rows the FK
        integrates with).  Without domain randomisation these are the nominal rows."""
        torch = _torch()
        n = self.num_envs
        table = torch.empty((n, 18), dtype=torch.float64, device=self.device)
        raw = torch.empty((n, 12), dtype=torch.float64, device=self.device)
        rc = self.lib.ctr_domain_params(self.cfg, self._batch, _abi.ptr(table), _abi.ptr(raw), _abi.stream_ptr(stream))
        _abi.check(rc, "ctr_domain_params")
        out = {k: table[:, 3 * i:3 * i + 3] for i, k in enumerate(("L", "L_c", "EI", "GJ", "U_x", "U_y"))}
        out.update({k: raw[:, 3 * i:3 * i + 3] for i, k in enumerate(("diameter_inner", "diameter_outer", "E", "G"))})
        out["table"] = table
        return out

    def enable_gather(self, backend="push", group=None, depth=3, wait_prev=False, wait_us=10_000_000):
        """Set up the push all-gather (collective: every rank calls it).  "push": every later
        step also stores its packed rows into every rank's receive ring (the fused push; no
        extra launch), paced by the ranks' slot releases: the gathered view of step s stays valid
        until this env launches step s + depth - 1; with ``wait_prev`` every step also waits until
        the previous step's rows of every rank are in this rank's ring (depth >= 3).  "sdma":
        gather_outputs(backend="sdma") copies them with the copy engines (needs
        pack_outputs=True; the caller paces the ranks).  ``wait_us`` is the wall-clock budget of every
        device-side wait, in microseconds (default 10 s: a rank may pause that long between steps
        -- checkpointing, evaluation -- before its peers' waits give up; raise it for longer
        pauses); a wait that gives up sets a CTR_GATHER_E_* bit in the gather's error word instead
        of hanging.  A producer that overruns a slot this rank has not released also flags it here
        (poison words): ``err_bits()`` read after a view's readers have run covers that view.
        Returns the distributed.PushGather."""
        if self._push_gather is not None:
            raise RuntimeError("the gather is already enabled")
        if backend == "sdma" and self.packed_bufs is None:
            raise RuntimeError("the sdma gather needs CtrReachVecEnv(..., pack_outputs=True)")
        if backend not in ("push", "sdma"):
            raise ValueError("backend must be 'push' or 'sdma'")
        self._push_gather = D.PushGather(self.num_envs, group=group, depth=depth, device=self.device,
                                         engine="fused" if backend == "push" else "sdma",
                                         wait_prev=wait_prev and backend == "push", wait_us=wait_us)
        return self._push_gather

    def gather_outputs(self, group=None, async_op=False, backend="rccl", depth=3):
        """Optional collective for a single-process trainer: every rank's last-step (tip, reward,
        done, success) packed to 16 B/env and all-gathered -> [world * n, 4] float32 in global-id
        order.  Not used on the stepping path.  async_op=True returns (out, work) and lets the
        next step() run while the gather is in flight; the pack buffers alternate, so one gather
        may be outstanding per env.

        backend "rccl": all_gather_into_tensor over RCCL (its own stream).  backend "push" (after
        enable_gather("push"): the last step already stored its rows into every rank's ring) or
        "sdma" (copy engines, needs pack_outputs=True; set up on first use, collectively): this
        rank's rows land in every rank's IPC-mapped receive ring (distributed.PushGather); ``out``
        is slot (step % depth) of this rank's ring, valid after ``work.wait()`` (which enqueues
        the wait for every rank's block on the current stream) until this env launches step +
        depth - 1 (push: the step kernels pace the ranks by their slot releases; sdma: the caller
        paces them).

        With ``pack_outputs=True`` the step kernel itself wrote the packed rows (no packing
        launch); otherwise they are packed here from the step's outputs."""
        import torch
        if backend in ("push", "sdma"):
            if self._push_gather is None:
                if backend == "push":
                    raise RuntimeError("the fused push gather is part of the step: call enable_gather('push') "
                                       "before stepping")
                self.enable_gather("sdma", group=group, depth=depth)
            g = self._push_gather
            if (g.engine == "fused") != (backend == "push"):
                raise RuntimeError("this env gathers with the %s engine" % g.engine)
            if g.engine == "fused":
                seq = self.gather_seq              # pushed by the last step itself
            else:
                ready = self._gather_ready = getattr(self, "_gather_ready", None) or torch.cuda.Event()
                ready.record(torch.cuda.current_stream(self.device))
                seq = self.packed_seq
                g.push(self.packed_bufs[self._packed_k], seq, ready, parity=self._packed_k)
            work = D.PushWork(g, seq)
            if async_op:
                return g.recv[seq % g.depth].reshape(-1, D.PACK_WIDTH), work
            return work.wait()
        if backend != "rccl":
            raise ValueError("backend must be 'rccl', 'push' or 'sdma'")
        if self.packed_bufs is not None:
            return D.all_gather_outputs(self.packed_bufs[self._packed_k][:self.num_envs], group=group,
                                        async_op=async_op)
        d = self.done.bool()
        tip = torch.where(d[:, None], self.terminal_achieved, self.achieved_goal) if self.autoreset else self.achieved_goal
        bufs = getattr(self, "_packed", None) or [None, None]
        k = self._packed_k
        bufs[k] = D.pack_step_outputs(tip, self.reward, d, self.success, out=bufs[k])
        self._packed, self._packed_k = bufs, k ^ 1
        return D.all_gather_outputs(bufs[k], group=group, async_op=async_op)

    def packed_outputs(self):
        """The last step's packed rows ([n, 4] float32, see gather_outputs); needs pack_outputs=True."""
        if self.packed_bufs is None:
            raise RuntimeError("packed_outputs() needs CtrReachVecEnv(..., pack_outputs=True)")
        return self.packed_bufs[self._packed_k][:self.num_envs]

    def update_goal_tolerance(self, timestep):
        self.goal_tolerance.update(timestep)

    def get_goal_tolerance(self):
        return self.goal_tolerance.get_tol()

    # ------------------------------------------------------------------ checkpoint
    _STATE_KEYS = ("joints", "desired_goal", "achieved_goal", "t", "system", "epoch", "obs")

    def state_dict(self):
        sd = {k: getattr(self, k).clone() for k in self._STATE_KEYS}
        sd["seed"] = self.seed_value
        sd["tol"] = self.goal_tolerance.get_tol()
        return sd

    def load_state_dict(self, sd):
        """Restore the batch state.  The reset pool is re-keyed to the restored reset numbers
        (queue dropped, next pool_depth resets requeued and refilled), the auto-reset miss
        counters are cleared, and a bound HER store drops its open episodes and opens new ones
        from the restored state (the finished episodes it holds stay sampleable).

        Every key of ``state_dict()`` is required: a checkpoint without the observation (or any
        other state buffer) would leave part of the live state from before the restore."""
        missing = [k for k in self._STATE_KEYS + ("seed", "tol") if k not in sd]
        if missing:
            raise KeyError("checkpoint lacks %s (saved by an older build?)" % ", ".join(missing))
        for k in self._STATE_KEYS:
            getattr(self, k).copy_(sd[k])
        self.goal_tolerance.current_tol = sd["tol"]
        self.cfg.tol = float(sd["tol"])
        self.work.zero_()
        self._batch.work_parity = 0
        seed_changed = int(sd["seed"]) != self.seed_value
        self.seed_value = int(sd["seed"])
        self.cfg.seed = self.seed_value & 0xFFFFFFFFFFFFFFFF
        if self.pool_depth:
            if seed_changed:
                # the ring's resets were drawn with the old seed: a slot whose reset number
                # matches a restored epoch + j would otherwise be kept (requeue and refill only
                # compare reset numbers)
                self.pool_r.zero_()
            self._requeue_pool()
        if self._her is not None:
            self._her._open(None, None)

    def close(self):
        pass


class StepGraph(object):
    """A captured sequence of CtrReachVecEnv steps (CtrReachVecEnv.capture_steps)."""

    def __init__(self, env, actions, stream=None):
        torch = _torch()
        k = len(actions)
        if env._her is not None or env._push_gather is not None:
            raise RuntimeError("capture_steps: not with the HER feed or the push gather")
        if env.autoreset and env.pool_depth:
            if k % env.refill_interval or env._steps_since_refill != 0 or not env._pool_full:
                raise RuntimeError("capture_steps: start right after a refill with a full pool and capture a "
                                   "multiple of refill_interval (%d) steps" % env.refill_interval)
        elif env.autoreset:
            raise RuntimeError("capture_steps: auto-reset needs the reset pool")
        if k % 2:
            raise RuntimeError("capture_steps: an even number of steps (buffer parities)")
        self.env, self.steps = env, k
        self.actions = [a for a in actions]
        self.stream = stream if stream is not None else torch.cuda.Stream(device=env.device)
        self.stream.wait_stream(torch.cuda.current_stream(env.device))
        refills, sweeps, seq = env.refills, env.sweeps, env.packed_seq
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=self.stream):
            for a in self.actions:
                env.step_raw(a, self.stream)
        self.refills_per_replay = env.refills - refills
        # the capture launched nothing: its host bookkeeping is undone, replay() redoes it
        env.refills, env.sweeps, env.packed_seq = refills, sweeps, seq
        assert env._steps_since_refill == 0 or not env.pool_depth

    def replay(self):
        """Run the captured steps (stream-ordered on the current stream, like step())."""
        self.graph.replay()
        self.env.refills += self.refills_per_replay
        if self.env.packed_bufs is not None:
            self.env.packed_seq += self.steps
