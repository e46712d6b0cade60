#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the UNMODIFIED reference.

Runs ONLY in the authoring container (it imports /root/reference, which does not exist
on the GPU box).  The committed .npz files are data (inputs and expected outputs); the
reference's source never leaves /root/reference.

Two local compatibility layers are needed to import the reference offline (both are
outside the reference's arithmetic):

* ``gym`` is absent from the image, so a minimal stand-in module is registered in
  ``sys.modules`` providing what the reference touches: ``GoalEnv`` (empty base class),
  ``spaces.Box`` / ``spaces.Dict`` with gym-0.15 semantics (low/high cast to ``dtype``,
  float32 by default; ``sample`` = ``uniform(low, high).astype(dtype)``) and
  ``envs.registration.register`` (which records the kwargs so the registration defaults
  of ``ctr_reach_envs/__init__.py:4-96`` are taken from the reference itself).
* ``envs/model.py:107`` builds a ragged array (scalar ``uz[0]`` next to shape-(1,)
  ``uy[0]``) that numpy >= 1.24 rejects.  The module-global ``np`` of
  ``ctr_reach_envs.envs.model`` is replaced by a proxy whose ``array()`` retries with
  size-1 arrays turned into scalars -- exactly what numpy < 1.24 did implicitly.

Outputs (all seeded, deterministic):
  fk_random.npz   joints f32[n,6], system i32[n] -> tip f64[n,3], nfev i32[n]
  fk_edge.npz     hand-built edge cases (ties, limits, |alpha| >> pi, reversed spans)
  step_single.npz env.step() fixtures, select_systems=[0]   (13-float observation)
  step_multi.npz  env.step() fixtures, select_systems=[0..3] (14-float observation)
  csv_known.npz   rows of saved_policies/**/evaluations*.csv (the reference's own
                  recorded FK outputs) with a per-row flag for whether today's reference
                  reproduces them to 1e-12
  systems.json    the registration tube tables (ctr_reach_envs/__init__.py:7-70)
  sampler.npz     Obs.sample_goal draws per system (joints f32[4,n,6], candidates tried i32[4,n])
  eval_info.npz   evaluation=True env.step() info dicts over short episodes from the reference's
                  own reset() (select_systems [1, 3])

Usage:  python tests/golden/make_golden.py  [--quick]
"""
import argparse
import glob
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- gym stand-in
def _install_gym_stub():
    gym = types.ModuleType("gym")
    spaces = types.ModuleType("gym.spaces")
    envs = types.ModuleType("gym.envs")
    registration = types.ModuleType("gym.envs.registration")
    registry = {}

    class GoalEnv(object):
        pass

    class Box(object):
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            low = np.asarray(low)
            high = np.asarray(high)
            if shape is None:
                shape = np.broadcast(low, high).shape
            self.shape = tuple(shape)
            self.low = np.broadcast_to(low, self.shape).astype(self.dtype)
            self.high = np.broadcast_to(high, self.shape).astype(self.dtype)
            self.np_random = np.random.RandomState()

        def sample(self):
            s = self.np_random.uniform(low=self.low, high=self.high, size=self.shape)
            return s.astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

    class Dict(object):
        def __init__(self, d):
            self.spaces = dict(d)

    def register(id, entry_point=None, kwargs=None, max_episode_steps=None, **kw):
        registry[id] = dict(entry_point=entry_point, kwargs=kwargs, max_episode_steps=max_episode_steps)

    spaces.Box, spaces.Dict = Box, Dict
    registration.register = register
    registration.registry = registry
    envs.registration = registration
    gym.GoalEnv, gym.spaces, gym.envs = GoalEnv, spaces, envs
    sys.modules.update({"gym": gym, "gym.spaces": spaces, "gym.envs": envs,
                        "gym.envs.registration": registration})
    # ctr_3d_graph imports matplotlib 3-D tooling; render is out of scope -> stub it
    g3 = types.ModuleType("ctr_reach_envs.envs.ctr_3d_graph")
    g3.Ctr3dGraph = object
    sys.modules["ctr_reach_envs.envs.ctr_3d_graph"] = g3
    return registry


class _NumpyRaggedProxy(object):
    """numpy with the pre-1.24 ragged-array behaviour for model.py:107 only."""

    def __getattr__(self, name):
        return getattr(np, name)

    @staticmethod
    def array(obj, *a, **k):
        try:
            return np.array(obj, *a, **k)
        except ValueError:
            def fix(v):
                if isinstance(v, (tuple, list)):
                    return type(v)(fix(x) for x in v)
                if isinstance(v, np.ndarray) and v.size == 1:
                    return v.reshape(()).item()
                return v
            return np.array(fix(obj), *a, **k)


def load_reference():
    registry = _install_gym_stub()
    sys.path.insert(0, REF)
    import ctr_reach_envs  # noqa: F401  (runs register(); kwargs captured by the stub)
    import ctr_reach_envs.envs.model as model_mod
    model_mod.np = _NumpyRaggedProxy()
    from ctr_reach_envs.envs.ctr_reach_env import CtrReachEnv
    kwargs = registry["CTR-Reach-v0"]["kwargs"]
    return CtrReachEnv, kwargs


def make_env(CtrReachEnv, kwargs, **over):
    kw = dict(kwargs)
    kw.update(over)
    return CtrReachEnv(**kw)


def counted_fk(env, joints, system):
    """Reference FK with the number of RHS evaluations (ode_eq calls) recorded."""
    model = env.model
    cls_ode = type(model).ode_eq
    count = [0]

    def ode(s, y, ux, uy, ei, gj):
        count[0] += 1
        return cls_ode(model, s, y, ux, uy, ei, gj)

    model.ode_eq = ode
    try:
        tip = model.forward_kinematics(joints, system)
    finally:
        del model.ode_eq
    return np.asarray(tip, dtype=np.float64), count[0]


def tube_lengths(kwargs, sys_id):
    p = kwargs["ctr_systems_parameters"]["ctr_%d" % sys_id]
    return [p["tube_%d" % i]["length"] for i in range(3)]


def sample_valid_joints(rng, L, n, alpha_range=np.pi):
    """Rejection sampling of the reference's sample_goal region (obs.py:185-207)."""
    out = []
    low = np.array([-L[0] + 1e-3, -L[1] + 1e-3, -L[2] + 1e-3], dtype=np.float32)
    while len(out) < n:
        b = rng.uniform(low.astype(np.float64), 0.0).astype(np.float32)
        ok = all(b[i - 1] <= b[i] and b[i - 1] + np.float32(L[i - 1]) >= np.float32(L[i]) + b[i]
                 for i in (1, 2))
        if ok:
            a = rng.uniform(-alpha_range, alpha_range, 3).astype(np.float32)
            out.append(np.concatenate([b, a]))
    return np.array(out, dtype=np.float32)


def gen_fk_random(CtrReachEnv, kwargs, per_sys):
    env = make_env(CtrReachEnv, kwargs, select_systems=[0, 1, 2, 3])
    rng = np.random.default_rng(1234)
    J, S, T, NF = [], [], [], []
    for s in range(4):
        L = tube_lengths(kwargs, s)
        j1 = sample_valid_joints(rng, L, per_sys)
        j2 = sample_valid_joints(rng, L, per_sys // 4, alpha_range=40.0)  # long rotations
        for q in np.concatenate([j1, j2]):
            tip, nf = counted_fk(env, q, s)
            J.append(q); S.append(s); T.append(tip); NF.append(nf)
    np.savez_compressed(os.path.join(OUT, "fk_random.npz"), joints=np.array(J, np.float32),
                        system=np.array(S, np.int32), tip=np.array(T), nfev=np.array(NF, np.int32))
    print("fk_random", len(J))


def tiny_first_segment_cases(L, Lc, s, want=6):
    """Search joints whose first breakpoint S[0] is below 1e-6 using the reference Segment."""
    from ctr_reach_envs.envs.CTR_Python.Segment import Segment
    from ctr_reach_envs.envs.CTR_Python.Tube import Tube
    tubes = [Tube(L[i], Lc[i], 1e-3, 2e-3, 1.0, 1.0, 1.0, 0.0) for i in range(3)]
    found, rng = [], np.random.default_rng(11 + s)
    for trial in range(20000):
        i = int(rng.integers(3))
        eps = float(rng.uniform(-2e-5, 4e-5))
        b = np.array([-0.6 * L[0], -0.5 * L[1], -0.4 * L[2]]) * rng.uniform(0.2, 1.0, 3)
        if rng.random() < 0.5:
            b[i] = Lc[i] - L[i] + eps          # curve-start point near s = 0
        else:
            b[i] = -L[i] + eps                 # tip near s = 0
        q = np.concatenate([b, rng.uniform(-np.pi, np.pi, 3)]).astype(np.float32)
        beta = q[:3] + np.zeros(3, dtype=np.int64)
        try:
            seg = Segment(tubes[0], tubes[1], tubes[2], beta)
        except Exception:
            continue
        if seg.S.size and seg.S[0] < 1.2e-6:
            found.append(q)
            if len(found) >= want:
                break
    return found


def edge_joints(kwargs, s):
    L = np.array(tube_lengths(kwargs, s))
    p = kwargs["ctr_systems_parameters"]["ctr_%d" % s]
    Lc = np.array([p["tube_%d" % i]["length_curved"] for i in range(3)])
    lo = -L + 1e-3
    cases = []
    f = np.float32
    cases.append([0, 0, 0, 0, 0, 0])                                  # fully extended
    cases.append([lo[0], lo[1], lo[2], 0.1, -0.2, 0.3])               # per-tube lower limit
    cases.append([lo[0], lo[0], lo[0], 1, 2, 3])                      # all bases equal
    b2 = -0.01
    b1 = b2 + L[2] - L[1]                                             # tip of tube1 == tip of tube2
    b0 = b1 + L[1] - L[0]                                             # tip of tube0 == tip of tube1
    cases.append([max(b0, lo[0]), max(b1, lo[1]), b2, 0.5, 0.5, 0.5])
    cases.append([max(b1, lo[0]), max(b1, lo[1]), b2, -3, 3, -3])
    # curve start of tube 1 coincides with base plane (d_c == 0)
    bc = -(L[1] - Lc[1])
    cases.append([max(bc - 0.01, lo[0]), bc, 0.0, 0.2, 0.4, 0.6])
    # tiny first segment: a breakpoint lands just above s = 0 after the 10 um floor
    # quantisation, so the first span [0, S0 - 1e-6] is reversed or zero (model.py:141-148)
    cases.extend(tiny_first_segment_cases(L, Lc, s))
    # rotations far outside [-pi, pi] (constrain_alpha=False lets them grow)
    cases.append([-0.05, -0.04, -0.03, 50.0, -60.0, 70.0])
    cases.append([-0.05, -0.04, -0.03, 123.4, 123.4, 123.4])
    cases.append([-0.05, -0.04, -0.03, np.pi, -np.pi, np.pi])
    # identical alphas (no relative twist) and opposite
    cases.append([-0.1, -0.08, -0.02, 0.0, 0.0, 0.0])
    cases.append([-0.1, -0.08, -0.02, 0.0, np.pi, 0.0])
    cases = [c for c in cases if c is not None]
    return np.array(cases, dtype=np.float64).astype(f)


def gen_fk_edge(CtrReachEnv, kwargs):
    env = make_env(CtrReachEnv, kwargs, select_systems=[0, 1, 2, 3])
    J, S, T, NF = [], [], [], []
    for s in range(4):
        for q in edge_joints(kwargs, s):
            tip, nf = counted_fk(env, q, s)
            J.append(q); S.append(s); T.append(tip); NF.append(nf)
    np.savez_compressed(os.path.join(OUT, "fk_edge.npz"), joints=np.array(J, np.float32),
                        system=np.array(S, np.int32), tip=np.array(T), nfev=np.array(NF, np.int32))
    print("fk_edge", len(J))


def gen_step(CtrReachEnv, kwargs, name, select, n, constrain_alpha_list=(False, True)):
    rng = np.random.default_rng(99 + len(select))
    rows = {k: [] for k in ("joints_in", "action", "system", "desired_goal", "t_in", "tol",
                            "constrain_alpha", "joints_out", "achieved_goal", "observation",
                            "reward", "done", "is_success", "error")}
    for ca in constrain_alpha_list:
        env = make_env(CtrReachEnv, kwargs, select_systems=list(select), constrain_alpha=ca)
        alim = env.action_space.high
        for k in range(n):
            sidx = int(rng.integers(len(select)))
            L = tube_lengths(kwargs, select[sidx])
            q = sample_valid_joints(rng, L, 1)[0]
            mode = k % 4
            if mode == 1:        # push against the extension limits / nesting constraints
                a = np.concatenate([rng.choice([-1, 1], 3) * alim[:3], rng.uniform(-1, 1, 3) * alim[3:]])
            elif mode == 2:      # alphas near +-pi (clip when constrain_alpha)
                q[3:] = (rng.choice([-1, 1], 3) * (np.pi - rng.uniform(0, 0.05, 3))).astype(np.float32)
                a = rng.uniform(-1, 1, 6) * alim
            else:
                a = rng.uniform(-1, 1, 6) * alim
            a = a.astype(np.float32)
            tol = float(rng.choice([0.02, 0.005, 0.001]))
            t_in = int(rng.choice([0, 5, 148, 149]))
            # desired goal: FK of other valid joints, or near the current tip (to hit success)
            if k % 3 == 0:
                dg, _ = counted_fk(env, sample_valid_joints(rng, L, 1)[0], sidx)
            else:
                tip0, _ = counted_fk(env, q, sidx)
                dg = tip0 + rng.normal(0, 0.004, 3)
            env.reset()                       # consumes the env's RNG; then overwrite state
            env.system = sidx
            env.trig_obj.joints = q.copy()
            env.desired_goal = np.asarray(dg, np.float64)
            env.t = t_in
            env.goal_tolerance.current_tol = tol
            obs, reward, done, info = env.step(a)
            rows["joints_in"].append(q); rows["action"].append(a); rows["system"].append(sidx)
            rows["desired_goal"].append(dg); rows["t_in"].append(t_in); rows["tol"].append(tol)
            rows["constrain_alpha"].append(ca)
            rows["joints_out"].append(np.asarray(env.trig_obj.joints))
            rows["achieved_goal"].append(obs["achieved_goal"]); rows["observation"].append(obs["observation"])
            rows["reward"].append(float(reward)); rows["done"].append(bool(done))
            rows["is_success"].append(bool(info["is_success"])); rows["error"].append(float(info["error"]))
    out = {k: np.array(v) for k, v in rows.items()}
    out["joints_in"] = out["joints_in"].astype(np.float32)
    out["action"] = out["action"].astype(np.float32)
    out["select_systems"] = np.array(select, np.int32)
    out["joints_out_dtype_f32"] = np.array(out["joints_out"].dtype == np.float32)
    np.savez_compressed(os.path.join(OUT, name), **out)
    print(name, len(out["reward"]), "joints_out dtype", out["joints_out"].dtype)


def gen_csv_known(CtrReachEnv, kwargs, rows_per_file):
    env = make_env(CtrReachEnv, kwargs, select_systems=[0, 1, 2, 3])
    files = sorted(glob.glob(os.path.join(REF, "ctr_reach_envs/saved_policies/**/evaluations*.csv"),
                             recursive=True))
    rng = np.random.default_rng(7)
    J, S, T, REFT, FILE = [], [], [], [], []
    import pandas as pd
    for fi, f in enumerate(files):
        df = pd.read_csv(f)
        idx = rng.choice(len(df), size=min(rows_per_file, len(df)), replace=False)
        for r in idx:
            row = df.iloc[r]
            s = int(row["system_id"])
            for kind, goal in (("desired", "desired_goal"), ("achieved", "achieved_goal"),
                               ("starting", "starting_position")):
                q = np.array([row["B_%s_%d" % (kind, i)] for i in (1, 2, 3)] +
                             [row["alpha_%s_%d" % (kind, i)] for i in (1, 2, 3)]).astype(np.float32)
                pre = goal + "_" if goal != "starting_position" else "starting_position_"
                tip_csv = np.array([row[pre + c] for c in "xyz"], np.float64)
                tip_ref, _ = counted_fk(env, q, s)
                J.append(q); S.append(s); T.append(tip_csv); REFT.append(tip_ref); FILE.append(fi)
    T = np.array(T); REFT = np.array(REFT)
    dev = np.linalg.norm(T - REFT, axis=1)
    np.savez_compressed(os.path.join(OUT, "csv_known.npz"), joints=np.array(J, np.float32),
                        system=np.array(S, np.int32), tip_csv=T, tip_reference=REFT, reference_reproduces=dev <= 1e-12,
                        reference_dev=dev, file_index=np.array(FILE, np.int32),
                        files=np.array([os.path.relpath(f, REF) for f in files]))
    print("csv_known", len(J), "reproduced<=1e-12:", int((dev <= 1e-12).sum()), "max dev", dev.max())


def gen_jacobian(CtrReachEnv, kwargs, per_sys, eps=1e-4):
    """Forward-difference tip Jacobian of the reference FK over float64 joints, the scheme of
    CTR_Model.jac (CTR_Python/CTR_Model.py:251-262) applied to Model.forward_kinematics."""
    env = make_env(CtrReachEnv, kwargs, select_systems=[0, 1, 2, 3])
    rng = np.random.default_rng(4321)
    Q, S, T, JAC = [], [], [], []
    for s in range(4):
        L = tube_lengths(kwargs, s)
        for q32 in sample_valid_joints(rng, L, per_sys):
            q = q32.astype(np.float64)
            # keep the perturbed extensions inside the region (b_i + eps <= 0)
            q[:3] = np.minimum(q[:3], -2 * eps)
            r0 = np.asarray(env.model.forward_kinematics(q, s), np.float64)
            jac = np.zeros((3, 6))
            for i in range(6):
                qp = q.copy()
                qp[i] = q[i] + eps
                jac[:, i] = (np.asarray(env.model.forward_kinematics(qp, s), np.float64) - r0) / eps
            Q.append(q); S.append(s); T.append(r0); JAC.append(jac)
    np.savez_compressed(os.path.join(OUT, "jacobian.npz"), joints=np.array(Q), system=np.array(S, np.int32),
                        tip=np.array(T), jac=np.array(JAC), eps=eps)
    print("jacobian", len(Q))


def gen_backbone(CtrReachEnv, kwargs, per_sys, max_pts=270):
    """Backbone shape model.r (30 t_eval points per segment, RK45 dense output) with the tube
    tip indices of ctr_model (model.py:119-174) and the r1/r2/r3 slices (model.py:66-68)."""
    env = make_env(CtrReachEnv, kwargs, select_systems=[0, 1, 2, 3])
    model = env.model
    rng = np.random.default_rng(777)
    cls_ctr = type(model).ctr_model
    cap = {}

    def ctr_model(*a, **k):
        out = cls_ctr(model, *a, **k)
        cap["tip_idx"] = np.asarray(out[2], np.int64)
        return out

    Q, S, R, NPT, TIPI, TIP = [], [], [], [], [], []
    for s in range(4):
        L = tube_lengths(kwargs, s)
        qs = list(sample_valid_joints(rng, L, per_sys)) + list(edge_joints(kwargs, s)[:4])
        for q in qs:
            model.ctr_model = ctr_model
            try:
                tip = model.forward_kinematics(np.asarray(q, np.float32), s)
            finally:
                del model.ctr_model
            r = np.asarray(model.r, np.float64)
            assert len(r) <= max_pts
            pad = np.full((max_pts, 3), np.nan)
            pad[:len(r)] = r
            Q.append(np.asarray(q, np.float32)); S.append(s); R.append(pad); NPT.append(len(r))
            TIPI.append(cap["tip_idx"]); TIP.append(np.asarray(tip, np.float64))
    R = np.array(R)[:, :max(NPT)]
    np.savez_compressed(os.path.join(OUT, "backbone.npz"), joints=np.array(Q), system=np.array(S, np.int32),
                        r=R, n_points=np.array(NPT, np.int32), tip_idx=np.array(TIPI, np.int64),
                        tip=np.array(TIP))
    print("backbone", len(Q), "max points", max(NPT))


def gen_sampler(CtrReachEnv, kwargs, per_sys):
    """Obs.sample_goal (obs.py:185-207) draws of the reference: the sampled joints and the number
    of candidates each took (the reference's own numpy RNG, seeded per system)."""
    env = make_env(CtrReachEnv, kwargs, select_systems=[0, 1, 2, 3])
    J, T = [], []
    for s in range(4):
        box = env.trig_obj.joint_sample_spaces[s]
        box.np_random = np.random.RandomState(1234 + s)
        calls = [0]
        orig = box.sample

        def counting_sample(orig=orig):
            calls[0] += 1
            return orig()

        box.sample = counting_sample
        js, ts = [], []
        for _ in range(per_sys):
            calls[0] = 0
            js.append(np.asarray(env.trig_obj.sample_goal(s), np.float32))
            ts.append(calls[0])
        box.sample = orig
        J.append(js)
        T.append(ts)
    np.savez_compressed(os.path.join(OUT, "sampler.npz"), joints=np.array(J, np.float32), tries=np.array(T, np.int32))


def gen_eval(CtrReachEnv, kwargs, episodes, steps):
    """env.step() with evaluation=True (ctr_reach_env.py:144-153): the info dict the reference's
    evaluation runs record (errors_pos, q_desired, q_achieved, q_starting, starting_position,
    system_idx, ...), over short episodes.  select_systems [1, 3], so system_idx (the
    registration index) differs from the episode's system (an index into select_systems).
    Each episode starts from the reference's own reset() (np.random seeded per episode)."""
    env = make_env(CtrReachEnv, kwargs, select_systems=[1, 3], evaluation=True, constrain_alpha=False)
    alim = env.action_space.high
    rng = np.random.default_rng(2024)
    keys_vec = ("achieved_goal", "desired_goal", "starting_position", "q_desired", "q_achieved", "q_starting")
    keys_sc = ("is_success", "errors_pos", "errors_orient", "system_idx", "position_tolerance",
               "orientation_tolerance")
    rows = {k: [] for k in keys_vec + keys_sc + ("episode", "t", "action", "reward", "done", "observation",
                                                 "tol")}
    resets = {k: [] for k in ("system", "desired_joints", "desired_goal", "starting_joints", "starting_position",
                              "observation")}
    for ep in range(episodes):
        np.random.seed(500 + ep)
        tol = float(rng.choice([0.02, 0.005]))
        env.goal_tolerance.current_tol = tol
        obs0 = env.reset()
        resets["system"].append(int(env.system))
        resets["desired_joints"].append(np.asarray(env.desired_joints, np.float32))
        resets["desired_goal"].append(np.asarray(env.desired_goal, np.float64))
        resets["starting_joints"].append(np.asarray(env.starting_joints, np.float32))
        resets["starting_position"].append(np.asarray(env.starting_position, np.float64))
        resets["observation"].append(np.asarray(obs0["observation"], np.float64))
        for t in range(steps):
            a = (rng.uniform(-1, 1, 6) * alim).astype(np.float32)
            obs, reward, done, info = env.step(a)
            assert set(info) == set(keys_vec + keys_sc)
            for k in keys_vec:
                rows[k].append(np.asarray(info[k], np.float64))
            for k in keys_sc:
                rows[k].append(float(info[k]))
            rows["episode"].append(ep); rows["t"].append(t); rows["action"].append(a)
            rows["reward"].append(float(reward)); rows["done"].append(bool(done)); rows["tol"].append(tol)
            rows["observation"].append(np.asarray(obs["observation"], np.float64))
            if done:
                break
    out = {k: np.array(v) for k, v in rows.items()}
    out.update({"reset_" + k: np.array(v) for k, v in resets.items()})
    out["select_systems"] = np.array([1, 3], np.int32)
    np.savez_compressed(os.path.join(OUT, "eval_info.npz"), **out)
    print("eval_info", episodes, "episodes", len(out["t"]), "steps")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", nargs="*", help="generate only these fixtures (jacobian, backbone)")
    args = ap.parse_args()
    CtrReachEnv, kwargs = load_reference()
    if args.only:
        if "jacobian" in args.only:
            gen_jacobian(CtrReachEnv, kwargs, 4 if args.quick else 32)
        if "backbone" in args.only:
            gen_backbone(CtrReachEnv, kwargs, 4 if args.quick else 16)
        if "sampler" in args.only:
            gen_sampler(CtrReachEnv, kwargs, 400 if args.quick else 4000)
        if "eval" in args.only:
            gen_eval(CtrReachEnv, kwargs, 4 if args.quick else 24, 12)
        return
    sysj = {}
    for s in range(4):
        p = kwargs["ctr_systems_parameters"]["ctr_%d" % s]
        sysj["ctr_%d" % s] = {t: dict(p[t]) for t in sorted(p)}
    defaults = {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in kwargs.items()
                if k != "ctr_systems_parameters"}
    with open(os.path.join(OUT, "systems.json"), "w") as fh:
        json.dump({"ctr_systems_parameters": sysj, "defaults": defaults}, fh, indent=1, sort_keys=True)
    per = 16 if args.quick else 192
    gen_fk_random(CtrReachEnv, kwargs, per)
    gen_fk_edge(CtrReachEnv, kwargs)
    gen_step(CtrReachEnv, kwargs, "step_single.npz", [0], 8 if args.quick else 96)
    gen_step(CtrReachEnv, kwargs, "step_multi.npz", [0, 1, 2, 3], 8 if args.quick else 96)
    gen_csv_known(CtrReachEnv, kwargs, 2 if args.quick else 25)
    gen_jacobian(CtrReachEnv, kwargs, 4 if args.quick else 32)
    gen_backbone(CtrReachEnv, kwargs, 4 if args.quick else 16)
    gen_sampler(CtrReachEnv, kwargs, 400 if args.quick else 4000)
    gen_eval(CtrReachEnv, kwargs, 4 if args.quick else 24, 12)


if __name__ == "__main__":
    main()
