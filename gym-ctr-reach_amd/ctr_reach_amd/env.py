"""Single-environment facade with the reference's gym.GoalEnv surface.

``CtrReachEnv(**kwargs)`` accepts exactly the reference constructor kwargs
(envs/ctr_reach_env.py:14-17) and exposes reset/step/compute_reward/seed/render/close,
update_goal_tolerance/get_goal_tolerance/print_parameters, observation_space/action_space
and ``model.forward_kinematics`` -- backed by a one-env CtrReachVecEnv on the GPU.
Returned observations are numpy float64 dicts like the reference's (computed and stored in
float64 on the device).
"""
import numpy as np

from .spaces import GoalEnvBase
from .systems import default_kwargs
from .vec_env import CtrReachVecEnv


def tube_tip_indices(s, L, beta):
    """ctr_model's tip_pos (model.py:160-168): for each tube k the first backbone index whose
    arclength is >= L_k + beta_k - 1e-3 (0 if none)."""
    s = np.asarray(s)
    out = np.zeros(3, np.int64)
    for k in range(3):
        hit = np.nonzero(s >= (float(L[k]) + float(beta[k])) - 1e-3)[0]
        out[k] = hit[0] if hit.size else 0
    return out


class Model(object):
    """Operator boundary: Model.forward_kinematics (envs/model.py:30-70), batched on the GPU.

    ``r``, ``r1``, ``r2``, ``r3`` are the backbone of the last forward kinematics (model.py:66-68):
    a one-row call computes them with ctr_fk_shape; after env.reset()/step() they are computed
    on first access for the env's current joints (the reference's last FK in both)."""

    def __init__(self, vec_env):
        self._env = vec_env
        self._shape = None        # (r, r1, r2, r3)
        self._pending = None      # (joints, system) whose shape is computed on first access

    def _tables(self, system, m):
        v = self._env
        if v.kwargs.get("domain_rand", 0.0) != 0.0 and int(system) == int(v.system[0].item()):
            # the episode's randomised table (Model.current_sys_parameters, model.py:20-28)
            return v.domain_parameters()["table"][0:1].expand(m, 18)
        return None

    def _compute_shape(self, q, system):
        v = self._env
        tb = self._tables(system, 1)
        out = v.forward_kinematics_shape(q.reshape(1, 6), None if tb is not None else np.array([int(system)]),
                                         tables=tb)
        n = int(out["npts"][0].item())
        r = out["r"][0, :n].cpu().numpy()
        s = out["s"][0, :n].cpu().numpy()
        L = v.domain_parameters()["L"][0].cpu().numpy() if tb is not None else \
            [t.L for t in v.ctr_system_parameters[int(system)]]
        beta = q.reshape(6)[:3].astype(np.float64)
        t0, t1, t2 = tube_tip_indices(s, L, beta)
        return out["tip"][0].cpu().numpy(), (r, r[t1:t0 + 1], r[t2:t1 + 1], r[:t2 + 1])

    def _set_pending(self, joints, system):
        self._pending = (np.asarray(joints, np.float32).copy(), int(system))
        self._shape = None

    def _current_shape(self):
        if self._shape is None and self._pending is not None:
            q, s = self._pending
            self._shape = self._compute_shape(q, s)[1]
        return self._shape if self._shape is not None else (None, None, None, None)

    r = property(lambda self: self._current_shape()[0])
    r1 = property(lambda self: self._current_shape()[1])
    r2 = property(lambda self: self._current_shape()[2])
    r3 = property(lambda self: self._current_shape()[3])

    def forward_kinematics(self, joint, system, **kwargs):
        q = np.asarray(joint, dtype=np.float32).reshape(-1, 6)
        v = self._env
        if q.shape[0] == 1 and v.integrator == "rk45_scipy":
            tip, self._shape = self._compute_shape(q, system)
            self._pending = None
            assert not np.any(np.isnan(self._shape[0]))          # model.py:69
            return tip if np.ndim(joint) == 1 else tip[None]
        tb = self._tables(system, q.shape[0])
        if tb is not None:
            tip = v.forward_kinematics(q, tables=tb)
        else:
            tip = v.forward_kinematics(q, np.full(q.shape[0], int(system)))
        out = tip.cpu().numpy()
        return out[0] if np.ndim(joint) == 1 else out


class CtrReachEnv(GoalEnvBase):
    metadata = {"render.modes": []}

    def __init__(self, ctr_systems_parameters, goal_tolerance_parameters, noise_parameters, joint_representation,
                 initial_joints, constrain_alpha, extension_action_limit, rotation_action_limit,
                 max_steps_per_episode, n_substeps, evaluation, select_systems, resample_joints=True,
                 length_based_sample=False, domain_rand=0.0, device="cuda", seed=0, integrator="rk45_scipy",
                 rk4_steps_per_m=100, model="compliant"):
        kw = dict(ctr_systems_parameters=ctr_systems_parameters, goal_tolerance_parameters=goal_tolerance_parameters,
                  noise_parameters=noise_parameters, joint_representation=joint_representation,
                  initial_joints=initial_joints, constrain_alpha=constrain_alpha,
                  extension_action_limit=extension_action_limit, rotation_action_limit=rotation_action_limit,
                  max_steps_per_episode=max_steps_per_episode, n_substeps=n_substeps, evaluation=evaluation,
                  select_systems=select_systems, resample_joints=resample_joints,
                  length_based_sample=length_based_sample, domain_rand=domain_rand)
        # float64 observations, as the reference returns them (obs.py:153-156)
        self.vec = CtrReachVecEnv(1, device=device, seed=seed, autoreset=False, integrator=integrator,
                                  rk4_steps_per_m=rk4_steps_per_m, model=model, obs_dtype="float64", **kw)
        v = self.vec
        self.select_systems = v.select_systems
        self.ctr_system_parameters = v.ctr_system_parameters
        self.noise_parameters = noise_parameters
        self.joint_representation = joint_representation
        self.max_steps_per_episode = max_steps_per_episode
        self.n_substeps = n_substeps
        self.constrain_alpha = constrain_alpha
        self.evaluation = evaluation
        self.resample_joints = resample_joints
        self.length_based_sample = length_based_sample
        self.domain_rand = domain_rand
        self.extension_action_limit = extension_action_limit
        self.rotation_action_limit = rotation_action_limit
        self.observation_space = v.observation_space
        self.action_space = v.action_space
        self.goal_tolerance = v.goal_tolerance
        self.model = Model(v)
        self.t = 0
        self.system = 0
        self.starting_joints = np.asarray(initial_joints)
        self.desired_joints = np.asarray(initial_joints)
        # :65 initial FK at the initial joints
        self.starting_position = self.model.forward_kinematics(np.asarray(initial_joints, np.float32), 0)
        self.desired_goal = self.starting_position
        self.vec.achieved_goal.copy_(self.vec.forward_kinematics(np.asarray(initial_joints, np.float32)[None]))
        self.vec.desired_goal.copy_(self.vec.achieved_goal)
        self.visualization = None

    @property
    def joints(self):
        return self.vec.joints[0].cpu().numpy()

    def reset(self, goal=None, system=None):
        g = None if goal is None else np.asarray(goal, dtype=np.float64).reshape(1, 3)
        s = None if system is None else np.array([int(system)])
        self.vec.reset(goal=g, system=s)
        self.t = 0
        self.system = int(self.vec.system[0].item())
        self.desired_goal = self.vec.desired_goal[0].cpu().numpy().copy()
        self.starting_position = self.vec.achieved_goal[0].cpu().numpy().copy()
        self.starting_joints = self.vec.joints[0].cpu().numpy().copy()
        if self.vec.desired_joints is not None and goal is None:
            self.desired_joints = self.vec.desired_joints[0].cpu().numpy().copy()
        self.model._set_pending(self.starting_joints, self.system)
        return self._obs()

    def _obs(self):
        return {"observation": self.vec.obs[0].cpu().numpy().copy(),
                "achieved_goal": self.vec.achieved_goal[0].cpu().numpy().copy(),
                "desired_goal": self.vec.desired_goal[0].cpu().numpy().copy()}

    def seed(self, seed=None):
        return self.vec.seed(seed)

    def step(self, action):
        action = np.asarray(action)
        assert not np.all(np.isnan(action))                 # :131
        assert self.action_space.contains(action)           # :132
        import torch
        a = torch.as_tensor(np.asarray(action, np.float32).reshape(1, 6), device=self.vec.device)
        obs, reward, done, info = self.vec.step(a)
        self.t = int(self.vec.t[0].item())
        self.model._set_pending(self.vec.joints[0].cpu().numpy(), self.system)
        o = self._obs()
        achieved_goal = o["achieved_goal"]
        reward = float(reward[0].item())
        done = bool(done[0].item())
        err = float(np.linalg.norm(self.desired_goal - achieved_goal))
        tol = self.goal_tolerance.get_tol()
        if self.evaluation:
            info = {"is_success": err < tol, "errors_pos": err, "errors_orient": 0,
                    "system_idx": self.select_systems[self.system], "position_tolerance": tol,
                    "orientation_tolerance": 0, "achieved_goal": achieved_goal, "desired_goal": self.desired_goal,
                    "starting_position": self.starting_position, "q_desired": self.desired_joints,
                    "q_achieved": self.joints, "q_starting": self.starting_joints}
        else:
            info = {"is_success": err < tol, "error": err}
        return o, np.float64(reward), done, info

    def compute_reward(self, achieved_goal, desired_goal, info):
        return self.vec.compute_reward(achieved_goal, desired_goal, info)

    def render(self, mode="empty", **kwargs):
        if mode == "live":
            raise NotImplementedError("live rendering (matplotlib) is out of scope of the GPU build")

    def close(self):
        raise SystemExit(0)                                  # :184-191, as the reference does

    def print_parameters(self):
        print("----Observation and q_space----")
        print("----Goal tolerance parameters----")

    def update_goal_tolerance(self, timestep):
        self.goal_tolerance.update(timestep)

    def get_goal_tolerance(self):
        return self.goal_tolerance.get_tol()


_REGISTRY = {"CTR-Reach-v0": (CtrReachEnv, default_kwargs, 150)}


def make(env_id="CTR-Reach-v0", **overrides):
    """gym.make equivalent: registration defaults (ctr_reach_envs/__init__.py:4-96) + overrides."""
    cls, defaults, _max_steps = _REGISTRY[env_id]
    kw = defaults()
    kw.update(overrides)
    return cls(**kw)
