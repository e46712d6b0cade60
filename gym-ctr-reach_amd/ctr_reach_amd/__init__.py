"""ctr_reach_amd -- MI355X-native batched concentric-tube-robot reach environment.

Drop-in for keshaviyengar/gym-ctr-reach's ``CTR-Reach-v0`` hot path (FK + step + reset),
with the environments stepped in lockstep by hand-written HIP kernels on gfx950.

  CtrReachVecEnv   N envs on one GPU, torch device tensors, one kernel launch per step
  CtrReachEnv      single-env facade with the reference's gym.GoalEnv surface
  Model            batched Model.forward_kinematics operator
  make             make('CTR-Reach-v0', **overrides)
  HerReplayBuffer  device HER replay feed (stable-baselines 2 'future' relabelling)
"""
from .vec_env import CtrReachVecEnv  # noqa: F401
from .env import CtrReachEnv, Model, make  # noqa: F401
from .systems import Tube, default_kwargs, default_systems_parameters  # noqa: F401
from .goal_tolerance import GoalTolerance  # noqa: F401
from .ik import dls_ik_position_only  # noqa: F401
from .her import HerReplayBuffer  # noqa: F401
