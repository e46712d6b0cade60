"""Tube systems and registration defaults of ``CTR-Reach-v0``.

The physical constants are the four systems registered by the reference
(ctr_reach_envs/__init__.py:7-70: Khadem, Grassmann, RViM lab, unnamed); the scalar
defaults are ctr_reach_envs/__init__.py:72-93.  ``derive`` restates Tube.__init__
(envs/CTR_Python/Tube.py:7-19): I = pi (d_o^4 - d_i^4) / 64, J = 2 I, with the same
Python ``math`` arithmetic so the products EI = E * I and GJ = G * J are bit-identical.
"""
import copy
import math

import numpy as np

from . import _abi

# (length, length_curved, d_inner, d_outer, E, G, U_x, U_y) per tube, innermost first.
_SYSTEM_TABLE = {
    "ctr_0": ((431e-3, 103e-3, 0.7e-3, 1.10e-3, 10.25e+10, 18.79e+10, 21.3, 0),
              (332e-3, 113e-3, 1.4e-3, 1.8e-3, 68.6e+10, 11.53e+10, 13.1, 0),
              (174e-3, 134e-3, 2e-3, 2.4e-3, 16.96e+10, 14.25e+10, 3.5, 0)),
    "ctr_1": ((370e-3, 45e-3, 0.3e-3, 0.4e-3, 50e+10, 2.3e+10, 15.8, 0),
              (305e-3, 100e-3, 0.7e-3, 0.9e-3, 50e+10, 2.3e+10, 9.27, 0),
              (170e-3, 100e-3, 1.2e-3, 1.5e-3, 50e+10, 2.3e+10, 4.37, 0)),
    "ctr_2": ((309e-3, 145e-3, 0.7e-3, 1.1e-3, 75e+9, 25e+9, 13.52, 0),
              (275e-3, 114e-3, 1.4e-3, 1.8e-3, 75e+9, 25e+9, 11.68, 0),
              (173e-3, 173e-3, 1.83e-3, 2.39e-3, 75e+9, 25e+9, 10.8, 0)),
    "ctr_3": ((150e-3, 100e-3, 1.0e-3, 2.4e-3, 5e+10, 2.3e+10, 15.82, 0),
              (100e-3, 21.6e-3, 3.0e-3, 3.8e-3, 5e+10, 2.3e+10, 11.8, 0),
              (70e-3, 8.8e-3, 4.4e-3, 5.4e-3, 5.0e+10, 2.3e+10, 20.04, 0)),
}
_KEYS = ("length", "length_curved", "diameter_inner", "diameter_outer", "stiffness", "torsional_stiffness",
         "x_curvature", "y_curvature")


def default_systems_parameters():
    """The registration ``ctr_systems_parameters`` dict (same nesting and key names)."""
    return {name: {"tube_%d" % i: dict(zip(_KEYS, tube)) for i, tube in enumerate(tubes)}
            for name, tubes in _SYSTEM_TABLE.items()}


def default_kwargs():
    """Constructor kwargs registered for CTR-Reach-v0 (ctr_reach_envs/__init__.py:6-94)."""
    return {
        "ctr_systems_parameters": default_systems_parameters(),
        "extension_action_limit": 0.001,
        "rotation_action_limit": 5,
        "max_steps_per_episode": 150,
        "n_substeps": 10,
        "goal_tolerance_parameters": {"inc_tol_obs": False, "final_tol": 0.001, "initial_tol": 0.020,
                                      "N_ts": 200000, "function": "constant", "set_tol": 0},
        "noise_parameters": {"rotation_std": np.deg2rad(0), "extension_std": 0.001 * np.deg2rad(0),
                             "tracking_std": 0.0},
        "select_systems": [0],
        "constrain_alpha": False,
        "initial_joints": np.array([0, 0, 0, 0, 0, 0]),
        "joint_representation": "egocentric",
        "resample_joints": True,
        "evaluation": False,
        "length_based_sample": False,
        "domain_rand": 0.0,
    }


class Tube(object):
    """Tube.__init__ (envs/CTR_Python/Tube.py:7-19), same attribute names."""

    def __init__(self, length, length_curved, diameter_inner, diameter_outer, stiffness, torsional_stiffness,
                 x_curvature, y_curvature):
        self.L = length
        self.L_c = length_curved
        self.L_s = length - length_curved
        self.diameter_inner = diameter_inner
        self.diameter_outer = diameter_outer
        d4 = math.pow(diameter_outer, 4) - math.pow(diameter_inner, 4)
        self.J = (math.pi * d4) / 32
        self.I = (math.pi * d4) / 64
        self.E = stiffness
        self.G = torsional_stiffness
        self.U_x = x_curvature
        self.U_y = y_curvature


def tubes_from_params(ctr_systems_parameters):
    """List (per system, registration order) of [Tube x3] like CtrReachEnv.__init__ :20-25."""
    out = []
    for sysname in ctr_systems_parameters:
        out.append([Tube(**ctr_systems_parameters[sysname][t]) for t in ctr_systems_parameters[sysname]])
    return out


def to_ctr_system(tubes):
    s = _abi.CtrSystem()
    for i, t in enumerate(tubes):
        s.L[i] = t.L
        s.Lc[i] = t.L_c
        s.EI[i] = t.E * t.I
        s.GJ[i] = t.G * t.J
        s.Ux[i] = t.U_x
        s.Uy[i] = t.U_y
    return s


def to_ctr_tube_raw(tubes):
    """Tube.__init__ inputs that domain randomisation re-samples (model_utils.py:15-18)."""
    r = _abi.CtrTubeRaw()
    for i, t in enumerate(tubes):
        r.Din[i] = t.diameter_inner
        r.Dout[i] = t.diameter_outer
        r.E[i] = t.E
        r.G[i] = t.G
    return r


def make_config(systems, n_substeps=10, max_steps=150, constrain_alpha=False, egocentric=True,
                resample_joints=True, tol=0.020, seed=0, integrator=_abi.CTR_INTEGRATOR_RK45_SCIPY,
                rk4_steps_per_m=0, model=_abi.CTR_MODEL_COMPLIANT, domain_rand=0.0):
    """Build the ctr_env_config_t for a list of [Tube x3] systems (already filtered)."""
    if not 1 <= len(systems) <= _abi.CTR_MAX_SYSTEMS:
        raise ValueError("between 1 and %d systems are supported" % _abi.CTR_MAX_SYSTEMS)
    cfg = _abi.CtrEnvConfig()
    cfg.n_systems = len(systems)
    cfg.n_substeps = int(n_substeps)
    cfg.max_steps = int(max_steps)
    cfg.constrain_alpha = int(bool(constrain_alpha))
    cfg.egocentric = int(bool(egocentric))
    cfg.resample_joints = int(bool(resample_joints))
    cfg.integrator = int(integrator)
    cfg.rk4_steps_per_m = int(rk4_steps_per_m)
    cfg.model = int(model)
    cfg.tol = float(tol)
    cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    cfg.domain_rand = float(domain_rand)
    for k, tubes in enumerate(systems):
        cfg.systems[k] = to_ctr_system(tubes)
        cfg.raw[k] = to_ctr_tube_raw(tubes)
    return cfg


def copy_config(cfg):
    return copy.copy(cfg)


INTEGRATORS = {"rk45_scipy": _abi.CTR_INTEGRATOR_RK45_SCIPY, "rk4": _abi.CTR_INTEGRATOR_RK4}
MODELS = {"compliant": _abi.CTR_MODEL_COMPLIANT, "rigid": _abi.CTR_MODEL_RIGID}


def solver_codes(integrator, rk4_steps_per_m, model):
    """Validate the build's solver kwargs (integrator / h / model as explicit
    extra kwargs) and return their ABI codes."""
    if integrator not in INTEGRATORS:
        raise ValueError("integrator must be one of %s" % sorted(INTEGRATORS))
    if model not in MODELS:
        raise ValueError("model must be one of %s" % sorted(MODELS))
    spm = int(rk4_steps_per_m)
    if integrator == "rk4" and spm <= 0:
        raise ValueError("rk4_steps_per_m must be > 0")
    return INTEGRATORS[integrator], spm, MODELS[model]
