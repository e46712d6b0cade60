"""Host-side logic and the C-ABI surface (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ctr_reach_amd.h")


def _declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char \*)\s*(ctr_\w+)\s*\(", src, re.M)))


def test_library_exports_every_declared_symbol():
    from ctr_reach_amd import _abi
    lib = _abi.load()
    names = _declared_functions()
    assert set(names) == set(_abi.EXPORTED)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.ctr_abi_version() == _abi.CTR_ABI_VERSION
    out = subprocess.check_output(["nm", "-D", "--defined-only", _abi.LIB_PATH]).decode()
    for n in names:
        assert re.search(r"\bT %s\b" % n, out), n


def test_refill_carry_bytes():
    """ctr_refill_carry_bytes (host arithmetic, no GPU): a 1-KB header (counts[2][64], parity),
    then two lists of 640-B suspended-reset records; negative capacities give 0."""
    from ctr_reach_amd import _abi
    lib = _abi.load()
    for cap in (0, 1, 256, 131072):
        assert lib.ctr_refill_carry_bytes(cap) == 1024 + 2 * cap * 640
    assert lib.ctr_refill_carry_bytes(-5) == 0


def test_abi_rejects_bad_arguments_without_gpu():
    from ctr_reach_amd import _abi, systems
    lib = _abi.load()
    cfg = systems.make_config(systems.tubes_from_params(systems.default_systems_parameters())[:1])
    cfg.n_systems = 0
    rc = lib.ctr_fk(None, None, 4, cfg, None, None, None, None)
    assert rc == -1 and b"n_systems" in lib.ctr_last_error()
    cfg.n_systems = 1
    rc = lib.ctr_fk(None, None, 4, cfg, None, None, None, None)
    assert rc == -1
    assert lib.ctr_fk(None, None, 0, cfg, None, None, None, None) == 0   # empty batch is a no-op
    b = _abi.CtrBatch()
    b.n = 0
    assert lib.ctr_step(cfg, b, ctypes.c_void_p(1), _abi.CtrStepOut(), 1, None) == 0
    b.n = 8
    assert lib.ctr_step(cfg, b, ctypes.c_void_p(1), _abi.CtrStepOut(), 1, None) == -1


def test_autoreset_modes_and_pool_requeue_validate_without_gpu():
    """The round-2 entry points reject bad arguments before any HIP call: an unknown autoreset
    mode, CTR_AUTORESET_POOLED without a reset pool, a HER store whose t_max / env_base disagree
    with the config / batch, ctr_pool_requeue without a batch."""
    from ctr_reach_amd import _abi, systems
    lib = _abi.load()
    cfg = systems.make_config(systems.tubes_from_params(systems.default_systems_parameters())[:1])
    fake = ctypes.c_void_p(16)
    b = _abi.CtrBatch()
    b.n = 8
    b.joints = b.desired_goal = b.achieved_goal = b.t = b.system = b.epoch = b.work = fake
    o = _abi.CtrStepOut()
    o.obs = o.reward = o.done = o.success = o.error = fake
    assert lib.ctr_step(cfg, b, fake, o, 3, None) == -1
    assert b"autoreset" in lib.ctr_last_error()
    assert lib.ctr_step(cfg, b, fake, o, _abi.AUTORESET_POOLED, None) == -1
    assert b"reset pool" in lib.ctr_last_error()
    h = _abi.CtrHer()
    h.obs_dim, h.t_max, h.n_sampled_goal, h.strategy, h.n, h.slots = 13, cfg.max_steps + 1, 4, 0, 8, 4
    h.state = h.step = h.dg = h.tol = h.len = h.epoch = h.cur_t = h.cur_epoch = h.cdf = fake
    assert lib.ctr_step_her(cfg, b, fake, o, _abi.AUTORESET_SWEEP, h, None) == -1
    assert b"t_max" in lib.ctr_last_error()
    h.t_max, h.env_base = cfg.max_steps, 64
    assert lib.ctr_step_her(cfg, b, fake, o, _abi.AUTORESET_SWEEP, h, None) == -1
    assert b"env_base" in lib.ctr_last_error()
    assert lib.ctr_pool_requeue(cfg, None, None) == -1
    # ABI 15: the pool is one array of 128-B slots, which must be line-aligned
    b.pool_depth, b.refill, b.refill_cap = 4, fake, 64
    b.pool = ctypes.c_void_p(16 + 64)
    assert lib.ctr_pool_refill(cfg, b, None) == -1
    assert b"128-B aligned" in lib.ctr_last_error()
    b.pool = None
    assert lib.ctr_pool_refill(cfg, b, None) == -1
    assert b"needs the pool" in lib.ctr_last_error()
    b.pool_depth = 0
    b.n = 0
    assert lib.ctr_pool_requeue(cfg, b, None) == 0                     # empty batch: no-op


def test_struct_layout_matches_header(tmp_path):
    """ctypes mirrors of the ABI structs have the C sizes and every field offset (gcc on the header)."""
    from ctr_reach_amd import _abi
    structs = [(_abi.CtrSystem, "ctr_system_t"), (_abi.CtrTubeRaw, "ctr_tube_raw_t"),
               (_abi.CtrEnvConfig, "ctr_env_config_t"), (_abi.CtrBatch, "ctr_batch_t"),
               (_abi.CtrStepOut, "ctr_step_out_t"), (_abi.CtrHer, "ctr_her_t"), (_abi.CtrHerBatch, "ctr_her_batch_t"),
               (_abi.CtrCopy, "ctr_copy_t"), (_abi.CtrGatherPush, "ctr_gather_push_t"),
               (_abi.CtrPoolSlot, "ctr_pool_slot_t")]
    lines, want = [], []
    for cls, cname in structs:
        lines.append('  printf("%%zu\\n", sizeof(%s));' % cname)
        want.append(ctypes.sizeof(cls))
        for fname, _ in cls._fields_:
            lines.append('  printf("%%zu\\n", offsetof(%s, %s));' % (cname, fname))
            want.append(getattr(cls, fname).offset)
    prog = tmp_path / "layout.c"
    prog.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"ctr_reach_amd.h\"\nint main(void) {\n"
                    + "\n".join(lines) + "\n  return 0; }\n")
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)])
    got = list(map(int, subprocess.check_output([str(exe)]).split()))
    assert got == want


def test_spaces_match_reference_definitions():
    from ctr_reach_amd.vec_env import action_space, joint_spaces, observation_space
    from ctr_reach_amd.systems import tubes_from_params, default_systems_parameters
    from ctr_reach_amd.goal_tolerance import GoalTolerance
    from ctr_reach_amd.systems import default_kwargs
    sysl = tubes_from_params(default_systems_parameters())
    a = action_space(0.001, 5)
    assert a.dtype == np.float32 and a.shape == (6,)
    np.testing.assert_allclose(a.high, np.float32([1e-3] * 3 + [np.deg2rad(5)] * 3))
    js, jss = joint_spaces(sysl[:1], False)
    assert js[0].low.dtype == np.float32
    assert js[0].low[0] == np.float32(-0.431 + 1e-3) and np.isinf(js[0].high[3])
    js, _ = joint_spaces(sysl[:1], True)
    assert js[0].high[3] == np.float32(np.pi)
    gt = GoalTolerance(default_kwargs()["goal_tolerance_parameters"])
    o1 = observation_space(sysl[:1], gt)
    o4 = observation_space(sysl, gt)
    assert o1["observation"].shape == (13,) and o4["observation"].shape == (14,)
    assert o4["observation"].high[-1] == 3
    assert o1["observation"].low[12] == np.float32(0.001) and o1["observation"].high[12] == np.float32(0.02)


@pytest.mark.parametrize("fn", ["constant", "linear", "decay"])
def test_goal_tolerance_schedule(fn):
    from ctr_reach_amd.goal_tolerance import GoalTolerance
    p = {"inc_tol_obs": False, "final_tol": 0.001, "initial_tol": 0.020, "N_ts": 1000, "function": fn, "set_tol": 0}
    g = GoalTolerance(p)
    assert g.get_tol() == 0.020
    g.update(500)
    if fn == "constant":
        assert g.get_tol() == 0.001          # reference quirk: constant -> final_tol after update
    elif fn == "linear":
        assert abs(g.get_tol() - (0.020 + (0.001 - 0.020) / 1000 * 500)) < 1e-15
    else:
        assert 0.001 < g.get_tol() < 0.020
    g.update(2000)
    assert g.get_tol() == 0.001
    p["set_tol"] = 0.005
    g = GoalTolerance(p)
    g.update(10)
    assert g.get_tol() == 0.005


def test_make_uses_registration_defaults():
    from ctr_reach_amd.systems import default_kwargs
    kw = default_kwargs()
    assert kw["select_systems"] == [0] and kw["n_substeps"] == 10 and kw["max_steps_per_episode"] == 150
    assert kw["joint_representation"] == "egocentric" and kw["domain_rand"] == 0.0


def test_config_encoding():
    from ctr_reach_amd import systems
    sysl = systems.tubes_from_params(systems.default_systems_parameters())
    cfg = systems.make_config(sysl, tol=0.01, seed=2**64 - 1, constrain_alpha=True)
    assert cfg.n_systems == 4 and cfg.constrain_alpha == 1 and cfg.seed == 2**64 - 1
    t = sysl[2][1]
    assert cfg.systems[2].EI[1] == t.E * t.I and cfg.systems[2].GJ[1] == t.G * t.J
    with pytest.raises(ValueError):
        systems.make_config(sysl * 3)


def test_new_entry_points_validate_arguments_without_gpu():
    """ctr_jacobian / ctr_fk_shape / ctr_fk_tables / ctr_domain_params reject bad arguments before
    touching the device (no GPU needed)."""
    from ctr_reach_amd import _abi, systems
    lib = _abi.load()
    cfg = systems.make_config(systems.tubes_from_params(systems.default_systems_parameters())[:1])
    p = ctypes.c_void_p(1)
    assert lib.ctr_jacobian(p, None, 4, cfg, 0.0, None, p, None, None) == -1          # eps = 0
    assert b"eps" in lib.ctr_last_error()
    assert lib.ctr_jacobian(None, None, 4, cfg, 1e-4, None, p, None, None) == -1      # no joints
    assert lib.ctr_jacobian(None, None, 0, cfg, 1e-4, None, None, None, None) == 0     # empty
    assert lib.ctr_fk_tables(p, None, 4, cfg, p, None, None, None) == -1              # no tables
    assert lib.ctr_fk_shape(p, None, None, 4, cfg, 270, p, None, None, p, None, None) == -1   # no r/s
    rk4 = systems.make_config(systems.tubes_from_params(systems.default_systems_parameters())[:1],
                              integrator=_abi.CTR_INTEGRATOR_RK4, rk4_steps_per_m=100)
    assert lib.ctr_fk_shape(p, None, None, 4, rk4, 270, p, p, p, p, None, None) == -1
    assert b"rk45" in lib.ctr_last_error()
    bad = systems.make_config(systems.tubes_from_params(systems.default_systems_parameters())[:1],
                              integrator=_abi.CTR_INTEGRATOR_RK4, rk4_steps_per_m=0)
    assert lib.ctr_fk(p, None, 4, bad, p, None, None, None) == -1                     # RK4 without steps
    cfg.domain_rand = float("nan")
    assert lib.ctr_domain_params(cfg, _abi.CtrBatch(), p, None, None) == -1
    cfg.domain_rand = 0.05
    b = _abi.CtrBatch()
    b.n = 4
    assert lib.ctr_domain_params(cfg, b, p, None, None) == -1                         # no system/epoch


def test_solver_kwargs_validation():
    from ctr_reach_amd.systems import solver_codes
    assert solver_codes("rk45_scipy", 0, "compliant") == (0, 0, 0)
    assert solver_codes("rk4", 100, "rigid") == (1, 100, 1)
    with pytest.raises(ValueError):
        solver_codes("rk4", 0, "compliant")
    with pytest.raises(ValueError):
        solver_codes("euler", 10, "compliant")
    with pytest.raises(ValueError):
        solver_codes("rk45_scipy", 0, "stiff")


def test_her_abi_rejects_bad_arguments_without_gpu():
    from ctr_reach_amd import _abi
    lib = _abi.load()
    h = _abi.CtrHer()
    h.obs_dim, h.t_max, h.n_sampled_goal, h.strategy, h.slots, h.n = 13, 150, 4, 0, 4, 0
    b = _abi.CtrBatch()
    assert lib.ctr_her_open(h, b, ctypes.c_void_p(1), None, None) == 0          # empty store: no-op
    h.slots = 1
    assert lib.ctr_her_open(h, b, ctypes.c_void_p(1), None, None) == -1 and b"slots" in lib.ctr_last_error()
    h.slots, h.strategy = 4, 7
    assert lib.ctr_her_record(h, b, ctypes.c_void_p(1), _abi.CtrStepOut(), 0.02, None) == -1
    h.strategy, h.n = 0, 8
    assert lib.ctr_her_sample(h, 4, 0, 0, _abi.CtrHerBatch(), None) == -1 and b"buffer" in lib.ctr_last_error()
    assert lib.ctr_her_sample(None, 4, 0, 0, _abi.CtrHerBatch(), None) == -1


def test_gather_row_pack_roundtrip():
    """The 16-B gather row (distributed.PACK_WIDTH = 4 float32 words): tip rounded to float32,
    and done / success / (reward = -1) as flag bits; the env's sparse reward (-1 or 0,
    ctr_reach_env.py:160-170) comes back exactly, with +0 rather than -0."""
    import torch
    from ctr_reach_amd import distributed as D
    rng = np.random.default_rng(0)
    n = 1000
    tip = torch.tensor(rng.normal(0, 0.1, (n, 3)))
    reward = torch.tensor(-(rng.random(n) < 0.7).astype(np.float32))
    done = torch.tensor(rng.random(n) < 0.3).to(torch.uint8)
    success = (reward == 0).to(torch.uint8)
    p = D.pack_step_outputs(tip, reward, done, success)
    assert p.shape == (n, D.PACK_WIDTH) and p.dtype == torch.float32 and p.element_size() * D.PACK_WIDTH == 16
    t2, r2, d2, s2 = D.unpack_step_outputs(p)
    assert torch.equal(t2, tip.float())
    assert torch.equal(r2, reward) and not torch.signbit(r2[r2 == 0]).any()
    assert torch.equal(d2, done.bool()) and torch.equal(s2, success.bool())
