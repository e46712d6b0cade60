#!/usr/bin/env python3
"""Benchmark: env-steps/s of the batched CTR-Reach step on MI355X.

Workload (BASELINE.json configs[2], the headline): 65 536 parallel 3-tube envs per GPU,
torsionally-compliant model, scipy-faithful RK45 (parity mode, fp64), default CTR-Reach-v0
kwargs (system 0, n_substeps 10, tol 0.020 m, max 150 steps), synthetic uniform actions.
A "step" = one batched CtrReachVecEnv.step over all envs of the GPU.

Steady state ("including auto-resets at their natural rate"): the episode
clocks t are staggered uniformly over [0, max_steps) and the batch runs max_steps untimed
steps first, so time-limit resets arrive every step at the rate of a long-running trainer
(about n / 150 per step, plus successes).  The reset-pool refill interval is chosen to divide
the timed steps (largest divisor <= 64) and the window starts right after a refill, so the
window holds exactly steps / interval refills, each precomputing the resets the window itself
consumed.  resets_in_window and refills_in_window are reported.

Multi-GPU: ``python bench.py --gpus N`` launches N ranks itself (one process per GPU, before
anything touches a GPU); under ``torch.distributed.run`` the ranks come from the environment.
Rank r owns the contiguous global env ids [r n, (r + 1) n) (weak scaling, no collective on the
step itself).  With N > 1 every timed step also all-gathers the packed step outputs (16 B/env:
tip, done | success | reward) -- BASELINE configs[3] -- while the next step runs; k_step writes
the packed rows itself (pack_outputs).  Default gather (--gather-backend auto): the fused push
(distributed.PushGather: k_step itself stores every env's row into every rank's IPC-mapped
receive ring, paced by the ranks' slot releases, and waits until every rank's rows of the previous
step are in its own ring), checked bit for bit against a process-group all_gather on every step
of two refill periods before any timing, then timed against RCCL (whose kernels hold CUs the next
step needs); a failed check sends every rank to RCCL, and a failed check after the
window exits non-zero without a line.  A barrier + device sync bracket the timed region and the
time is the MAX over ranks.

Also reported: the dominant kernel's roofline (algorithmic FP64 flops / its average launch
time measured with HIP events on the launch stream) and the CPU oracle timed on this host
(cpu_baseline, rank 0 only).
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))

# Algorithmic work per RHS evaluation / RK attempt / segment:
FLOP_RHS = 102          # 3 angle differences, ux/uy (10 FMA per tube), u_z' (4/tube), R [u]x (27)
FLOP_ATTEMPT = 1050     # stage combinations 15x18 FMA, y_new 5x18, error 6x18, scale + norm
FLOP_SEGMENT = 150      # select_initial_step arithmetic
FLOP_RK4_STEP = 252     # RK4: 3 stage inputs 3x18 FMA + y_new 18 x 5 (+ stage sums), per step
FLOP_STEP_EXTRA = 220   # 10 x set_action (160) + reward/obs (60)
# configs[1] (rigid model, RK4): the executed work of the segment-power path (csrc/ctr_device.hpp
# rigid_segment_map / fk_group_rigid4), not the stepped RK4 count it replaces
FLOP_RIGID_MAP = 125    # per segment: [u]x (45), the step map's W-polynomial coefficients (23), the
                        # expansion of M^n to a 3x4 map (57)
FLOP_COMPOSE = 37       # one composition of two W-polynomial maps (2 x 17 + 3)
FLOP_TREE = 63          # one general 3x4 affine composition (9 x (mul + 2 fma) + 3 x 3 fma)
RIGID_TREE = 7          # compositions of the 8-lane group's ordered product (3 shuffle rounds)
SINCOS_RHS = 3
PEAK_FP64_VALU = 78.6   # TFLOP/s, MI355X FP64 vector (spec)
PEAK_HBM = 8000.0       # GB/s (spec)
# algorithmic bytes per env-step of this layout: reads system 4, joints 24, actions 24, epoch 4,
# t 4, desired goal 24 (f64) = 84; writes joints 24, achieved goal 24 (f64), t 4, obs 52, reward 4,
# done 1, success 1, error 4, status 4 = 118.  SURVEY.md 8(d)'s 170 B assumed float32 goals and
# no system / epoch / status words.  An auto-reset adds its pooled reset (the 108 B of fields of a
# ctr_pool_slot_t) read, and written: the terminal observation (13 x 4 B, or x 8 with float64
# observations), the terminal achieved goal 24, the new desired goal 24, system 4, epoch 4 (the
# bench env records no info buffers).
BYTES_STEP = 84 + 118
BYTES_RESET = 108
BYTES_RESET_WRITE_FIXED = 24 + 24 + 4 + 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                    help="GPUs (ranks); default: WORLD_SIZE of a torch.distributed launcher, else 1")
    ap.add_argument("--steps", type=int, default=128, help="timed steps")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=3, choices=(2, 3, 5),
                    help="BASELINE.json config (1-based): 3 = headline (65 536 envs, compliant, scipy RK45); "
                         "2 = 4 096 envs, rigid model, fixed-step RK4 (h = 10 mm); "
                         "5 = 65 536 envs, compliant, fixed-step RK4 at h = 2.5 mm (4x finer)")
    ap.add_argument("--envs", type=int, default=None, help="environments per GPU (default: the config's)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--profile-only", action="store_true", help="no timing extras (for rocprofv3)")
    ap.add_argument("--refill-interval", type=int, default=None,
                    help="reset-pool refill interval (steps); default: the largest divisor of --steps <= 64")
    ap.add_argument("--gather", choices=("auto", "on", "off"), default="auto",
                    help="all-gather of the packed step outputs in every timed step (auto: on when N > 1)")
    ap.add_argument("--gather-backend", choices=("auto", "push", "sdma", "rccl"), default="auto",
                    help="push: k_step itself stores every env's row into every rank's IPC-mapped receive ring "
                         "(the fused push); sdma: copy-engine copies after the step (host-synchronous per copy in "
                         "this runtime); rccl: all_gather_into_tensor over RCCL; auto: time push and rccl on 2 "
                         "refill periods each (untimed) and run the window with the faster.  push / sdma / auto fall "
                         "back to rccl if the IPC setup fails")
    ap.add_argument("--graph", choices=("auto", "on", "off"), default="auto",
                    help="replay each refill period's steps from one captured HIP graph (CtrReachVecEnv."
                         "capture_steps) instead of launching step by step from Python; auto: on without the "
                         "per-step gather")
    ap.add_argument("--pool-depth", type=int, default=None,
                    help="reset pool slots per env (default: the env's for the refill interval and budget)")
    ap.add_argument("--refill-budget", type=int, default=None,
                    help="resumable refill: RK45 iterations (RK4 steps) per reset FK and refill (default: the "
                         "env's, 6 (32); 0 = every refill runs its FKs to the end)")
    ap.add_argument("--obs-dtype", choices=("float32", "float64"), default="float32",
                    help="stored observation dtype (computed in float64 either way; float64 = the reference's)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / process-group check only (CPU, gloo): no GPU, no env, no bench line")
    ap.add_argument("--no-stagger", action="store_true",
                    help="start every episode at t = 0 (synchronised resets; not the steady state)")
    ap.add_argument("--systems", default="0",
                    help="select_systems, comma-separated registration indices (default 0, the headline; "
                         "'0,1,2,3' is SURVEY.md 8(d)'s mixed-system divergence check)")
    ap.add_argument("--untimed-min", type=int, default=480,
                    help="at least this many untimed steps before the window, and at least one episode "
                         "length + --warmup (the clocks of a GPU that just started stepping settle over "
                         "the first ~30-50 ms of sustained load)")
    return ap.parse_args()


def self_launch(args):
    """--gpus N without a torch.distributed launcher: start N ranks of this script (one per GPU)
    as child processes and exit with the worst return code.  Nothing here touches a GPU."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll: if a rank dies (e.g. a communicator init failure) the others would block in a
    # collective forever, so stop them and return the failed rank's code
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.05)


def dist_init(args):
    """One process per GPU.  RCCL (backend "nccl") by default.  Rehearsal overrides for a one-GPU
    box or a CPU-only host: CTR_BENCH_BACKEND=gloo with CTR_BENCH_SAME_DEVICE=1 puts every rank on
    cuda:0 (RCCL refuses two ranks on one GPU); the timing logic is the same."""
    import torch
    if args.dry_run:
        os.environ["CTR_BENCH_BACKEND"] = "gloo"
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws != args.gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started %d ranks" % (args.gpus, ws))
    if os.environ.get("CTR_BENCH_SAME_DEVICE") == "1":
        local = 0
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not args.dry_run:
            torch.cuda.set_device(local)
        backend = os.environ.get("CTR_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        return dist, rank, ws, local, backend
    return None, 0, 1, local, None


def D_max_over_ranks(v):
    sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
    from ctr_reach_amd import distributed as D
    return D.max_over_ranks(v, device="cpu")


def measured_traffic(n, cfgd, systems):
    """HBM bytes per k_step launch from the PMC passes committed under profiles/ (rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE, corrected by the factors measured on k_step's own access shapes:
    scripts/profile.sh + tools/summarize_profile.py), when they were taken on this workload; the
    bench cannot read hardware counters itself.  (None, reason) otherwise."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/traffic.json"
    if t.get("envs") != n or cfgd["integrator"] != "rk45_scipy" or cfgd["model"] != "compliant" or systems != [0]:
        return None, "profiles/traffic.json was measured on another workload"
    return t["bytes_per_launch"], ("profiles/traffic.json: k_step's average under rocprofv3 --pmc passes of "
                                   "this workload, FETCH_SIZE x %.3f + WRITE_SIZE x %.3f (factors calibrated on "
                                   "k_step's own access shapes)" % (t["read_factor"], t["write_factor"]))


def refill_interval_for(steps, cap=64):
    """Largest divisor of the timed steps that is <= cap: the window then holds whole refill
    periods (every reset it consumes is precomputed inside it)."""
    return max(d for d in range(1, min(cap, steps) + 1) if steps % d == 0)


def make_actions(env, k, seed):
    import torch
    g = torch.Generator(device=env.device)
    g.manual_seed(seed + 1)
    hi = torch.tensor(env.action_space.high, device=env.device)
    return [((torch.rand((env.num_envs, 6), generator=g, device=env.device) * 2 - 1) * hi).contiguous()
            for _ in range(k)]


CONFIGS = {
    2: dict(envs=4096, integrator="rk4", rk4_steps_per_m=100, model="rigid",
            text="configs[1]: %d envs/GPU, 3-tube torsionally-rigid CTR, fixed-step RK4 (h = 10 mm) fp64"),
    3: dict(envs=65536, integrator="rk45_scipy", rk4_steps_per_m=100, model="compliant",
            text="configs[2]: %d envs/GPU, 3-tube torsionally-compliant CTR, scipy-RK45 (rtol 1e-3, atol 1e-6) fp64"),
    5: dict(envs=65536, integrator="rk4", rk4_steps_per_m=400, model="compliant",
            text="configs[4]: %d envs/GPU, 3-tube torsionally-compliant CTR, fixed-step RK4 (h = 2.5 mm, 4x finer) "
                 "fp64"),
}


def fk_work(env, joints):
    """Algorithmic FP64 flops + sincos of one FK per env at the given joints (device counters).
    Fixed-step RK4 (both models): stats nstep counts the steps taken stage by stage, maps the
    segments run as segment maps and compositions their square-and-multiply products; a mapped
    segment is priced at its EXECUTED work (the map, its compositions, its application to [R | r]),
    not at the stepped RK4 count it replaces (nfev still reports 4 per RK4 step for parity)."""
    _, st = env.forward_kinematics(joints, env.system, return_stats=True)
    nfev = st["nfev"].double()
    seg = st["nseg"].double()
    if env.integrator == "rk4":
        maps, comps = st["maps"].double(), st["compositions"].double()
        stepped = st["nstep"].double()
        rhs = 4 * stepped
        if env.model == "rigid":
            # k_step's 8-lane groups build the same maps and join them in RIGID_TREE compositions
            per = maps * FLOP_RIGID_MAP + comps * FLOP_COMPOSE + RIGID_TREE * FLOP_TREE
        else:
            # stepped gaps at the SURVEY 8(d) count; the tube-0-alone tail as maps applied to [R | r]
            per = rhs * FLOP_RHS + stepped * FLOP_RK4_STEP + maps * (FLOP_RIGID_MAP + FLOP_TREE) + comps * FLOP_COMPOSE
    else:
        rhs = nfev
        att = (st["nstep"] + st["nrej"]).double()
        per = nfev * FLOP_RHS + att * FLOP_ATTEMPT + seg * FLOP_SEGMENT
    flops = per.sum().item() + FLOP_STEP_EXTRA * joints.shape[0]
    sincos = (rhs * SINCOS_RHS).sum().item()
    return flops, sincos, nfev.mean().item()


def parity_probe(env, cfgd):
    """tip-position L2 of the GPU FK against the CPU restatement of the reference
    (oracle/, pinned to the reference's fixtures) on every env's current joints, and agreement of
    the reached flag outside a +-1e-6 m band around tol.  Part of the CPU leg (rank 0, N = 1)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    q = env.joints.detach().cpu().numpy()
    sysid = env.system.detach().cpu().numpy()
    dg = env.desired_goal.detach().cpu().numpy()
    tip = env.forward_kinematics(env.joints, env.system).cpu().numpy()
    ref = oracle.fk(q, sysid, systems=oracle.make_systems(select=env.select_systems), integrator=cfgd["integrator"],
                    steps_per_m=cfgd["rk4_steps_per_m"], model=cfgd["model"])["tip"]
    l2 = np.linalg.norm(tip - ref, axis=1)
    tol = env.goal_tolerance.get_tol()
    d_gpu = np.linalg.norm(tip - dg, axis=1)
    d_cpu = np.linalg.norm(ref - dg, axis=1)
    outside = np.abs(d_cpu - tol) > 1e-6
    agree = ((d_gpu < tol) == (d_cpu < tol))[outside].mean() if outside.any() else 1.0
    out = {"envs": int(q.shape[0]), "tip_l2_max_m": float(l2.max()), "tip_l2_p999_m": float(np.quantile(l2, 0.999)),
           "reached_flag_agreement": float(agree), "band_m": 1e-6,
           "checker": "oracle/ctr_oracle.c (CPU restatement, pinned to the reference's fixtures)"}
    if cfgd["integrator"] != "rk45_scipy" or cfgd["model"] != "compliant":
        # the solver mode above is the build's own (no reference counterpart): the same GPU tips
        # against the reference's arithmetic (compliant model, scipy RK45 rtol 1e-3 / atol 1e-6,
        # model.py:141-151), restated by the oracle pinned to the reference's fixtures
        ref45 = oracle.fk(q, sysid, systems=oracle.make_systems(select=env.select_systems),
                          integrator="rk45_scipy", model="compliant")["tip"]
        l2r = np.linalg.norm(tip - ref45, axis=1)
        d_ref = np.linalg.norm(ref45 - dg, axis=1)
        out_r = np.abs(d_ref - tol) > 1e-6
        agree_r = ((d_gpu < tol) == (d_ref < tol))[out_r].mean() if out_r.any() else 1.0
        out_4 = np.abs(d_ref - tol) > 1e-4          # outside the tip bar: the flag must agree there
        agree_4 = ((d_gpu < tol) == (d_ref < tol))[out_4].mean() if out_4.any() else 1.0
        rigid = cfgd["model"] == "rigid"
        out["parity_vs_reference_arithmetic"] = {
            "tip_l2_max_m": float(l2r.max()), "tip_l2_p999_m": float(np.quantile(l2r, 0.999)),
            "tip_l2_mean_m": float(l2r.mean()), "frac_le_1e-4_m": float((l2r <= 1e-4).mean()),
            "reached_flag_agreement": float(agree_r), "band_m": 1e-6,
            "reached_flag_agreement_outside_1e-4_m": float(agree_4),
            "against": "oracle rk45_scipy, compliant model (the reference's solve_ivp RK45, rtol 1e-3, atol 1e-6)",
            "bar": ("none: a different model (torsionally rigid), outside the 1e-4 m bar by design"
                    if rigid else "north_star: tip <= 1e-4 m vs the reference CPU FK"),
            "within_bar": None if rigid else bool(l2r.max() <= 1e-4 or np.quantile(l2r, 0.999) <= 1e-4)}
    return out


def cpu_baseline(args, cfgd):
    """Oracle (C port, OpenMP) on this host: env-steps/s on a bounded sample of the workload, with
    the same staggered episode clocks and auto-resets (2 sampled joint sets + 2 FKs per reset) as
    the GPU window."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    fkw = dict(integrator=cfgd["integrator"], steps_per_m=cfgd["rk4_steps_per_m"], model=cfgd["model"])
    n = 4096
    rng = np.random.default_rng(args.seed + 1)
    q, _ = oracle.sample_joints(n, seed=args.seed, stream=1)
    dg = oracle.fk(oracle.sample_joints(n, seed=args.seed, stream=0)[0], **fkw)["tip"]
    hi = np.array([1e-3] * 3 + [np.deg2rad(5)] * 3, np.float32)
    t = rng.integers(0, 150, n).astype(np.int32)
    steps = resets = 0
    epoch = 1
    t0 = time.perf_counter()
    while True:
        a = ((rng.random((n, 6)) * 2 - 1) * hi).astype(np.float32)
        r = oracle.step(q, a, dg, t, 0.020, **fkw)
        q, t = r["joints"], r["t"]
        d = np.where(r["done"])[0]
        if d.size:                                     # CtrReachEnv.reset (ctr_reach_env.py:70-114)
            epoch += 1
            qd, _ = oracle.sample_joints(d.size, seed=args.seed, stream=0, epoch=epoch, env_base=int(d[0]))
            q0, _ = oracle.sample_joints(d.size, seed=args.seed, stream=1, epoch=epoch, env_base=int(d[0]))
            dg[d] = oracle.fk(qd, **fkw)["tip"]
            oracle.fk(q0, **fkw)
            q[d] = q0
            t[d] = 0
            resets += d.size
        steps += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    out = {"value": n * steps / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
           "sample": "%d envs x %d steps (%d auto-resets, staggered episode clocks) of oracle/ctr_oracle.c "
                     "(%s, %s model, fp64), OpenMP %d threads, %.1f s" % (n, steps, resets, cfgd["integrator"],
                                                                          cfgd["model"], threads, el)}
    # the reference's own CPU path (scipy solve_ivp, pure Python) cannot travel to this host: its
    # figures were measured in the build container (tools/time_reference.py), together with the
    # same port on the same cores, which calibrates the port against the reference per core
    try:
        with open(os.path.join(ROOT, "profiles", "cpu_reference_r01.json")) as fh:
            ref = json.load(fh)
        per_core = ref["port_over_reference_1core"]
        out["reference_python_here"] = {
            "env_steps_per_s_1core": ref["env_steps_per_s_1proc"],
            "env_steps_per_s_%dcores" % ref["nproc"]: ref["env_steps_per_s_nproc"],
            "what": ref["what"], "cpu": ref["cpu"] + " (the build container, not this host)",
            "port_over_reference_per_core": per_core,
            "reference_equivalent_on_these_cores": (out["value"] / per_core
                                                    if cfgd["integrator"] == "rk45_scipy" else None),
            "source": "profiles/cpu_reference_r01.json (tools/time_reference.py: CtrReachEnv.step() of the unmodified "
                      "reference, default kwargs, 20 s per run)"}
    except (OSError, ValueError, KeyError):
        pass
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args)
    import torch
    dist, rank, ws, local, backend = dist_init(args)
    if args.dry_run:
        # the multi-rank plumbing without a GPU: every rank reports in, rank 0 prints the count
        t = torch.ones(1)
        if dist:
            dist.all_reduce(t)
        el = D_max_over_ranks(0.001 * (rank + 1))
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": ws, "ranks_reporting": int(t.item()),
                              "backend": backend, "max_over_ranks_s": el}), flush=True)
        if dist:
            dist.destroy_process_group()
        return 0
    from ctr_reach_amd import CtrReachVecEnv
    from ctr_reach_amd import distributed as D
    from ctr_reach_amd import _abi
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cfgd = CONFIGS[args.config]
    n = args.envs or cfgd["envs"]
    gather = (args.gather == "on") or (args.gather == "auto" and ws > 1)
    if gather and not dist:
        raise SystemExit("--gather on needs more than one rank")
    R = args.refill_interval or refill_interval_for(args.steps)
    systems = [int(s) for s in args.systems.split(",")]
    env = CtrReachVecEnv(n, device=dev, seed=args.seed, env_base=D.shard(n, rank), autoreset=True, record_info=False,
                         integrator=cfgd["integrator"], rk4_steps_per_m=cfgd["rk4_steps_per_m"], model=cfgd["model"],
                         select_systems=systems, refill_interval=R, pack_outputs=gather, obs_dtype=args.obs_dtype,
                         refill_budget=args.refill_budget if cfgd["model"] == "compliant" else None,
                         pool_depth=args.pool_depth)
    env.reset()
    max_steps = env.max_steps_per_episode
    if not args.no_stagger:
        # the episode phase of a long-running batch is uniform over [0, max_steps)
        g = torch.Generator(device="cpu")
        g.manual_seed(args.seed + 17 + rank)
        env.t.copy_(torch.randint(0, max_steps, (n,), generator=g, dtype=torch.int32))
    acts = make_actions(env, 8, args.seed + rank)
    backend_used = None
    fallback_note = None
    calibration = None
    if gather:
        backend_used = args.gather_backend
        if backend_used in ("push", "sdma", "auto"):
            try:
                # push: depth 3 and the fused consumer wait (k_step(t) returns only once every
                # rank's rows of step t - 1 are in this rank's ring), so every timed step also
                # completes a gather, as RCCL's stream-ordered collective does
                if backend_used == "sdma":
                    env.enable_gather("sdma")
                else:
                    env.enable_gather("push", depth=3, wait_prev=True)
            except Exception as ex:          # noqa: BLE001 -- reported in the line, RCCL measured instead
                print("bench.py: %s gather setup failed (%s); using rccl" % (backend_used, ex), file=sys.stderr,
                      flush=True)
                fallback_note = "%s setup failed: %s" % (args.gather_backend, str(ex)[:160])
                backend_used = "rccl"
        # the env steps on a high-priority stream (RCCL's gather runs on its normal-priority one).
        # RCCL's gather kernel (248-256 VGPRs, 37 KB LDS per workgroup) cannot share a SIMD with a
        # k_step wave (368 of the 512 registers), so whichever is dispatched first holds the CU:
        # with the step first, the gather of step t fills the CUs the slowest waves of step t+1
        # leave idle instead of keeping step t+1's workgroups off the CUs it took
        hp = torch.cuda.Stream(device=dev, priority=-1)
        hp.wait_stream(torch.cuda.current_stream())
        torch.cuda.set_stream(hp)
    stream = torch.cuda.current_stream()
    works = [None, None]
    push_gather = env._push_gather
    state = {"mode": "push" if backend_used == "auto" else backend_used}

    def one_step(i):
        mode = state["mode"]
        k = env._packed_k ^ 1        # the pack buffer this step writes
        if mode == "rccl" and works[k] is not None:
            works[k].wait()          # the gather that last read this pack buffer (stream-ordered, no host wait)
        env.step_raw(acts[i % len(acts)])    # push: the step itself stores its rows into every ring;
        if mode == "sdma":                   # sdma: the step waited for the copies that read buffer k
            env.gather_outputs(backend="sdma", async_op=True)
        elif mode == "rccl":
            _, works[k] = env.gather_outputs(async_op=True)

    def timed_steps(count, start):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(count):
            one_step(start + i)
        for w in works:
            if w is not None:
                w.wait()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        return D.max_over_ranks(time.perf_counter() - t0, device=dev if backend in (None, "nccl") else "cpu")

    # the window's bookkeeping (and the first barrier) once here: their first use loads kernels /
    # builds communicators for tens of ms, and a GPU left idle that long before the window drops
    # its clocks (the first steps after such a gap ran 94-102 us instead of 88-90 us)
    env.epoch.to(torch.int64).sum().item()
    if dist:
        dist.barrier()
    # untimed: one whole episode length (every env passes a time-limit reset) and the warmup,
    # rounded up to whole refill periods so the last untimed step ends with a pool refill and the
    # window starts on a refill boundary with the GPU still busy
    pre = -(-max(max_steps + args.warmup, args.untimed_min) // R) * R
    # no collector pass from here to the end of the window: a full pass takes tens of ms (a host
    # pause that idles the GPU before the window, or starves it while the window is queued)
    gc.collect()
    gc.disable()
    done_pre = 0
    check = None
    if backend_used in ("push", "auto"):
        # before any timing: every push step of 2 refill periods waited on and bit-compared, on
        # every rank, with a process-group all_gather of the ranks' own rows (the reference copy);
        # a mismatch or a wait error on any rank sends every rank to RCCL, with the reason
        def push_step(i):
            one_step(done_pre + i)
            return env.gather_seq
        check = D.check_push_steps(push_step, push_gather, env.packed_outputs, 2 * R,
                                   stream=torch.cuda.current_stream())
        done_pre += check["steps_checked"]
        if not check["passed"]:
            print("bench.py: push gather check failed (%s); using rccl" % check, file=sys.stderr, flush=True)
            fallback_note = "push gather check failed: %s" % json.dumps(check)
            backend_used = state["mode"] = "rccl"
            env._push_gather = None
    if backend_used == "auto":
        # pick the faster gather on this node: 2 refill periods of each (untimed, max over ranks);
        # the push stores ride inside the steps, so RCCL's turn runs with the push detached
        calibration = {}
        for _ in range(2):                   # the first pair warms both paths up
            for m in ("rccl", "push"):
                state["mode"] = m
                env._push_gather = push_gather if m == "push" else None
                calibration[m + "_ms_per_step"] = timed_steps(2 * R, done_pre) / (2 * R) * 1e3
                done_pre += 2 * R
        backend_used = min(("push", "rccl"), key=lambda m: calibration[m + "_ms_per_step"])
        state["mode"] = backend_used
        env._push_gather = push_gather if backend_used == "push" else None
    # the window starts on a refill boundary: whole refill periods before it
    pre = max(pre, -(-(done_pre + R) // R) * R)
    for i in range(done_pre, pre):
        one_step(i)
    use_graph = args.graph == "on" or (args.graph == "auto" and not gather)
    graph = None
    if use_graph:
        # one refill period (R steps, the pool refill at its end) captured once; the window replays
        # it steps / R times.  The capture launches nothing; two untimed replays warm the graph.
        graph = env.capture_steps([acts[i % len(acts)] for i in range(R)])
        for _ in range(2):
            graph.replay()
    R_steps = R
    if args.profile_only:
        for i in range(args.steps):
            one_step(i)
        torch.cuda.synchronize()
        return 0

    # ---- timed region: K whole-job steps, auto-resets and pool refills at their natural rate
    epoch0 = env.epoch.to(torch.int64).sum()
    refills0, sweeps0 = env.refills, env.sweeps
    carried0 = sum(env.carried())                 # suspended resets the window's first refill finishes
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if graph is not None:
        for _ in range(args.steps // R_steps):
            graph.replay()
    else:
        for i in range(args.steps):
            one_step(i)
    for w in works:
        if w is not None:
            w.wait()
    if backend_used == "sdma":
        # every rank's pushes of the window: own copies done (sync), then the barrier after which
        # every peer's copies into this rank's ring are done too (push: the rows are stored by the
        # window's own k_step launches)
        for ev in env._push_gather.done[0] + env._push_gather.done[1]:
            torch.cuda.current_stream().wait_event(ev)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el_local = time.perf_counter() - t0
    gc.enable()
    if backend_used in ("push", "sdma"):
        # the window's last gather, checked where it landed: this rank's slot holds every rank's
        # rows of the last timed step (consumer wait, then a bit-exact compare with the gloo/RCCL
        # copy of the same rows), and no rank's error word has a bit set (a wait or a slot
        # release that timed out in any step of the window); outside the timed region
        seq = env.gather_seq if backend_used == "push" else env.packed_seq
        ok, rep = D.verify_gathered(env._push_gather.wait(seq, torch.cuda.current_stream()), env.packed_outputs(),
                                    env._push_gather.err, group=None)
        gather_check = dict(rep, last_step_rows_equal=rep["rows_equal_all_ranks"], passed=ok)
        if not ok:
            # a fast, wrong headline is worse than none: no line, non-zero exit on every rank
            print("bench.py: the %s gather of the window failed its check: %s" % (backend_used, json.dumps(rep)),
                  file=sys.stderr, flush=True)
            if dist:
                dist.destroy_process_group()
            return 3
    el = D.max_over_ranks(el_local, device=dev if backend in (None, "nccl") else "cpu")
    traffic, traffic_note = measured_traffic(n, cfgd, systems) if ws == 1 else (None, None)
    resets_local = int((env.epoch.to(torch.int64).sum() - epoch0).item())
    refills = env.refills - refills0
    sweeps = env.sweeps - sweeps0
    resets = resets_local
    if dist:
        rt = torch.tensor([resets_local], dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(rt)
        resets = int(rt.item())
    total_steps = n * ws * args.steps

    # ---- k_step as the window runs it (pooled auto-resets), from the window's end state (right
    # after a refill): R - 1 back-to-back step launches bracketed by one event pair on the launch
    # stream, no refill among them (the R-th step, untimed, brings the refill that falls due).
    # Without the per-step gather only (its steps also wait for / launch the gather).
    k_ms_pooled = None
    if not gather and R_steps > 1 and env._steps_since_refill == 0:
        ep0, ep1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ep0.record(stream)
        for i in range(R_steps - 1):
            one_step(i)
        ep1.record(stream)
        one_step(R_steps - 1)
        torch.cuda.synchronize()
        k_ms_pooled = ep0.elapsed_time(ep1) / (R_steps - 1)

    # ---- dominant kernel (k_step) alone: HIP events on the launch stream, no auto-reset.
    # ctr_step with autoreset = 0 launches exactly one kernel (k_step) on `stream`; one event pair
    # brackets k_iters back-to-back launches (per-launch event pairs add their own few us), so the
    # average includes the ~1.5 us launch boundaries and slightly over-states the kernel time.
    j_probe = env.joints.clone()
    flops_env_step, sincos, nfev_mean = fk_work(env, j_probe)
    k_iters = 32
    sp = _abi.stream_ptr(stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(256):             # untimed: back to sustained-load clocks after fk_work's host sync
        _abi.check(env.lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[i % len(acts)]), env._out, 0, sp), "ctr_step")
    env.joints.copy_(j_probe)        # the timed launches start from the state fk_work priced
    e0.record(stream)
    for i in range(k_iters):
        rc = env.lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[i % len(acts)]), env._out, 0, sp)
        _abi.check(rc, "ctr_step")
    e1.record(stream)
    torch.cuda.synchronize()
    k_ms = e0.elapsed_time(e1) / k_iters

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return 0
    achieved_tf = flops_env_step / (k_ms * 1e-3) / 1e12
    out = {
        "metric": "env-steps/sec at 65 536 parallel 3-tube envs; tip-pos L2 vs CPU ref",
        "value": total_steps / el,
        "unit": "env-steps/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: Philox-sampled joints/goals (sample_goal region), uniform actions in the action box",
        "config": {"workload": (cfgd["text"] % n) + ", %s, n_substeps 10, tol 0.020, max 150 steps, "
                                                     "auto-reset" % ("system %d" % systems[0] if len(systems) == 1 else
                                                                     "systems %s drawn per reset" % args.systems)
                   + (", %s all-gather of packed tip/reward/done every step" %
                      {"push": "fused-push", "sdma": "copy-engine (SDMA)", "rccl": "RCCL"}[backend_used]
                      if gather else ""),
                   "obs_dtype": args.obs_dtype,
                   "integrator": cfgd["integrator"], "model": cfgd["model"],
                   "rk4_steps_per_m": cfgd["rk4_steps_per_m"] if cfgd["integrator"] == "rk4" else None,
                   "envs_per_gpu": n, "global_envs": n * ws, "parallelism": "env-shard x%d" % ws,
                   "process_group": {"backend": backend, "world_size": ws} if dist else None,
                   "all_gather": dict({"bytes_per_env": 4 * D.PACK_WIDTH, "async": True, "backend": backend_used},
                                      **({"engine": env._push_gather.engine, "depth": env._push_gather.depth,
                                          "consumer_wait": "fused: k_step(t) completes once every rank's rows of "
                                                           "step t - 1 are in this rank's ring"
                                          if env._push_gather.wait_prev else "none in the window",
                                          "check": gather_check}
                                         if backend_used in ("push", "sdma") else {}),
                                      **({"pre_window_check": check} if check else {}),
                                      **({"rccl_channels": "RCCL's own choice (uncapped): on one GPU an RCCL-footprint "
                                                           "gather costs its duration + ~7 us whatever its workgroup "
                                                           "count, so a channel cap only lengthens it (DESIGN.md 6.2)"}
                                         if backend_used == "rccl" else {}),
                                      **({"calibration": calibration, "chosen_by": "calibration"}
                                         if calibration else {}),
                                      **({"fallback": fallback_note} if fallback_note else {}))
                   if gather else None,
                   "launch": ("one HIP graph per refill period (%d steps + the refill), replayed" % R_steps
                              if graph is not None else "per step from Python (ctypes -> ctr_step)"),
                   "reset_pool": {"depth": env.pool_depth, "refill_interval": env.refill_interval,
                                  "autoreset": "pooled (no miss sweep)" if env._pooled_steps() >= env.refill_interval
                                  else "pooled + miss sweep",
                                  "refill_budget": env.refill_budget,
                                  "suspended_resets_before_window": carried0,
                                  "suspended_resets_after_window": sum(env.carried())},
                   "steady_state": {"staggered_t": not args.no_stagger, "untimed_steps_before": pre,
                                    "resets_in_window": resets, "refills_in_window": refills * ws,
                                    "refills_in_window_per_rank": refills,
                                    "miss_sweep_launches_in_window_per_rank": sweeps,
                                    "mean_episode_steps_est": (total_steps / resets) if resets else None}},
        "roofline": {"bound": "valu", "achieved": achieved_tf, "peak": PEAK_FP64_VALU, "unit": "TFLOP/s",
                     "frac": achieved_tf / PEAK_FP64_VALU, "traffic": traffic,
                     "traffic_source": traffic_note,
                     "kernel": "k_step", "kernel_ms": k_ms,
                     "kernel_autoreset": "off (achieved / frac time k_step with CTR_AUTORESET_OFF: 32 back-to-back "
                                         "launches from the window's joints, the FK work priced on those joints)",
                     "kernel_ms_autoreset_pooled": k_ms_pooled,
                     "frac_autoreset_pooled": (flops_env_step / (k_ms_pooled * 1e-3) / 1e12 / PEAK_FP64_VALU
                                               if k_ms_pooled else None),
                     "kernel_ms_autoreset_pooled_note": ("k_step as the window launches it (CTR_AUTORESET_POOLED: done "
                                                         "envs copy their precomputed reset), %d back-to-back launches "
                                                         "after the window, no refill among them; its frac prices the "
                                                         "same FK work as kernel_ms" % (R_steps - 1)
                                                         if k_ms_pooled else
                                                         "not measured: the window's steps also run the per-step gather "
                                                         "(or a refill period of one step)"),
                     "flops_per_launch": flops_env_step, "sincos_per_launch": sincos,
                     "nfev_per_env_step": nfev_mean,
                     "bytes_per_launch_algorithmic": BYTES_STEP * n,
                     "hbm_gbs_algorithmic": BYTES_STEP * n / (k_ms * 1e-3) / 1e9,
                     "hbm_frac_algorithmic": BYTES_STEP * n / (k_ms * 1e-3) / 1e9 / PEAK_HBM,
                     "note": ("bound is the FP64 vector pipe: no GEMM-shaped work for MFMA, far above the HBM ridge; "
                              "peak = MI355X FP64 vector spec; flops from device counters (sincos not priced): " +
                              ("the EXECUTED work of the rigid segment-power path (125 flop per segment map, 37 per "
                               "W-polynomial composition, 63 per 3x4 composition of the 8-lane group product), not the "
                               "stepped RK4 count"
                               if cfgd["model"] == "rigid" else
                               "SURVEY 8(d) count for the RK4 steps taken stage by stage (4 RHS x 102 + 252 per step); the "
                               "tube-0-alone tail segments run as segment maps and are priced at their EXECUTED work (125 "
                               "per map + 63 to apply it + 37 per composition), not at the stepped count"
                               if cfgd["integrator"] == "rk4" else "SURVEY 8(d) count"))},
    }
    tr = os.path.join(ROOT, "profiles", "traffic.json" if args.config == 3 else "traffic_c%d.json" % args.config)
    if ws > 1:
        # the one-GPU PMC passes do not see a rank's stores into its peers' rings (16 B per env and
        # peer) nor RCCL's traffic
        out["roofline"]["traffic"] = None
        out["roofline"]["traffic_source"] = ("not measured for N > 1: profiles/traffic.json is k_step on one GPU "
                                             "without the gather's peer stores")
    elif os.path.exists(tr):
        with open(tr) as fh:
            t = json.load(fh)
        if t.get("envs") == n and t.get("config", 3) == args.config and systems == [0]:
            out["roofline"]["traffic"] = t.get("bytes_per_launch")
            out["roofline"]["traffic_source"] = "profiles/%s: %s" % (os.path.basename(tr), t.get("note", ""))
            out["roofline"]["traffic_over_algorithmic"] = t.get("bytes_per_launch") / (BYTES_STEP * n)
            # the PMC passes run the window's pooled steps, so their bytes include the auto-resets at
            # the window's rate: the algorithmic bytes of those resets beside them
            if resets:
                per_reset = BYTES_RESET + BYTES_RESET_WRITE_FIXED + 13 * (8 if args.obs_dtype == "float64" else 4)
                alg_r = BYTES_STEP * n + per_reset * resets / args.steps
                out["roofline"]["bytes_per_launch_algorithmic_with_resets"] = alg_r
                out["roofline"]["bytes_per_reset_algorithmic"] = per_reset
                out["roofline"]["traffic_over_algorithmic_with_resets"] = t.get("bytes_per_launch") / alg_r
    if not args.no_cpu_baseline and ws == 1:
        out["parity"] = parity_probe(env, cfgd)
        out["cpu_baseline"] = cpu_baseline(args, cfgd)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
