#!/usr/bin/env python3
"""Benchmark: env-steps/s of the batched CTR-Reach step on MI355X.

Workload (BASELINE.json configs[2], the headline): 65 536 parallel 3-tube envs per GPU,
torsionally-compliant model, scipy-faithful RK45 (parity mode, fp64), default CTR-Reach-v0
kwargs (system 0, n_substeps 10, tol 0.020 m, max 150 steps), synthetic uniform actions,
auto-resets at their natural rate inside the timed region.  A "step" = one batched
CtrReachVecEnv.step over all envs of the GPU.

Multi-GPU (``torchrun --nproc-per-node N``): one process per GPU, contiguous shards of the
global env id space (env_base = rank * n), no collective on the data path (weak scaling);
a barrier + device sync bracket the timed region and the time is the MAX over ranks.

Also reported: the dominant kernel's roofline (algorithmic FP64 flops / its average launch
time measured with HIP events on the launch stream) and the CPU oracle timed on this host
(cpu_baseline, rank 0 only).
"""
import argparse
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
SINCOS_RHS = 3
PEAK_FP64_VALU = 78.6   # TFLOP/s, MI355X FP64 vector (spec)
PEAK_HBM = 8000.0       # GB/s (spec)
BYTES_STEP = 170        # algorithmic bytes per env-step


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=128, help="timed steps (a multiple of the 64-step pool refill by default)")
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
    ap.add_argument("--refill-interval", type=int, default=None, help="reset-pool refill interval (steps)")
    ap.add_argument("--systems", default="0",
                    help="select_systems, comma-separated registration indices (default 0, the headline; "
                         "'0,1,2,3' is SURVEY.md 8(d)'s mixed-system divergence check)")
    return ap.parse_args()


def dist_init():
    """One process per GPU (torchrun).  RCCL (backend "nccl") by default.  Rehearsal overrides for
    a one-GPU box: CTR_BENCH_BACKEND=gloo with CTR_BENCH_SAME_DEVICE=1 puts every rank on cuda:0
    (RCCL refuses two ranks on one GPU); the timing logic is the same."""
    import torch
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("CTR_BENCH_SAME_DEVICE") == "1":
        local = 0
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        backend = os.environ.get("CTR_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        return dist, rank, ws, local
    return None, 0, 1, local


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
    """Algorithmic FP64 flops + sincos of one FK per env at the given joints (device counters)."""
    _, st = env.forward_kinematics(joints, env.system, return_stats=True)
    nfev = st["nfev"].double()
    att = (st["nstep"] + st["nrej"]).double()
    seg = st["nseg"].double()
    if env.integrator == "rk4":
        per = nfev * FLOP_RHS + att * FLOP_RK4_STEP
    else:
        per = nfev * FLOP_RHS + att * FLOP_ATTEMPT + seg * FLOP_SEGMENT
    flops = per.sum().item() + FLOP_STEP_EXTRA * joints.shape[0]
    sincos = (nfev * SINCOS_RHS).sum().item()
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
    return {"envs": int(q.shape[0]), "tip_l2_max_m": float(l2.max()), "tip_l2_p999_m": float(np.quantile(l2, 0.999)),
            "reached_flag_agreement": float(agree), "band_m": 1e-6,
            "checker": "oracle/ctr_oracle.c (CPU restatement, pinned to the reference's fixtures)"}


def cpu_baseline(args, cfgd):
    """Oracle (C port, OpenMP) on this host: env-steps/s on a bounded sample of the workload."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.build()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count()
    n = 4096
    q, _ = oracle.sample_joints(n, seed=args.seed, stream=1)
    dg = oracle.fk(oracle.sample_joints(n, seed=args.seed, stream=0)[0], integrator=cfgd["integrator"],
                   steps_per_m=cfgd["rk4_steps_per_m"], model=cfgd["model"])["tip"]
    rng = np.random.default_rng(args.seed + 1)
    hi = np.array([1e-3] * 3 + [np.deg2rad(5)] * 3, np.float32)
    t = np.zeros(n, np.int32)
    steps = 0
    t0 = time.perf_counter()
    while True:
        a = ((rng.random((n, 6)) * 2 - 1) * hi).astype(np.float32)
        r = oracle.step(q, a, dg, t, 0.020, integrator=cfgd["integrator"], steps_per_m=cfgd["rk4_steps_per_m"],
                        model=cfgd["model"])
        q, t = r["joints"], r["t"]
        t[t >= 150] = 0
        steps += 1
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    return {"value": n * steps / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "%d envs x %d steps of oracle/ctr_oracle.c (%s, %s model, fp64), OpenMP %d threads, "
                      "%.1f s" % (n, steps, cfgd["integrator"], cfgd["model"], threads, el)}


def main():
    args = parse()
    import torch
    dist, rank, ws, local = dist_init()
    from ctr_reach_amd import CtrReachVecEnv
    from ctr_reach_amd import distributed as D
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    cfgd = CONFIGS[args.config]
    n = args.envs or cfgd["envs"]
    extra = {} if args.refill_interval is None else {"refill_interval": args.refill_interval}
    systems = [int(s) for s in args.systems.split(",")]
    env = CtrReachVecEnv(n, device=dev, seed=args.seed, env_base=D.shard(n, rank), autoreset=True, record_info=False,
                         integrator=cfgd["integrator"], rk4_steps_per_m=cfgd["rk4_steps_per_m"], model=cfgd["model"],
                         select_systems=systems, **extra)
    env.reset()
    acts = make_actions(env, 8, args.seed + rank)
    stream = torch.cuda.current_stream()

    for i in range(args.warmup):
        env.step_raw(acts[i % len(acts)])
    torch.cuda.synchronize()
    if args.profile_only:
        for i in range(args.steps):
            env.step_raw(acts[i % len(acts)])
        torch.cuda.synchronize()
        return

    # ---- timed region: K whole-job steps (includes auto-resets at their natural rate)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        env.step_raw(acts[i % len(acts)])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el = D.max_over_ranks(time.perf_counter() - t0,
                          device=dev if os.environ.get("CTR_BENCH_BACKEND", "nccl") == "nccl" else "cpu")
    total_steps = n * ws * args.steps

    # ---- dominant kernel (k_step) alone: HIP events on the launch stream, no auto-reset.
    # ctr_step with autoreset = 0 launches exactly one kernel (k_step) on `stream`; one event pair
    # brackets k_iters back-to-back launches (per-launch event pairs add their own few us), so the
    # average includes the ~1.5 us launch boundaries and slightly over-states the kernel time.
    j_probe = env.joints.clone()
    flops_env_step, sincos, nfev_mean = fk_work(env, j_probe)
    from ctr_reach_amd import _abi
    k_iters = max(5, min(args.steps, 32))
    sp = _abi.stream_ptr(stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
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
        return
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
                                                                     "systems %s drawn per reset" % args.systems),
                   "integrator": cfgd["integrator"], "model": cfgd["model"],
                   "rk4_steps_per_m": cfgd["rk4_steps_per_m"] if cfgd["integrator"] == "rk4" else None,
                   "envs_per_gpu": n, "global_envs": n * ws, "parallelism": "env-shard x%d" % ws,
                   "reset_pool": {"depth": env.pool_depth, "refill_interval": env.refill_interval}},
        "roofline": {"bound": "valu", "achieved": achieved_tf, "peak": PEAK_FP64_VALU, "unit": "TFLOP/s",
                     "frac": achieved_tf / PEAK_FP64_VALU, "traffic": None,
                     "kernel": "k_step", "kernel_ms": k_ms,
                     "flops_per_launch": flops_env_step, "sincos_per_launch": sincos,
                     "nfev_per_env_step": nfev_mean,
                     "hbm_gbs_algorithmic": BYTES_STEP * n / (k_ms * 1e-3) / 1e9,
                     "hbm_frac_algorithmic": BYTES_STEP * n / (k_ms * 1e-3) / 1e9 / PEAK_HBM,
                     "note": "bound is the FP64 vector pipe: an adaptive RK45 ODE per lane, no GEMM-shaped work for "
                             "MFMA, ~140 flop/B so HBM is not the limit; peak = MI355X FP64 vector spec; flops = "
                             "SURVEY 8(d) count from device counters (sincos not priced)"},
    }
    tr = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tr):
        with open(tr) as fh:
            t = json.load(fh)
        if t.get("envs") == n and t.get("config", 3) == args.config and systems == [0]:
            out["roofline"]["traffic"] = t.get("bytes_per_launch")
            out["roofline"]["traffic_source"] = "profiles/traffic.json: rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE per k_step"
    if not args.no_cpu_baseline and ws == 1:
        out["parity"] = parity_probe(env, cfgd)
        out["cpu_baseline"] = cpu_baseline(args, cfgd)
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
