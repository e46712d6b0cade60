"""Time the UNMODIFIED reference CtrReachEnv.step() on this container's CPU (authoring container
only -- /root/reference does not exist on the GPU box).  Uses the same offline shims as
tests/golden/make_golden.py.  Writes profiles/cpu_reference_<tag>.json.

usage: python tools/time_reference.py [tag] [seconds]
"""
import json
import multiprocessing as mp
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def run(seconds, seed, q):
    import numpy as np
    import make_golden as mg
    CtrReachEnv, kwargs = mg.load_reference()
    env = CtrReachEnv(**kwargs)
    np.random.seed(seed)
    env.action_space.np_random = np.random.RandomState(seed)
    for s in env.trig_obj.joint_sample_spaces:
        s.np_random = np.random.RandomState(seed + 1)
    env.reset()
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, _, done, _ = env.step(env.action_space.sample())
        steps += 1
        if done or env.t >= 150:
            env.reset()
    q.put((steps, time.perf_counter() - t0))


def measure(procs, seconds):
    q = mp.Queue()
    ps = [mp.Process(target=run, args=(seconds, 100 + i, q)) for i in range(procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    return sum(s for s, _ in res) / max(t for _, t in res)


def time_port(threads, seconds):
    """The C restatement (oracle/, bench.py's cpu_baseline leg) on this same CPU, so the GPU box's
    cpu_baseline (kind "port") can be read against the reference: env-steps/s."""
    code = ("import sys, json, types; sys.path.insert(0, %r); import bench; "
            "a = types.SimpleNamespace(seed=0, cpu_seconds=%r); "
            "print(json.dumps(bench.cpu_baseline(a, bench.CONFIGS[3])))" % (ROOT, seconds))
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = subprocess.check_output([sys.executable, "-c", code], env=env, text=True)
    return json.loads(out.strip().splitlines()[-1])["value"]


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    sec = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
    cpu = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    out = {"what": "reference CtrReachEnv.step() (scipy solve_ivp RK45), default CTR-Reach-v0 kwargs, random "
                   "actions, resets at their natural rate (included)",
           "cpu": cpu, "nproc": os.cpu_count(), "python": platform.python_version(), "seconds": sec,
           "env_steps_per_s_1proc": measure(1, sec), "env_steps_per_s_nproc": measure(os.cpu_count(), sec),
           "port_env_steps_per_s_1thread": time_port(1, sec),
           "port_env_steps_per_s_nthreads": time_port(os.cpu_count(), sec)}
    out["port_over_reference_1core"] = out["port_env_steps_per_s_1thread"] / out["env_steps_per_s_1proc"]
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "cpu_reference_%s.json" % tag), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))
