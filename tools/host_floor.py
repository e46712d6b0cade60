"""Host-side floor of one CtrReachVecEnv.step_raw (ctypes call + ctr_step's launches) next to the
GPU time of the same steps: tiny batches, where the kernels take a few microseconds.

usage: python tools/host_floor.py [--envs N] [--steps K] [--config 2|3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-ctr-reach_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--config", type=int, default=2)
    a = ap.parse_args()
    import torch
    import bench
    from ctr_reach_amd import CtrReachVecEnv
    c = bench.CONFIGS[a.config]
    env = CtrReachVecEnv(a.envs, device="cuda", seed=0, record_info=False, integrator=c["integrator"],
                         rk4_steps_per_m=c["rk4_steps_per_m"], model=c["model"])
    env.reset()
    acts = bench.make_actions(env, 8, 0)
    for i in range(50):
        env.step_raw(acts[i % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        env.step_raw(acts[i % 8])
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print("envs %d config %d: host enqueue %.2f us/step, enqueue+drain %.2f us/step"
          % (a.envs, a.config, t_host / a.steps * 1e6, t_all / a.steps * 1e6))
    # breakdown of the host part
    import ctypes
    from ctr_reach_amd import _abi
    K = a.steps

    def per(fn):
        t = time.perf_counter()
        for _ in range(K):
            fn()
        return (time.perf_counter() - t) / K * 1e6
    empty = _abi.CtrBatch.from_buffer_copy(env._batch)
    empty.n = 0
    sp = _abi.stream_ptr()
    print("  stream_ptr() %.2f us, ptr(actions) %.2f us, ctypes+checks (n = 0) %.2f us, "
          "ctr_step with cached args %.2f us" % (
              per(lambda: _abi.stream_ptr()), per(lambda: _abi.ptr(acts[0])),
              per(lambda: env.lib.ctr_step(env.cfg, empty, _abi.ptr(acts[0]), env._out, 1, sp)),
              per(lambda: env.lib.ctr_step(env.cfg, env._batch, _abi.ptr(acts[0]), env._out, 1, sp))))
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
