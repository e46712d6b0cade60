// ctr_kernels.hip -- HIP kernels + the extern "C" ABI of libctr_reach_amd.so (gfx950).
//
// Kernels (one environment per lane, 256-lane workgroups):
//   k_fk          Model.forward_kinematics for a batch                 (envs/model.py:30-70)
//   k_set_action  n_substeps x Obs.set_action                          (envs/obs.py:166-183)
//   k_step        fused CtrReachEnv.step: set_action x n_substeps, FK, reward, done,
//                 success, error, observation; appends done envs to a reset work list
//                 with one wave-aggregated atomic per wave          (envs/ctr_reach_env.py:124-158)
//   k_reset       CtrReachEnv.reset for listed / masked envs: system pick, two
//                 sample_goal draws (Philox), two FKs, observation   (envs/ctr_reach_env.py:70-114)
//   k_reward      compute_reward over a batch                          (envs/ctr_reach_env.py:160-170)
//
// The tube tables (<= 8 systems x 18 doubles) travel as a kernel argument and are staged
// once per workgroup into LDS; every lane then reads its system's row from LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "ctr_device.hpp"
#include "ctr_reach_amd.h"

using namespace ctr;

namespace {

constexpr int BLOCK = 256;

thread_local char g_err[512] = "";

int fail(int code, const char *msg)
{
    snprintf(g_err, sizeof g_err, "%s", msg);
    return code;
}

int hip_check(const char *what)
{
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
        return CTR_EHIP;
    }
    return 0;
}

// Kernel-argument copy of the config (by value, <= 1.2 KB of kernarg).
struct KCfg {
    ctr_env_config_t c;
    int32_t has_uy;
};

__device__ __forceinline__ void stage_systems(const KCfg &kc, ctr_system_t *lds)
{
    const double *src = reinterpret_cast<const double *>(kc.c.systems);
    double *dst = reinterpret_cast<double *>(lds);
    const int nd = kc.c.n_systems * (int)(sizeof(ctr_system_t) / sizeof(double));
    for (int i = threadIdx.x; i < nd; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

__device__ __forceinline__ int clamp_sys(int s, int n) { return (s < 0 || s >= n) ? 0 : s; }

template <bool HAS_UY>
__device__ __forceinline__ void fk_dispatch(const ctr_system_t &sy, const float q[6], double tip[3], FkStats &st)
{
    fk_lane<HAS_UY>(sy, q, tip, st);
}

// ------------------------------------------------------------------------------------------
template <bool HAS_UY>
__global__ __launch_bounds__(BLOCK) void k_fk(KCfg kc, const float *__restrict__ joints,
                                                 const int32_t *__restrict__ sys_idx, int64_t n,
                                                 double *__restrict__ tip, uint32_t *__restrict__ stats,
                                                 uint32_t *__restrict__ status)
{
    __shared__ ctr_system_t s_sys[CTR_MAX_SYSTEMS];
    stage_systems(kc, s_sys);
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    float q[6];
    #pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = joints[6 * e + i];
    const int s = sys_idx ? clamp_sys(sys_idx[e], kc.c.n_systems) : 0;
    FkStats st = {0, 0, 0, 0, 0};
    double out[3];
    fk_dispatch<HAS_UY>(s_sys[s], q, out, st);
    #pragma unroll
    for (int i = 0; i < 3; ++i) tip[3 * e + i] = out[i];
    if (stats) {
        stats[4 * e + 0] = st.nfev;
        stats[4 * e + 1] = st.nstep;
        stats[4 * e + 2] = st.nrej;
        stats[4 * e + 3] = st.nseg;
    }
    if (status) status[e] = st.status;
}

__global__ __launch_bounds__(BLOCK) void k_set_action(KCfg kc, float *__restrict__ joints,
                                                         const int32_t *__restrict__ sys_idx,
                                                         const float *__restrict__ actions, int64_t n)
{
    __shared__ ctr_system_t s_sys[CTR_MAX_SYSTEMS];
    stage_systems(kc, s_sys);
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    float q[6], a[6];
    #pragma unroll
    for (int i = 0; i < 6; ++i) { q[i] = joints[6 * e + i]; a[i] = actions[6 * e + i]; }
    const int s = sys_idx ? clamp_sys(sys_idx[e], kc.c.n_systems) : 0;
    for (int k = 0; k < kc.c.n_substeps; ++k) set_action_lane(s_sys[s], kc.c.constrain_alpha != 0, q, a);
    #pragma unroll
    for (int i = 0; i < 6; ++i) joints[6 * e + i] = q[i];
}

// ------------------------------------------------------------------------------------------
template <bool HAS_UY>
__global__ __launch_bounds__(BLOCK) void k_step(KCfg kc, ctr_batch_t b, const float *__restrict__ actions,
                                                   ctr_step_out_t o, int32_t autoreset)
{
    __shared__ ctr_system_t s_sys[CTR_MAX_SYSTEMS];
    stage_systems(kc, s_sys);
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    const bool live = e < b.n;
    bool done = false;
    if (live) {
        const int s = clamp_sys(b.system[e], kc.c.n_systems);
        const ctr_system_t &sy = s_sys[s];
        float q[6], a[6];
        #pragma unroll
        for (int i = 0; i < 6; ++i) { q[i] = b.joints[6 * e + i]; a[i] = actions[6 * e + i]; }
        for (int k = 0; k < kc.c.n_substeps; ++k) set_action_lane(sy, kc.c.constrain_alpha != 0, q, a);
        FkStats st = {0, 0, 0, 0, 0};
        double ag[3];
        fk_dispatch<HAS_UY>(sy, q, ag, st);
        const int32_t t = b.t[e] + 1;
        double dg[3];
        #pragma unroll
        for (int i = 0; i < 3; ++i) dg[i] = b.desired_goal[3 * e + i];
        const double dx = ag[0] - dg[0], dy = ag[1] - dg[1], dz = ag[2] - dg[2];
        const double d = sqrt(dx * dx + dy * dy + dz * dz);
        const double tol = kc.c.tol;
        const float reward = (d > tol) ? -1.0f : 0.0f;              // ctr_reach_env.py:170
        done = (reward == 0.0f) || (t >= kc.c.max_steps);           // :140
        const bool multi = kc.c.n_systems > 1;
        const int od = multi ? 14 : 13;
        float obs[14];
        obs_lane(q, dg, ag, tol, s, multi, kc.c.egocentric != 0, obs);
        #pragma unroll
        for (int i = 0; i < 6; ++i) b.joints[6 * e + i] = q[i];
        #pragma unroll
        for (int i = 0; i < 3; ++i) b.achieved_goal[3 * e + i] = ag[i];
        b.t[e] = t;
        #pragma unroll
        for (int i = 0; i < 13; ++i) o.obs[od * e + i] = obs[i];
        if (multi) o.obs[od * e + 13] = obs[13];
        o.reward[e] = reward;
        o.done[e] = done ? 1 : 0;
        o.success[e] = (d < tol) ? 1 : 0;                           // :155
        o.error[e] = (float)d;
        if (o.status) o.status[e] = st.status;
        if (o.nfev) o.nfev[e] = st.nfev;
        if (autoreset && done) {
            if (o.terminal_obs) {
                #pragma unroll
                for (int i = 0; i < 13; ++i) o.terminal_obs[od * e + i] = obs[i];
                if (multi) o.terminal_obs[od * e + 13] = obs[13];
            }
            if (o.terminal_achieved)
                #pragma unroll
                for (int i = 0; i < 3; ++i) o.terminal_achieved[3 * e + i] = ag[i];
        }
    }
    if (autoreset) {
        // wave-aggregated append of done envs to the reset list b.work[1 + slot]
        const uint64_t m = __ballot(live && done);
        if (m) {
            const int lane = threadIdx.x & 63;
            const int leader = __builtin_ctzll(m);
            int base = 0;
            if (lane == leader) base = atomicAdd(&b.work[0], __popcll(m));
            base = __shfl(base, leader);
            if (live && done) {
                const int off = __popcll(m & ((1ull << lane) - 1ull));
                b.work[1 + base + off] = (int32_t)e;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Reset.  Two lanes per environment: the even lane draws the desired joints and runs the goal
// FK (ctr_reach_env.py:100-101), the odd lane draws the start joints and runs the start FK
// (:104-112); the pair then swaps results with a lane shuffle and the odd lane writes the env.
// mode 0: envs from the auto-reset work list (count in work[0]); mode 1: all envs (or mask).
template <bool HAS_UY>
__global__ __launch_bounds__(BLOCK) void k_reset(KCfg kc, ctr_batch_t b, int mode, const uint8_t *__restrict__ mask,
                                                    const double *__restrict__ goal,
                                                    const int32_t *__restrict__ sys_in, float *__restrict__ obs,
                                                    uint32_t *__restrict__ status)
{
    __shared__ ctr_system_t s_sys[CTR_MAX_SYSTEMS];
    __shared__ int s_count;
    if (mode == 0 && threadIdx.x == 0) s_count = b.work[0];
    stage_systems(kc, s_sys);
    const int64_t slot = ((int64_t)blockIdx.x * BLOCK + threadIdx.x) >> 1;
    const bool odd = threadIdx.x & 1;
    int64_t e = -1;
    if (mode == 0) {
        if (slot < s_count) e = b.work[1 + slot];
    } else if (slot < b.n && (!mask || mask[slot])) {
        e = slot;
    }
    const bool active = e >= 0;
    const uint64_t genv = (uint64_t)(b.env_base + (active ? e : 0));
    const uint32_t epoch = active ? b.epoch[e] + 1 : 0;        // reset number of this reset
    const uint64_t seed = kc.c.seed;
    const int ns = kc.c.n_systems;
    const int s = !active ? 0 : sys_in ? clamp_sys(sys_in[e], ns) : sample_system(seed, epoch, genv, ns);
    const ctr_system_t &sy = s_sys[s];
    uint32_t stat = 0;
    float qv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    double tip[3] = {0.0, 0.0, 0.0};
    if (active) {
        const bool sample = odd ? (kc.c.resample_joints != 0) : (goal == nullptr);
        if (sample) {
            if (sample_joints_lane(sy, seed, epoch, odd ? 1u : 0u, genv, qv) > 1000) stat |= CTR_STATUS_SAMPLER_STUCK;
        } else if (odd) {
            #pragma unroll
            for (int k = 0; k < 6; ++k) qv[k] = b.joints[6 * e + k];
        }
        if (!odd && goal) {
            #pragma unroll
            for (int k = 0; k < 3; ++k) tip[k] = goal[3 * e + k];
        } else {
            FkStats st = {0, 0, 0, 0, 0};
            fk_dispatch<HAS_UY>(sy, qv, tip, st);                 // :101 (even) / :108, :112 (odd)
            stat |= st.status;
        }
    }
    // exchange within the pair (all lanes of the wave are converged here)
    double other[3];
    #pragma unroll
    for (int k = 0; k < 3; ++k) other[k] = __shfl_xor(tip[k], 1);
    float qother[6];
    #pragma unroll
    for (int k = 0; k < 6; ++k) qother[k] = __shfl_xor(qv[k], 1);
    const uint32_t stat_other = __shfl_xor(stat, 1);
    if (!active) return;
    if (!odd) {
        if (b.desired_joints)
            #pragma unroll
            for (int k = 0; k < 6; ++k) b.desired_joints[6 * e + k] = qv[k];
        return;
    }
    const double *dg = other;        // from the even lane
    const double *ag = tip;
    (void)qother;
    #pragma unroll
    for (int k = 0; k < 6; ++k) b.joints[6 * e + k] = qv[k];
    #pragma unroll
    for (int k = 0; k < 3; ++k) { b.desired_goal[3 * e + k] = dg[k]; b.achieved_goal[3 * e + k] = ag[k]; }
    b.t[e] = 0;
    b.system[e] = s;
    b.epoch[e] = epoch;
    if (b.starting_joints)
        #pragma unroll
        for (int k = 0; k < 6; ++k) b.starting_joints[6 * e + k] = qv[k];
    if (b.starting_position)
        #pragma unroll
        for (int k = 0; k < 3; ++k) b.starting_position[3 * e + k] = ag[k];
    const bool multi = ns > 1;
    const int od = multi ? 14 : 13;
    float ob[14];
    obs_lane(qv, dg, ag, kc.c.tol, s, multi, kc.c.egocentric != 0, ob);   // :114
    #pragma unroll
    for (int k = 0; k < 13; ++k) obs[od * e + k] = ob[k];
    if (multi) obs[od * e + 13] = ob[13];
    if (status) status[e] |= stat | stat_other;
}

__global__ __launch_bounds__(BLOCK) void k_clear_work(int32_t *work)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) work[0] = 0;
}

__global__ __launch_bounds__(BLOCK) void k_reward(const double *__restrict__ ag, const double *__restrict__ dg,
                                                     int64_t n, double tol, float *__restrict__ reward)
{
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    const double dx = ag[3 * e] - dg[3 * e], dy = ag[3 * e + 1] - dg[3 * e + 1], dz = ag[3 * e + 2] - dg[3 * e + 2];
    reward[e] = (sqrt(dx * dx + dy * dy + dz * dz) > tol) ? -1.0f : 0.0f;
}

int check_cfg(const ctr_env_config_t *cfg)
{
    if (!cfg) return fail(CTR_EINVAL, "cfg is NULL");
    if (cfg->n_systems < 1 || cfg->n_systems > CTR_MAX_SYSTEMS) return fail(CTR_EINVAL, "n_systems out of range");
    if (cfg->n_substeps < 0) return fail(CTR_EINVAL, "n_substeps < 0");
    if (cfg->integrator != CTR_INTEGRATOR_RK45_SCIPY) return fail(CTR_EINVAL, "integrator not supported yet");
    return 0;
}

KCfg make_kcfg(const ctr_env_config_t *cfg)
{
    KCfg kc;
    memcpy(&kc.c, cfg, sizeof *cfg);
    kc.has_uy = 0;
    for (int s = 0; s < cfg->n_systems; ++s)
        for (int i = 0; i < 3; ++i)
            if (cfg->systems[s].Uy[i] != 0.0) kc.has_uy = 1;
    return kc;
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

}  // namespace

extern "C" {

int ctr_abi_version(void) { return CTR_ABI_VERSION; }

const char *ctr_last_error(void) { return g_err; }

int ctr_fk(const float *joints, const int32_t *sys_idx, int64_t n, const ctr_env_config_t *cfg, double *tip,
           uint32_t *stats, uint32_t *status, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (n < 0 || (n > 0 && (!joints || !tip))) return fail(CTR_EINVAL, "ctr_fk: bad buffers");
    if (n == 0) return 0;
    KCfg kc = make_kcfg(cfg);
    hipStream_t s = (hipStream_t)stream;
    if (kc.has_uy)
        hipLaunchKernelGGL(k_fk<true>, dim3(grid_for(n)), dim3(BLOCK), 0, s, kc, joints, sys_idx, n, tip, stats, status);
    else
        hipLaunchKernelGGL(k_fk<false>, dim3(grid_for(n)), dim3(BLOCK), 0, s, kc, joints, sys_idx, n, tip, stats, status);
    return hip_check("ctr_fk launch");
}

int ctr_set_action(const ctr_env_config_t *cfg, float *joints, const int32_t *sys_idx, const float *actions,
                   int64_t n, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (n < 0 || (n > 0 && (!joints || !actions))) return fail(CTR_EINVAL, "ctr_set_action: bad buffers");
    if (n == 0) return 0;
    KCfg kc = make_kcfg(cfg);
    hipLaunchKernelGGL(k_set_action, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, kc, joints, sys_idx,
                       actions, n);
    return hip_check("ctr_set_action launch");
}

int ctr_step(const ctr_env_config_t *cfg, const ctr_batch_t *batch, const float *actions, const ctr_step_out_t *out,
             int32_t autoreset, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (!batch || !out || !actions) return fail(CTR_EINVAL, "ctr_step: NULL argument");
    const ctr_batch_t b = *batch;
    const ctr_step_out_t o = *out;
    if (b.n < 0) return fail(CTR_EINVAL, "ctr_step: n < 0");
    if (b.n == 0) return 0;
    if (!b.joints || !b.desired_goal || !b.achieved_goal || !b.t || !b.system || !b.epoch)
        return fail(CTR_EINVAL, "ctr_step: batch buffer missing");
    if (!o.obs || !o.reward || !o.done || !o.success || !o.error) return fail(CTR_EINVAL, "ctr_step: output missing");
    if (autoreset && !b.work) return fail(CTR_EINVAL, "ctr_step: autoreset needs batch->work");
    KCfg kc = make_kcfg(cfg);
    hipStream_t s = (hipStream_t)stream;
    const unsigned g = grid_for(b.n), g2 = grid_for(2 * b.n);
    if (autoreset) hipLaunchKernelGGL(k_clear_work, dim3(1), dim3(64), 0, s, b.work);
    if (kc.has_uy)
        hipLaunchKernelGGL(k_step<true>, dim3(g), dim3(BLOCK), 0, s, kc, b, actions, o, autoreset);
    else
        hipLaunchKernelGGL(k_step<false>, dim3(g), dim3(BLOCK), 0, s, kc, b, actions, o, autoreset);
    if (int r = hip_check("ctr_step launch")) return r;
    if (autoreset) {
        if (kc.has_uy)
            hipLaunchKernelGGL(k_reset<true>, dim3(g2), dim3(BLOCK), 0, s, kc, b, 0, nullptr, nullptr, nullptr, o.obs,
                               o.status);
        else
            hipLaunchKernelGGL(k_reset<false>, dim3(g2), dim3(BLOCK), 0, s, kc, b, 0, nullptr, nullptr, nullptr, o.obs,
                               o.status);
        return hip_check("ctr_step reset launch");
    }
    return 0;
}

int ctr_reset(const ctr_env_config_t *cfg, const ctr_batch_t *batch, const uint8_t *mask, const double *goal,
              const int32_t *system, float *obs, uint32_t *status, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (!batch || !obs) return fail(CTR_EINVAL, "ctr_reset: NULL argument");
    const ctr_batch_t b = *batch;
    if (b.n < 0) return fail(CTR_EINVAL, "ctr_reset: n < 0");
    if (b.n == 0) return 0;
    if (!b.joints || !b.desired_goal || !b.achieved_goal || !b.t || !b.system || !b.epoch)
        return fail(CTR_EINVAL, "ctr_reset: batch buffer missing");
    KCfg kc = make_kcfg(cfg);
    hipStream_t s = (hipStream_t)stream;
    if (kc.has_uy)
        hipLaunchKernelGGL(k_reset<true>, dim3(grid_for(2 * b.n)), dim3(BLOCK), 0, s, kc, b, 1, mask, goal, system, obs,
                           status);
    else
        hipLaunchKernelGGL(k_reset<false>, dim3(grid_for(2 * b.n)), dim3(BLOCK), 0, s, kc, b, 1, mask, goal, system, obs,
                           status);
    return hip_check("ctr_reset launch");
}

int ctr_compute_reward(const double *achieved, const double *desired, int64_t n, double tol, float *reward,
                       void *stream)
{
    if (n < 0 || (n > 0 && (!achieved || !desired || !reward))) return fail(CTR_EINVAL, "ctr_compute_reward: bad buffers");
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_reward, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, achieved, desired, n, tol,
                       reward);
    return hip_check("ctr_compute_reward launch");
}

}  // extern "C"
