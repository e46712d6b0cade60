// ctr_kernels.hip -- HIP kernels + the extern "C" ABI of libctr_reach_amd.so (gfx950).
//
// Kernels (one environment per lane unless stated, 256-lane workgroups):
//   k_fk          Model.forward_kinematics for a batch                 (envs/model.py:30-70)
//   k_set_action  n_substeps x Obs.set_action                          (envs/obs.py:166-183)
//   k_step        fused CtrReachEnv.step: set_action x n_substeps, FK, reward, done,
//                 success, error, observation; a done env takes its next reset from the
//                 reset pool (a copy), or is queued for k_reset      (envs/ctr_reach_env.py:124-158);
//                 rigid model + fixed-step RK4: one env per 8-lane group (fk_group_rigid4)
//   k_reset       CtrReachEnv.reset, TWO lanes per env (goal FK | start FK in parallel),
//                 for the queued / masked envs                        (envs/ctr_reach_env.py:70-114)
//   k_refill      precomputes queued resets into the pool, two lanes per reset
//   k_reward      compute_reward over a batch                          (envs/ctr_reach_env.py:160-170)
//   k_fk_shape    FK + backbone shape r at 30 dense-output points/segment (envs/model.py:66-68,119-174)
//   k_jacobian    forward-difference tip Jacobian, 7 lanes per env       (CTR_Python/CTR_Model.py:251-262)
//   k_domain_params  each env's current (domain-randomised) tube table  (envs/model.py:20-28)
//   k_her_*       HER replay feed: episode recording, row prefix sums, relabelled uniform
//                 sampling by inverse CDF (ctr_her.inc)
//
// Work lists (auto-reset misses, pool refills) are appended with one wave-aggregated atomic per
// wave.  The tube tables (<= 8 systems x 18 doubles) travel as a kernel argument and are staged
// once per workgroup into LDS; every lane then reads its system's row from LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

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

// Kernel-argument copy of the config (by value, ~2.7 KB of kernarg).
// sysk: every system's SysK divisions (kz[3], inv[8], sysk_derive's arithmetic, correctly rounded
// IEEE divisions and sums, so host and device give the same bits), computed once by make_kcfg
// on the host: the workgroups copy them with the system rows instead of deriving them behind a
// barrier of their own.
constexpr int SYSK_ND = (int)(sizeof(ctr_system_t) / sizeof(double)) + 11;   // rows + kz + inv
struct KCfg {
    ctr_env_config_t c;
    int32_t mode;       // fk_dispatch MODE bits
    double sysk[CTR_MAX_SYSTEMS][11];
};

// LUT = false: skip the per-description segment table (SysK::lut stays NULL; seg_par_at then
// derives the row itself), for kernels whose FK never reads it (the rigid 8-lane group path).
// The workgroup's table inputs in registers: this lane's four trig-table entries, its element of
// the system rows and of the raw tube rows (<= 8 x 18 and 8 x 12 doubles, one per lane of a
// 256-lane workgroup).  stage_load issues the loads; a kernel may issue its own loads before
// stage_systems stores them, so both latencies overlap.
struct StageRegs {
    TrigRegs trig;
    double sys, raw;
};

static_assert(offsetof(SysK, kz) == sizeof(ctr_system_t) && offsetof(SysK, inv) == offsetof(SysK, kz) + 3 * sizeof(double),
              "SysK: the rows, kz and inv contiguous (one copy image)");

// Element k of system s's SysK image (the table row, then kz and inv from the kernel config).
__device__ __forceinline__ double sysk_elem(const KCfg &kc, int s, int k)
{
    constexpr int ND = (int)(sizeof(ctr_system_t) / sizeof(double));
    return k < ND ? reinterpret_cast<const double *>(&kc.c.systems[s])[k] : kc.sysk[s][k - ND];
}

__device__ __forceinline__ void stage_load(const KCfg &kc, StageRegs &r)
{
    constexpr int NR = (int)(sizeof(ctr_tube_raw_t) / sizeof(double));
    static_assert(CTR_MAX_SYSTEMS * SYSK_ND <= BLOCK && CTR_MAX_SYSTEMS * NR <= BLOCK, "one element per lane");
    trig_table_load(r.trig);
    const int i = (int)threadIdx.x;
    const int j = i < kc.c.n_systems * SYSK_ND ? i : 0;
    r.sys = sysk_elem(kc, j / SYSK_ND, j % SYSK_ND);
    r.raw = reinterpret_cast<const double *>(kc.c.raw)[i < kc.c.n_systems * NR ? i : 0];
}

// pre: the inputs already loaded (stage_load).
template <bool LUT = true>
__device__ __forceinline__ void stage_systems(const KCfg &kc, SysK *lds, ctr_tube_raw_t *raw_lds = nullptr,
                                              const StageRegs *pre = nullptr)
{
    constexpr int NR = (int)(sizeof(ctr_tube_raw_t) / sizeof(double));
    // seg_par of every (system, 6-bit gap description): SysK::lut, read at segment starts
    __shared__ double s_lut[CTR_MAX_SYSTEMS][64][8];
    const int nd = kc.c.n_systems * SYSK_ND;
    if (pre) {
        // unconditional stores (lanes past the rows write a dummy slot): a conditional store would
        // let the compiler sink its load behind the caller's loads
        __shared__ double s_stage_dummy[BLOCK];
        const int i = (int)threadIdx.x;
        double *ds = i < nd ? reinterpret_cast<double *>(&lds[i / SYSK_ND]) + i % SYSK_ND : &s_stage_dummy[i];
        *ds = pre->sys;
        trig_table_store(pre->trig);
        if (raw_lds) *(i < kc.c.n_systems * NR ? reinterpret_cast<double *>(raw_lds) + i : &s_stage_dummy[i]) = pre->raw;
    } else {
        for (int i = threadIdx.x; i < nd; i += blockDim.x)
            reinterpret_cast<double *>(&lds[i / SYSK_ND])[i % SYSK_ND] = sysk_elem(kc, i / SYSK_ND, i % SYSK_ND);
        trig_table_fill();
        if (raw_lds) {
            const double *rs = reinterpret_cast<const double *>(kc.c.raw);
            for (int i = threadIdx.x; i < kc.c.n_systems * NR; i += blockDim.x)
                reinterpret_cast<double *>(raw_lds)[i] = rs[i];
        }
    }
    for (int i = threadIdx.x; i < kc.c.n_systems; i += blockDim.x) lds[i].lut = LUT ? &s_lut[i][0][0] : nullptr;
    if (LUT) {
        // the table rows from the kernel config (wave-uniform system: scalar loads), not from the
        // LDS copy above, so the workgroup needs one barrier for both
        for (int i = threadIdx.x; i < kc.c.n_systems * 64; i += blockDim.x) {
            const int sy = i / 64;
            SysK t;
            #pragma unroll
            for (int j = 0; j < 3; ++j) {
                t.EI[j] = kc.c.systems[sy].EI[j];
                t.Ux[j] = kc.c.systems[sy].Ux[j];
                t.Uy[j] = kc.c.systems[sy].Uy[j];
                t.kz[j] = kc.sysk[sy][j];
            }
            // inv read by its dynamic index from the kernel config, not from t (a dynamic index
            // into the private copy put it in scratch: 72 B per lane written back to HBM)
            SegPar q = seg_par_inv(t, (uint32_t)(i % 64), false, kc.sysk[sy][3 + (i & 7)]);
            seg_fold_inv(q);
            double *e = s_lut[sy][i % 64];
            for (int j = 0; j < 3; ++j) { e[j] = q.wx[j]; e[3 + j] = q.g[j]; }
            e[6] = q.inv;
            e[7] = (double)q.present;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ int clamp_sys(int s, int n) { return (s < 0 || s >= n) ? 0 : s; }

// Per-lane tube tables for domain randomisation: dynamic LDS, BLOCK entries (launched with
// lane_lds_bytes(kc), 0 when randomisation is off).
extern __shared__ SysK s_lane_dyn[];

__host__ __device__ inline size_t lane_lds_bytes(const KCfg &kc)
{
    return kc.c.domain_rand != 0.0 ? (size_t)BLOCK * sizeof(SysK) : 0;
}

// The tube table episode `epoch` of env `genv` integrates with: the system row, or with domain
// randomisation the lane's re-sampled table (epoch 0 = before the first reset: the nominal
// table, as the reference constructor's FK, ctr_reach_env.py:65).
// slot: this env's entry of the dynamic LDS table (the lane; both lanes of a k_step_pair env
// share one and store the same values).
__device__ __forceinline__ const SysK &episode_sys_at(const KCfg &kc, const SysK *s_sys, const ctr_tube_raw_t *s_raw,
                                                      int s, uint32_t epoch, uint64_t genv, int slot)
{
    if (kc.c.domain_rand == 0.0 || epoch == 0) return s_sys[s];
    SysK &me = s_lane_dyn[slot];
    domain_system(s_sys[s], s_raw[s], kc.c.domain_rand, kc.c.seed, epoch, genv, me, nullptr);
    #pragma unroll
    for (int j = 0; j < 11; ++j) sysk_derive(me, j);
    me.lut = nullptr;
    return me;
}

__device__ __forceinline__ const SysK &episode_sys(const KCfg &kc, const SysK *s_sys, const ctr_tube_raw_t *s_raw,
                                                   int s, uint32_t epoch, uint64_t genv)
{
    if (kc.c.domain_rand == 0.0 || epoch == 0) return s_sys[s];
    SysK &me = s_lane_dyn[threadIdx.x];
    domain_system(s_sys[s], s_raw[s], kc.c.domain_rand, kc.c.seed, epoch, genv, me, nullptr);
    #pragma unroll
    for (int j = 0; j < 11; ++j) sysk_derive(me, j);
    me.lut = nullptr;
    return me;
}

// MODE bits: 1 = some tube has y pre-curvature, 2 = fixed-step RK4 (else scipy RK45),
// 4 = torsionally rigid model.
template <int MODE>
__device__ __forceinline__ void fk_dispatch_d(const KCfg &kc, const SysK &sy, const double qd[6], double tip[3],
                                              FkStats &st)
{
    constexpr bool UY = (MODE & 1) != 0, RG = (MODE & 4) != 0;
    const bool careful = fk_needs_careful_trig(qd);
    if (MODE & 2) {
        if (careful) fk_lane_rk4<UY, RG, true>(sy, qd, tip, st, (double)kc.c.rk4_steps_per_m);
        else fk_lane_rk4<UY, RG, false>(sy, qd, tip, st, (double)kc.c.rk4_steps_per_m);
    } else {
        if (careful) fk_lane<UY, RG, false, true>(sy, qd, tip, st);
        else fk_lane<UY, RG, false, false>(sy, qd, tip, st);
    }
}

// Model.forward_kinematics widens the float32 joints of Obs to float64 (model.py:48-62).
template <int MODE>
__device__ __forceinline__ void fk_dispatch(const KCfg &kc, const SysK &sy, const float q[6], double tip[3],
                                            FkStats &st)
{
    const double qd[6] = {(double)q[0], (double)q[1], (double)q[2], (double)q[3], (double)q[4], (double)q[5]};
    fk_dispatch_d<MODE>(kc, sy, qd, tip, st);
}

// Wave-aggregated append of `n_items` int32 per active lane to a list (one atomic per wave).
__device__ __forceinline__ void wave_append(int32_t *counter, int32_t *items_base, int64_t cap, bool active,
                                            const int32_t *items, int n_items)
{
    const uint64_t m = __ballot(active);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    const int leader = __builtin_ctzll(m);
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(m));
    base = __shfl(base, leader);
    if (active) {
        const int64_t slot = base + __popcll(m & ((1ull << lane) - 1ull));
        if (slot < cap)
            for (int k = 0; k < n_items; ++k) items_base[n_items * slot + k] = items[k];
    }
}

// Auto-reset miss list: counters work[0] / work[1] alternate between steps (work_parity) so the
// consumer of one step's list can zero the next step's counter without a separate launch.
__device__ __forceinline__ int32_t *miss_counter(const ctr_batch_t &b) { return b.work + (b.work_parity & 1); }
__device__ __forceinline__ int32_t *miss_items(const ctr_batch_t &b) { return b.work + 2; }

// The fused push gather (ctr_step_out_t.gather): env e's packed row into every rank's receive
// slot (IPC-mapped peer memory; the descriptor's pointers are wave-uniform scalar loads) with
// system-scope stores (sc0 sc1: written through, not held in this GPU's L2), then one wait for
// all of them (gather_rows_performed): the rows are performed at system scope before the wave
// ends, with no L2 write-back.  (A system-scope release fence per wave did the same through a
// write-back of the whole XCD L2: +15 us per step, tools/gather_interference.py.)  The stores are
// inline asm, invisible to the compiler's wait counting: the caller waits for them right after
// (vmcnt(0): nothing is in flight afterwards, so the compiler's later waits stay conservative).
typedef unsigned int row16_t __attribute__((ext_vector_type(4)));   // one packed row

__device__ __forceinline__ void gather_store_row(const ctr_gather_push_t *g, int64_t e, float4 row)
{
    const row16_t v = {__float_as_uint(row.x), __float_as_uint(row.y), __float_as_uint(row.z),
                       __float_as_uint(row.w)};
    const int W = g->world;
    for (int k = 0; k < W; ++k) {
        row16_t *dst = static_cast<row16_t *>(g->dst[k]) + e;
        // the s_nop inside the statement: a VALU write of a > 8-byte store's data VGPRs needs wait
        // states after the store, and the compiler's hazard recognizer cannot see into the asm
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" : : "v"(dst), "v"(v) : "memory");
    }
}

__device__ __forceinline__ void gather_rows_performed()
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Lane k < world publishes seq into rank k's sequence word (a system-scope store).  Called only
// after the kernel that pushed step seq has completed, whose waves each waited for their rows'
// system-scope stores: the rows are performed, so a relaxed store orders after them (a release
// would add a write-back of this XCD's L2 at the start of every step).
__device__ __forceinline__ void gather_publish_lane(const ctr_gather_push_t *g, uint32_t seq)
{
    if ((int)threadIdx.x < g->world)
        __hip_atomic_store(g->seqw[threadIdx.x], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Sequence numbers wrap modulo 2^32: a has reached b.
__device__ __forceinline__ bool seq_reached(uint32_t a, uint32_t b) { return (int32_t)(a - b) >= 0; }

// Fused push flow control (include/ctr_reach_amd.h, "Push all-gather"): lane k < world stores
// `released` into this rank's release word in rank k's memory (a system-scope store; the
// launch's stream predecessors, which held this rank's reads of the released slot, are complete).
__device__ __forceinline__ void gather_release_lane(const ctr_gather_push_t *g, uint32_t released)
{
    if ((int)threadIdx.x < g->world)
        __hip_atomic_store(g->relw[threadIdx.x], released, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// This lane's release word of consumer (lane) -- ~0u for lanes >= world (always free).
__device__ __forceinline__ uint32_t gather_release_load(const ctr_gather_push_t *g, uint32_t seq)
{
    const int lane = (int)(threadIdx.x & 63);
    return lane < g->world ? __hip_atomic_load(g->rel + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                           : seq - (uint32_t)g->depth;
}

// Wave-uniform: every consumer has released the slot step seq rewrites (step seq - depth).
// Call with every lane of the wave active.
__device__ __forceinline__ bool gather_slot_free(const ctr_gather_push_t *g, uint32_t seq, uint32_t rel)
{
    return __ballot(!seq_reached(rel, seq - (uint32_t)g->depth)) == 0;
}

// Bounded waits have a wall-clock budget: s_memrealtime counts at 100 MHz.
__device__ __forceinline__ bool wait_expired(uint64_t t0, uint32_t wait_us)
{
    return __builtin_amdgcn_s_memrealtime() - t0 >= (uint64_t)wait_us * 100u;
}

// Bounded wait (every lane active) for the slot of step seq; false after wait_us microseconds.
__device__ __noinline__ bool gather_wait_slot(const ctr_gather_push_t *g, uint32_t seq)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (gather_slot_free(g, seq, gather_release_load(g, seq))) return true;
        if (wait_expired(t0, g->wait_us)) return false;
        __builtin_amdgcn_s_sleep(8);
    }
}

// The release wait of step seq timed out: lane c < world whose consumer c has not released the
// slot stores seq into this rank's poison word in c's memory (system scope), and the wave waits
// for those stores before any of its rows overwrite the slot -- so a consumer that reads its
// poison words after reading a view sees every overwrite that reached it (include/ctr_reach_amd.h).
__device__ __noinline__ void gather_poison_lanes(const ctr_gather_push_t *g, uint32_t seq)
{
    const int lane = (int)(threadIdx.x & 63);
    // a NULL poison word: not enabled for that consumer (a C caller that left the ABI-14 fields
    // zeroed gets only its own err bit).  The stored marker is never 0 (0 = not poisoned), also
    // when the step counter has wrapped to 0.
    if (lane < g->world && g->poisonw[lane] != nullptr &&
        !seq_reached(__hip_atomic_load(g->rel + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                     seq - (uint32_t)g->depth))
        __hip_atomic_store(g->poisonw[lane], seq ? seq : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The fused consumer wait (ctr_step_out_t.gather_wait_prev): lane k < world polls this rank's
// sequence word of rank k's block of the previous slot until it reaches seq (system-scope loads;
// the slot's readers are later kernels, and the ring is uncached: no stale line to invalidate);
// bounded, errors into g->err.
__device__ __noinline__ void gather_wait_prev_lane(const ctr_gather_push_t *g, uint32_t seq)
{
    const int lane = (int)threadIdx.x;
    if (lane >= g->world) return;
    // producer `lane` overran a slot of this rank before (its poison word): the views this rank
    // read before this launch may hold rows of a later step
    if (g->poison != nullptr && __hip_atomic_load(g->poison + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
        atomicOr(g->err, CTR_GATHER_E_RELEASE_TIMEOUT);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        const uint32_t v = __hip_atomic_load(g->wait_seqw + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (seq_reached(v, seq)) {
            if (v != seq) atomicOr(g->err, CTR_GATHER_E_OVERWRITTEN);
            return;
        }
        if (wait_expired(t0, g->wait_us)) {
            atomicOr(g->err, CTR_GATHER_E_PREV_TIMEOUT);
            return;
        }
        __builtin_amdgcn_s_sleep(8);
    }
}

// Row e of an observation buffer: float32 [n][od] or, with cfg.obs_f64, float64 [n][od].
__device__ __forceinline__ void write_obs(void *base, int64_t e, const double ob[14], bool multi, bool f64)
{
    const int od = multi ? 14 : 13;
    if (f64) {
        double *dst = static_cast<double *>(base) + od * e;
        #pragma unroll
        for (int k = 0; k < 13; ++k) dst[k] = ob[k];
        if (multi) dst[13] = ob[13];
    } else {
        float *dst = static_cast<float *>(base) + od * e;
        #pragma unroll
        for (int k = 0; k < 13; ++k) dst[k] = (float)ob[k];
        if (multi) dst[13] = (float)ob[13];
    }
}

__device__ __forceinline__ void obs_to_f32(const double ob[14], float out[14])
{
    #pragma unroll
    for (int k = 0; k < 14; ++k) out[k] = (float)ob[k];
}

// ------------------------------------------------------------------------------------------
// tables != NULL: row e integrates with its own tube table tables[e] (staged per lane in LDS).
template <int MODE>
__global__ __launch_bounds__(BLOCK) void k_fk(KCfg kc, const float *__restrict__ joints,
                                                 const int32_t *__restrict__ sys_idx,
                                                 const ctr_system_t *__restrict__ tables, int64_t n,
                                                 double *__restrict__ tip, uint32_t *__restrict__ stats,
                                                 uint32_t *__restrict__ status)
{
    __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
    stage_systems(kc, s_sys);
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    float q[6];
    #pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = joints[6 * e + i];
    const int s = sys_idx ? clamp_sys(sys_idx[e], kc.c.n_systems) : 0;
    const SysK *sy = &s_sys[s];
    if (tables) {
        SysK &me = s_lane_dyn[threadIdx.x];
        static_cast<ctr_system_t &>(me) = tables[e];
        #pragma unroll
        for (int j = 0; j < 11; ++j) sysk_derive(me, j);
        sy = &me;
    }
    FkStats st = {0, 0, 0, 0, 0};
    double out[3];
    fk_dispatch<MODE>(kc, *sy, q, out, st);
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


// Backbone shape (model.py:66-68, 119-174): the FK plus r at the 30 t_eval points of every
// segment from the RK45 dense output.  Row e writes r[e][cap][3], s[e][cap], npts[e].
template <int MODE>
__global__ __launch_bounds__(BLOCK) void k_fk_shape(KCfg kc, const float *__restrict__ joints,
                                                       const int32_t *__restrict__ sys_idx,
                                                       const ctr_system_t *__restrict__ tables, int64_t n, int32_t cap,
                                                       double *__restrict__ tip, double *__restrict__ r,
                                                       double *__restrict__ s_out, int32_t *__restrict__ npts,
                                                       uint32_t *__restrict__ status)
{
    if constexpr ((MODE & 2) == 0) {          // RK45 only (the host rejects RK4)
        __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
        stage_systems(kc, s_sys);
        const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
        if (e >= n) return;
        double q[6];
        #pragma unroll
        for (int i = 0; i < 6; ++i) q[i] = (double)joints[6 * e + i];
        const int s = sys_idx ? clamp_sys(sys_idx[e], kc.c.n_systems) : 0;
        const SysK *sy = &s_sys[s];
        if (tables) {
            SysK &me = s_lane_dyn[threadIdx.x];
            static_cast<ctr_system_t &>(me) = tables[e];
            #pragma unroll
            for (int j = 0; j < 11; ++j) sysk_derive(me, j);
            me.lut = nullptr;
            sy = &me;
        }
        FkStats st = {0, 0, 0, 0, 0};
        ShapeOut so = {r + (int64_t)3 * cap * e, s_out + (int64_t)cap * e, cap, 0};
        double out[3];
        if (fk_needs_careful_trig(q)) fk_lane<(MODE & 1) != 0, (MODE & 4) != 0, true, true>(*sy, q, out, st, &so);
        else fk_lane<(MODE & 1) != 0, (MODE & 4) != 0, true, false>(*sy, q, out, st, &so);
        #pragma unroll
        for (int i = 0; i < 3; ++i) tip[3 * e + i] = out[i];
        npts[e] = so.count;
        if (status) status[e] = st.status;
    }
}

// Forward-difference tip Jacobian, SEVEN lanes per environment: lane c < 6 integrates the FK at
// q + eps e_c, lane 6 at q (CTR_Model.jac, CTR_Python/CTR_Model.py:251-262, applied to this
// env's FK); the base tip is exchanged through LDS.  36 envs per 256-lane workgroup.
constexpr int JAC_ENVS = BLOCK / 7;

template <int MODE>
__global__ __launch_bounds__(BLOCK) void k_jacobian(KCfg kc, const double *__restrict__ joints,
                                                       const int32_t *__restrict__ sys_idx, int64_t n, double eps,
                                                       double *__restrict__ tip, double *__restrict__ jac,
                                                       uint32_t *__restrict__ status)
{
    __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
    __shared__ double s_tip[3][BLOCK];
    stage_systems(kc, s_sys);
    const int slot = threadIdx.x / 7, col = threadIdx.x % 7;
    const int64_t e = (int64_t)blockIdx.x * JAC_ENVS + slot;
    const bool active = slot < JAC_ENVS && e < n;
    double r[3] = {0.0, 0.0, 0.0};
    FkStats st = {0, 0, 0, 0, 0};
    if (active) {
        double q[6];
        #pragma unroll
        for (int i = 0; i < 6; ++i) q[i] = joints[6 * e + i];
        #pragma unroll
        for (int i = 0; i < 6; ++i)
            if (i == col) q[i] = q[i] + eps;
        const int s = sys_idx ? clamp_sys(sys_idx[e], kc.c.n_systems) : 0;
        fk_dispatch_d<MODE>(kc, s_sys[s], q, r, st);
    }
    #pragma unroll
    for (int k = 0; k < 3; ++k) s_tip[k][threadIdx.x] = r[k];
    __syncthreads();
    if (!active) return;
    const int base = slot * 7 + 6;
    if (col < 6) {
        #pragma unroll
        for (int k = 0; k < 3; ++k) jac[18 * e + 6 * k + col] = (r[k] - s_tip[k][base]) / eps;
    } else if (tip) {
        #pragma unroll
        for (int k = 0; k < 3; ++k) tip[3 * e + k] = r[k];
    }
    if (status) atomicOr(&status[e], st.status);
}

__global__ __launch_bounds__(BLOCK) void k_set_action(KCfg kc, float *__restrict__ joints,
                                                         const int32_t *__restrict__ sys_idx,
                                                         const float *__restrict__ actions, int64_t n)
{
    __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
    stage_systems(kc, s_sys);
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= n) return;
    float q[6], a[6];
    #pragma unroll
    for (int i = 0; i < 6; ++i) { q[i] = joints[6 * e + i]; a[i] = actions[6 * e + i]; }
    const int s = sys_idx ? clamp_sys(sys_idx[e], kc.c.n_systems) : 0;
    set_action_substeps(s_sys[s], kc.c.constrain_alpha != 0, kc.c.n_substeps, q, a);
    #pragma unroll
    for (int i = 0; i < 6; ++i) joints[6 * e + i] = q[i];
}

// ------------------------------------------------------------------------------------------
#include "ctr_her_device.inc"

// The per-env tail of CtrReachEnv.step after the FK (ctr_reach_env.py:136-158): reward, done,
// success, error, observation, and the auto-reset from the pool (or the miss flag).
// The pooled reset of an env whose episode hits the time limit this step (t + 1 >= max_steps:
// done whatever the FK gives, ~86 % of the resets at steady state), loaded when the step starts.
// The reset path at the end of the step then needs no dependent HBM round trips (pool_r, then
// the row) on the slowest wave's critical path; the other resets still load theirs at the end.
struct PoolPre {
    bool loaded = false;
    uint32_t pr;            // pool_r of the slot (the reset number it holds)
    int32_t sys;
    uint32_t stat;
    float q0[6], qd[6];
    double dg[3], ag[3];
};

// The slot's first 112 B (every field) as 7 dwordx4 loads of its one 128-B line.  The fields are
// rebuilt from the dwords by constant index (no aggregate copy: that went through scratch).
__device__ __forceinline__ void pool_load(const ctr_pool_slot_t *sl, PoolPre &pp)
{
    static_assert(sizeof(ctr_pool_slot_t) == 128 && offsetof(ctr_pool_slot_t, ag) == 24 &&
                  offsetof(ctr_pool_slot_t, qd) == 48 && offsetof(ctr_pool_slot_t, q0) == 72 &&
                  offsetof(ctr_pool_slot_t, sys) == 96 && offsetof(ctr_pool_slot_t, r) == 104, "ctr_pool_slot_t layout");
    const uint4 *v = reinterpret_cast<const uint4 *>(sl);
    uint32_t d[28];
    #pragma unroll
    for (int k = 0; k < 7; ++k) {
        const uint4 w = v[k];
        d[4 * k] = w.x; d[4 * k + 1] = w.y; d[4 * k + 2] = w.z; d[4 * k + 3] = w.w;
    }
    pp.loaded = true;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        pp.dg[i] = __hiloint2double((int)d[2 * i + 1], (int)d[2 * i]);
        pp.ag[i] = __hiloint2double((int)d[6 + 2 * i + 1], (int)d[6 + 2 * i]);
    }
    #pragma unroll
    for (int i = 0; i < 6; ++i) { pp.qd[i] = __uint_as_float(d[12 + i]); pp.q0[i] = __uint_as_float(d[18 + i]); }
    pp.sys = (int32_t)d[24];
    pp.stat = d[25];
    pp.pr = d[26];
}

// The slot as 8 dwordx4 stores (the whole line, pad zeroed): the refill's writes.
__device__ __forceinline__ void pool_store(ctr_pool_slot_t *sl, const float qd[6], const float q0[6], const double dg[3],
                                           const double ag[3], int32_t sys, uint32_t stat, uint32_t r)
{
    uint32_t d[32];
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        d[2 * i] = (uint32_t)__double2loint(dg[i]);
        d[2 * i + 1] = (uint32_t)__double2hiint(dg[i]);
        d[6 + 2 * i] = (uint32_t)__double2loint(ag[i]);
        d[6 + 2 * i + 1] = (uint32_t)__double2hiint(ag[i]);
    }
    #pragma unroll
    for (int i = 0; i < 6; ++i) { d[12 + i] = __float_as_uint(qd[i]); d[18 + i] = __float_as_uint(q0[i]); }
    d[24] = (uint32_t)sys;
    d[25] = stat;
    d[26] = r;
    #pragma unroll
    for (int i = 27; i < 32; ++i) d[i] = 0u;
    uint4 *v = reinterpret_cast<uint4 *>(sl);
    #pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = make_uint4(d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]);
}

// ALL: load every env's next reset, not only the time-limit ones (the rigid 8-lane group path:
// latency-bound, with registers to spare, and its successes are as likely to sit on the slowest
// wave's tail).
// t, epoch: the env's episode clock and reset count (already loaded by the caller).
template <bool ALL = false>
__device__ __forceinline__ void pool_prefetch(const KCfg &kc, const ctr_batch_t &b, int64_t e, int32_t autoreset,
                                              PoolPre &pp, int32_t t, uint32_t epoch)
{
    const int P = b.pool_depth;
    if (!autoreset || P <= 0 || (!ALL && t + 1 < kc.c.max_steps)) return;
    const uint32_t r = epoch + 1;
    pool_load(b.pool + ((int64_t)(r % (uint32_t)P) * b.n + e), pp);
}

struct StepFlags {
    bool miss = false;       // done, but no pooled reset available -> k_reset
    bool pooled = false;     // done and reset from the pool -> queue the refill
    uint32_t pooled_r = 0;
};

// t_prev, epoch, dg_prev: the env's clock, reset count and desired goal before the step (loaded
// at the start of the step).
__device__ __forceinline__ void step_finish(const KCfg &kc, const ctr_batch_t &b, const ctr_step_out_t &o, int64_t e,
                                            int s, float q[6], double ag[3], const FkStats &st, int32_t autoreset,
                                            StepFlags &fl, const ctr_her_t *her, const float *action,
                                            PoolPre &lp, int32_t t_prev, uint32_t epoch, const double dg_prev[3],
                                            float4 &grow)
{
    const int32_t t = t_prev + 1;
    double dg[3];
    #pragma unroll
    for (int i = 0; i < 3; ++i) dg[i] = dg_prev[i];
    const double dx = ag[0] - dg[0], dy = ag[1] - dg[1], dz = ag[2] - dg[2];
    const double d = sqrt(dx * dx + dy * dy + dz * dz);
    const double tol = kc.c.tol;
    const float reward = (d > tol) ? -1.0f : 0.0f;              // ctr_reach_env.py:170
    const bool done = (reward == 0.0f) || (t >= kc.c.max_steps); // :140
    const bool multi = kc.c.n_systems > 1;
    const bool f64 = kc.c.obs_f64 != 0;
    double obs[14];
    obs_lane(q, dg, ag, tol, s, multi, kc.c.egocentric != 0, obs);
    o.reward[e] = reward;
    o.done[e] = done ? 1 : 0;
    o.success[e] = (d < tol) ? 1 : 0;                           // :155
    o.error[e] = (float)d;
    uint32_t stat = st.status;
    if (o.nfev) o.nfev[e] = st.nfev;
    if (o.packed || o.gather) {
        // the gather row of this step (distributed.PACK_WIDTH, one 16-B store): the pre-reset tip,
        // so a done env reports where its episode ended, and done | success << 1 | (reward = -1)
        // << 2 (the sparse reward is -1 or 0, ctr_reach_env.py:169)
        const float fl = (float)((done ? 1 : 0) | ((d < tol) ? 2 : 0) | ((reward < 0.0f) ? 4 : 0));
        const float4 row = make_float4((float)ag[0], (float)ag[1], (float)ag[2], fl);
        if (o.packed) *reinterpret_cast<float4 *>(o.packed + 4 * e) = row;
        grow = row;                                             // the fused push (step_body)
    }
    // ctr_step_her: the transition goes into the env's HER episode before any auto-reset
    if (her) {
        float obf[14];
        obs_to_f32(obs, obf);
        her_record_lane(*her, e, action, reward, done, obf, ag, tol);
    }
    int32_t t_out = t;
    if (autoreset && done) {
        if (o.terminal_obs) write_obs(o.terminal_obs, e, obs, multi, f64);
        if (o.terminal_achieved)
            #pragma unroll
            for (int i = 0; i < 3; ++i) o.terminal_achieved[3 * e + i] = ag[i];
        const uint32_t r = epoch + 1;                           // reset number to take
        const int P = b.pool_depth;
        // the slot of reset r (one line), unless the step's start prefetched it
        if (P > 0 && !lp.loaded) pool_load(b.pool + ((int64_t)(r % (uint32_t)P) * b.n + e), lp);
        if (P > 0 && lp.pr == r) {
            // pooled reset: the precomputed draws + FKs of reset r (ctr_reach_env.py:70-114)
            const int s2 = clamp_sys(lp.sys, kc.c.n_systems);
            #pragma unroll
            for (int i = 0; i < 6; ++i) q[i] = lp.q0[i];
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                dg[i] = lp.dg[i];
                ag[i] = lp.ag[i];
            }
            if (b.desired_joints)
                #pragma unroll
                for (int i = 0; i < 6; ++i) b.desired_joints[6 * e + i] = lp.qd[i];
            if (b.starting_joints)
                #pragma unroll
                for (int i = 0; i < 6; ++i) b.starting_joints[6 * e + i] = q[i];
            if (b.starting_position)
                #pragma unroll
                for (int i = 0; i < 3; ++i) b.starting_position[3 * e + i] = ag[i];
            #pragma unroll
            for (int i = 0; i < 3; ++i) b.desired_goal[3 * e + i] = dg[i];
            b.system[e] = s2;
            b.epoch[e] = r;
            stat |= lp.stat;
            obs_lane(q, dg, ag, kc.c.tol, s2, multi, kc.c.egocentric != 0, obs);
            if (her) {                                              // the next episode starts now
                float obf[14];
                obs_to_f32(obs, obf);
                her_reopen(*her, e, r, obf, ag, dg);
            }
            fl.pooled = true;
            fl.pooled_r = r;
            t_out = 0;
        } else if (autoreset == CTR_AUTORESET_POOLED) {
            // the caller promised a full pool and launches no sweep: report, keep the env done
            // (it takes its reset on a later step, once a refill has precomputed it)
            stat |= CTR_STATUS_POOL_MISS;
        } else {
            fl.miss = true;
        }
    }
    b.t[e] = t_out;
    #pragma unroll
    for (int i = 0; i < 6; ++i) b.joints[6 * e + i] = q[i];
    #pragma unroll
    for (int i = 0; i < 3; ++i) b.achieved_goal[3 * e + i] = ag[i];
    write_obs(o.obs, e, obs, multi, f64);
    if (o.status) o.status[e] = stat;
}

// step_finish for the rigid 8-lane group path (no HER): the env's two observations -- of the
// post-step state (lane 0: the terminal one of a done env) and of the pooled reset's state (lane
// 1) -- come from ONE obs_lane call with per-lane operands instead of two calls in sequence on the
// lead lane; lane 1 also holds the env's prefetched pool row (pool_prefetch<true>) and writes the
// reset, lane 0 everything else.  Same values and the same flags as step_finish.  Every lane of
// the wave calls it (group shuffles); ag is valid on lane 0 of the group (fk_group_rigid4).
// pp: lane 1's pool_prefetch of the env's next reset; a done env whose row was not prefetched
// (pool_prefetch without ALL: only the time-limit ones) loads it here.
template <int G = SEG_GROUP>
__device__ __forceinline__ void step_finish_group(const KCfg &kc, const ctr_batch_t &b, const ctr_step_out_t &o,
                                                  int64_t e, int j, bool in, int s, const float q[6], double ag[3],
                                                  const FkStats &st, int32_t autoreset, StepFlags &fl,
                                                  PoolPre &pp, float4 &grow)
{
    const int lead = (int)(threadIdx.x & 63) & ~(G - 1);
    #pragma unroll
    for (int i = 0; i < 3; ++i) ag[i] = __shfl(ag[i], lead);
    if (!in || j > 1) return;
    const int32_t t = b.t[e] + 1;
    double dg[3];
    #pragma unroll
    for (int i = 0; i < 3; ++i) dg[i] = b.desired_goal[3 * e + i];
    const double dx = ag[0] - dg[0], dy = ag[1] - dg[1], dz = ag[2] - dg[2];
    const double d = sqrt(dx * dx + dy * dy + dz * dz);
    const double tol = kc.c.tol;
    const float reward = (d > tol) ? -1.0f : 0.0f;              // ctr_reach_env.py:170
    const bool done = (reward == 0.0f) || (t >= kc.c.max_steps); // :140
    const bool multi = kc.c.n_systems > 1;
    const bool f64 = kc.c.obs_f64 != 0;
    const uint32_t r = b.epoch[e] + 1;                          // reset number to take
    if (autoreset && done && b.pool_depth > 0 && j == 1 && !pp.loaded)
        pool_load(b.pool + ((int64_t)(r % (uint32_t)b.pool_depth) * b.n + e), pp);
    // lane 1 holds the row of reset r: a pooled reset if the env is done and it is there
    const bool reset = autoreset && done && b.pool_depth > 0 && j == 1 && pp.loaded && pp.pr == r;
    // lanes 0 and 1 of the group agree on the reset (shuffled while both are active)
    const bool reset_env = __shfl(reset ? 1 : 0, lead + 1) != 0;
    const uint32_t reset_stat = (uint32_t)__shfl(reset ? (int)pp.stat : 0, lead + 1);
    float qo[6];
    double dgo[3], ago[3];
    #pragma unroll
    for (int i = 0; i < 6; ++i) qo[i] = reset ? pp.q0[i] : q[i];
    #pragma unroll
    for (int i = 0; i < 3; ++i) { dgo[i] = reset ? pp.dg[i] : dg[i]; ago[i] = reset ? pp.ag[i] : ag[i]; }
    const int so = reset ? clamp_sys(pp.sys, kc.c.n_systems) : s;
    double obs[14];
    obs_lane(qo, dgo, ago, tol, so, multi, kc.c.egocentric != 0, obs);
    if (j == 0) {
        o.reward[e] = reward;
        o.done[e] = done ? 1 : 0;
        o.success[e] = (d < tol) ? 1 : 0;                       // :155
        o.error[e] = (float)d;
        if (o.nfev) o.nfev[e] = st.nfev;
        if (o.packed || o.gather) {
            const float fl4 = (float)((done ? 1 : 0) | ((d < tol) ? 2 : 0) | ((reward < 0.0f) ? 4 : 0));
            const float4 row = make_float4((float)ag[0], (float)ag[1], (float)ag[2], fl4);
            if (o.packed) *reinterpret_cast<float4 *>(o.packed + 4 * e) = row;
            grow = row;
        }
        uint32_t stat = st.status;
        if (autoreset && done) {
            if (o.terminal_obs) write_obs(o.terminal_obs, e, obs, multi, f64);
            if (o.terminal_achieved)
                #pragma unroll
                for (int i = 0; i < 3; ++i) o.terminal_achieved[3 * e + i] = ag[i];
            if (!reset_env) {
                if (autoreset == CTR_AUTORESET_POOLED) stat |= CTR_STATUS_POOL_MISS;   // see step_finish
                else fl.miss = true;
            }
        }
        if (reset_env) stat |= reset_stat;
        else {
            b.t[e] = t;
            #pragma unroll
            for (int i = 0; i < 6; ++i) b.joints[6 * e + i] = q[i];
            #pragma unroll
            for (int i = 0; i < 3; ++i) b.achieved_goal[3 * e + i] = ag[i];
            write_obs(o.obs, e, obs, multi, f64);
        }
        if (o.status) o.status[e] = stat;
    } else if (reset) {
        // pooled reset: the precomputed draws + FKs of reset r (ctr_reach_env.py:70-114)
        if (b.desired_joints)
            #pragma unroll
            for (int i = 0; i < 6; ++i) b.desired_joints[6 * e + i] = pp.qd[i];
        if (b.starting_joints)
            #pragma unroll
            for (int i = 0; i < 6; ++i) b.starting_joints[6 * e + i] = pp.q0[i];
        if (b.starting_position)
            #pragma unroll
            for (int i = 0; i < 3; ++i) b.starting_position[3 * e + i] = pp.ag[i];
        #pragma unroll
        for (int i = 0; i < 3; ++i) { b.desired_goal[3 * e + i] = pp.dg[i]; b.achieved_goal[3 * e + i] = pp.ag[i]; }
        #pragma unroll
        for (int i = 0; i < 6; ++i) b.joints[6 * e + i] = pp.q0[i];
        b.system[e] = so;
        b.epoch[e] = r;
        b.t[e] = 0;
        write_obs(o.obs, e, obs, multi, f64);
        fl.pooled = true;
        fl.pooled_r = r;
    }
}

// The end of every step (all lanes of the wave): the auto-reset lists (miss sweep, pool refill
// queue) and the fused push of the step's rows.
__device__ __forceinline__ void step_epilogue(const ctr_batch_t &b, const ctr_step_out_t &o, int32_t autoreset,
                                              const StepFlags &fl, int64_t e, bool live, const ctr_gather_push_t *gp,
                                              bool slot_free0, float4 grow)
{
    if (autoreset) {
        if (autoreset == CTR_AUTORESET_POOLED) {
            // no miss sweep follows: zero the next step's miss counter here (this step neither
            // reads nor appends to either counter)
            if (blockIdx.x == 0 && threadIdx.x == 0) b.work[(b.work_parity & 1) ^ 1] = 0;
        } else {
            const int32_t one[1] = {(int32_t)e};
            wave_append(miss_counter(b), miss_items(b), b.n, fl.miss, one, 1);
        }
        if (b.pool_depth > 0) {
            const int32_t two[2] = {(int32_t)e, (int32_t)(fl.pooled_r + (uint32_t)b.pool_depth)};
            wave_append(b.refill, b.refill + 1, b.refill_cap, fl.pooled, two, 2);
        }
    }
    if (gp) {
        // the fused push (every lane of the wave here): once every consumer has released the
        // slot (normally known since the staging), each env's row into every rank's ring with
        // system-scope stores, waited on, so the rows are performed at system scope before the
        // wave ends and the next launch publishes the sequence words (include/ctr_reach_amd.h)
        if (!slot_free0 && !gather_wait_slot(gp, o.gather_seq)) {
            if ((threadIdx.x & 63) == 0) atomicOr(gp->err, CTR_GATHER_E_RELEASE_TIMEOUT);
            gather_poison_lanes(gp, o.gather_seq);       // the overrun consumers learn it too
        }
        if (live) gather_store_row(gp, e, grow);
        gather_rows_performed();
        if (o.gather_wait_prev && blockIdx.x == 0 && threadIdx.x < 64)
            gather_wait_prev_lane(gp, o.gather_seq - 1u);
    }
}

// Torsionally rigid model with fixed-step RK4 (MODE bits 2 and 4): one env on a group of
// SEG_GROUP lanes, whose segments run in parallel (fk_group_rigid4); other modes: one env per lane.
// HER: record the step into the HER store (ctr_step_her); a compile-time switch, so the plain
// step carries no trace of it (a runtime flag measured +2.3 us on k_step).
template <int MODE, bool HER>
__device__ __forceinline__ void step_body(const KCfg &kc, const ctr_batch_t &b, const float *__restrict__ actions,
                                          const ctr_step_out_t &o, int32_t autoreset, const HerK &hk)
{
    const ctr_her_t *her = HER ? &hk.h : nullptr;
    constexpr bool GROUP = (MODE & 6) == 6;
    constexpr int G = GROUP ? SEG_GROUP : 1;
    __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
    __shared__ ctr_tube_raw_t s_raw[CTR_MAX_SYSTEMS];
    const int64_t gl = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    const int64_t e = gl / G;
    const int j = (int)(gl % G);
    const bool in = e < b.n;                 // the lane works on a live env
    const bool live = in && j == 0;          // ... and is its lead lane (every per-env write)
    // the table inputs' loads first, then the env's rows (system, joints, action; unconditional,
    // from a clamped row, so nothing waits for them before the staging): the rows' latency then
    // hides behind the tables', which the staging waits for anyway
    StageRegs stg;
    stage_load(kc, stg);
    __builtin_amdgcn_sched_barrier(0);       // keep the table loads ahead of the row loads
    const int64_t ec = in ? e : b.n - 1;
    const int s_in = b.system[ec];
    float q_in[6], a_in[6];
    #pragma unroll
    for (int i = 0; i < 6; ++i) { q_in[i] = b.joints[6 * ec + i]; a_in[i] = actions[6 * ec + i]; }
    const int32_t t_in = b.t[ec];
    const uint32_t ep_in = b.epoch[ec];
    double dg_in[3];
    #pragma unroll
    for (int i = 0; i < 3; ++i) dg_in[i] = b.desired_goal[3 * ec + i];
    // fused push: the consumers' release words, read behind the staging (checked after it)
    const ctr_gather_push_t *gp = o.gather;
    const uint32_t rel0 = gp ? gather_release_load(gp, o.gather_seq) : 0u;
    stage_systems<!GROUP>(kc, s_sys, s_raw, &stg);
    const bool slot_free0 = gp ? gather_slot_free(gp, o.gather_seq, rel0) : true;
    // one env per lane: the finish's inputs wait out the FK in LDS (they have landed during the
    // staging), not in registers the FK loop would have to keep
    __shared__ double s_fin_dg[3][BLOCK];
    __shared__ int32_t s_fin_t[BLOCK];
    __shared__ uint32_t s_fin_ep[BLOCK];
    if constexpr (!GROUP) {
        #pragma unroll
        for (int i = 0; i < 3; ++i) s_fin_dg[i][threadIdx.x] = dg_in[i];
        s_fin_t[threadIdx.x] = t_in;
        s_fin_ep[threadIdx.x] = ep_in;
    }
    // the step's sequence word after the packed rows (the copy-engine gather pushes it after them)
    if (o.packed && o.packed_seq && blockIdx.x == 0 && threadIdx.x == 0)
        *reinterpret_cast<uint4 *>(o.packed + 4 * b.n) = make_uint4(o.packed_seq, 0u, 0u, 0u);
    // fused push gather: the previous gathered step's launch has completed, so its rows are in
    // every rank's ring (performed at system scope); publish its sequence word there, and release
    // this rank's slot of step gather_seq + 1 - depth (its readers ran before this launch)
    if (blockIdx.x == 0) {
        if (o.gather_prev) gather_publish_lane(o.gather_prev, o.gather_prev_seq);
        if (gp) gather_release_lane(gp, o.gather_seq + 1u - (uint32_t)gp->depth);
    }
    StepFlags fl;
    float4 grow = make_float4(0.f, 0.f, 0.f, 0.f);   // this lane's gather row (fused push)
    if constexpr (GROUP) {
        // every lane of the wave takes part in the group's shuffles
        int s = 0;
        float q[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        PoolPre pp;
        // the env's next reset, in flight during set_action (lane 1 writes pooled resets without
        // HER; the lead lane with it)
        if (in && j == (HER ? 0 : 1)) pool_prefetch<true>(kc, b, e, autoreset, pp, t_in, ep_in);
        if (in) {
            s = clamp_sys(s_in, kc.c.n_systems);
            #pragma unroll
            for (int i = 0; i < 6; ++i) q[i] = q_in[i];
            set_action_substeps(s_sys[s], kc.c.constrain_alpha != 0, kc.c.n_substeps, q, a_in);
        }
        const SysK &sy = in ? episode_sys(kc, s_sys, s_raw, s, b.epoch[e], (uint64_t)(b.env_base + e)) : s_sys[0];
        const double qd[6] = {(double)q[0], (double)q[1], (double)q[2], (double)q[3], (double)q[4], (double)q[5]};
        FkStats st = {0, 0, 0, 0, 0};
        double ag[3];
        if (fk_needs_careful_trig(qd))
            fk_group_rigid4<(MODE & 1) != 0, true>(sy, qd, j, ag, st, (double)kc.c.rk4_steps_per_m);
        else
            fk_group_rigid4<(MODE & 1) != 0, false>(sy, qd, j, ag, st, (double)kc.c.rk4_steps_per_m);
        if constexpr (HER) {
            if (live)
                step_finish(kc, b, o, e, s, q, ag, st, autoreset, fl, her, actions + 6 * e, pp, t_in, ep_in, dg_in, grow);
        } else {
            step_finish_group(kc, b, o, e, j, in, s, q, ag, st, autoreset, fl, pp, grow);
        }
    } else if (live) {
        const int s = clamp_sys(s_in, kc.c.n_systems);
        const SysK &sy = s_sys[s];
        float q[6];
        #pragma unroll
        for (int i = 0; i < 6; ++i) q[i] = q_in[i];
        PoolPre pp;
        pool_prefetch(kc, b, e, autoreset, pp, t_in, ep_in);
        set_action_substeps(sy, kc.c.constrain_alpha != 0, kc.c.n_substeps, q, a_in);
        FkStats st = {0, 0, 0, 0, 0};
        double ag[3];
        fk_dispatch<MODE>(kc, episode_sys(kc, s_sys, s_raw, s, ep_in, (uint64_t)(b.env_base + e)), q, ag, st);
        double dg_f[3];
        #pragma unroll
        for (int i = 0; i < 3; ++i) dg_f[i] = s_fin_dg[i][threadIdx.x];
        step_finish(kc, b, o, e, s, q, ag, st, autoreset, fl, her, actions + 6 * e, pp, s_fin_t[threadIdx.x],
                    s_fin_ep[threadIdx.x], dg_f, grow);
    }
    step_epilogue(b, o, autoreset, fl, e, live, gp, slot_free0, grow);
}

// ------------------------------------------------------------------------------------------
// BASELINE configs[4] (compliant model, fixed-step RK4, no y pre-curvature: MODE 2): one env on a
// lane PAIR (fk_pair_rk4), 512-lane workgroups of 256 envs = 8 waves, two per SIMD (waves w and
// w + 4 of a workgroup share a SIMD: tools/ubench/simd_map.hip).  The launch lasts as long as its
// most loaded SIMD, so the workgroup first ranks its envs by predicted work (the RK4 steps at
// levels 3 and 2, from the post-action extensions) and deals them so that each SIMD gets one
// heavy and one light wave: rank chunk c (32 envs, c = 0 heaviest) goes to wave c < 4 ? c : 11 - c.
// The result of an env does not depend on its lanes (the pair's arithmetic is self-contained).
// ------------------------------------------------------------------------------------------
#ifndef CTR_RK4_PAIR
#define CTR_RK4_PAIR 1
#endif
// The headline (MODE 0, scipy RK45) on lane pairs (fk_pair_rk45): an A/B experiment, off in the
// product build.  Measured 92.5-95.5 us against 72.3 us one env per lane (VERDICT r5 item 4,
// DESIGN.md 3 "RK45 on lane pairs", profiles/r06_rk45pair_ab.txt); built by tools/experiments/ab_rk45pair.sh.
#ifndef CTR_RK45_PAIR
#define CTR_RK45_PAIR 0
#endif
template <int MODE>
constexpr bool pair_mode() { return (CTR_RK4_PAIR && MODE == 2) || (CTR_RK45_PAIR && MODE == 0); }
template <int MODE>
constexpr int step_block() { return pair_mode<MODE>() ? 2 * BLOCK : BLOCK; }
template <int MODE>
constexpr int step_lanes_per_env() { return pair_mode<MODE>() ? 2 : ((MODE & 6) == 6 ? SEG_GROUP : 1); }

// predicted cost of an env's stepped RK4 work, relative to its bound 4 L_1: level-3 steps over
// [0, beta_2 + L_2], level-2 steps over the rest of tube 1 (relative costs 4 : 3, the steps'
// instruction counts), as one of 256 buckets, the heaviest first
__device__ __forceinline__ int pair_work_bucket(const ctr_system_t &sy, const float q[6], double inv_wmax)
{
    const double e2 = fmax(0.0, (double)q[2] + sy.L[2]);
    const double e1 = fmax(e2, (double)q[1] + sy.L[1]);
    const double w = (4.0 * e2 + 3.0 * (e1 - e2)) * inv_wmax;     // in [0, 1] for nested tubes
    return 255 - (int)fmin(fmax(w * 255.0, 0.0), 255.0);
}

// scipy RK45 (the CTR_RK45_PAIR experiment): the attempts follow the segment count (each gap
// restarts the solver), so the key is the number of segment ends beyond s = 0 (the tubes'
// curvature starts and tips: correlation 0.88 with the oracle's RHS count, the extension key
// alone 0.68), the extension key breaking ties
__device__ __forceinline__ int pair_work_bucket_rk45(const ctr_system_t &sy, const float q[6], double inv_wmax)
{
    int nsa = 0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double tipi = (double)q[i] + sy.L[i];
        nsa += (tipi > 0.0) + (tipi - sy.Lc[i] > 0.0);
    }
    const int ext = 255 - pair_work_bucket(sy, q, inv_wmax);                   // 0 .. 255
    const double w = ((double)nsa + 0.9 * (double)ext * (1.0 / 255.0)) * (1.0 / 7.0);
    return 255 - (int)fmin(fmax(w * 255.0, 0.0), 255.0);
}

template <int MODE, bool HER>
__device__ __forceinline__ void step_body_pair(const KCfg &kc, const ctr_batch_t &b, const float *__restrict__ actions,
                                               const ctr_step_out_t &o, int32_t autoreset, const HerK &hk)
{
    const ctr_her_t *her = HER ? &hk.h : nullptr;
    constexpr int NE = BLOCK;                 // envs per 512-lane workgroup
    __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
    __shared__ ctr_tube_raw_t s_raw[CTR_MAX_SYSTEMS];
    __shared__ __attribute__((aligned(16))) int32_t s_hist[256];   // envs per work bucket, then the
                                                                    // buckets' first ranks (read as int4)
    __shared__ uint16_t s_src[NE];
    __shared__ float s_q[6][NE];
    __shared__ int32_t s_s[NE];
    const int pr = (int)(threadIdx.x >> 1);
    const int j = (int)(threadIdx.x & 1);
    const bool odd = j != 0;
    const int64_t base = (int64_t)blockIdx.x * NE;
    // the natural env of this pair: its post-action joints (set_action on both lanes, the same
    // values) and its work key
    const int64_t en = base + pr;
    const bool in_n = en < b.n;
    const int64_t ec = in_n ? en : b.n - 1;
    const int s_in = b.system[ec];
    float q[6], a_in[6];
    #pragma unroll
    for (int i = 0; i < 6; ++i) { q[i] = b.joints[6 * ec + i]; a_in[i] = actions[6 * ec + i]; }
    const ctr_gather_push_t *gp = o.gather;
    const uint32_t rel0 = gp ? gather_release_load(gp, o.gather_seq) : 0u;
    if (threadIdx.x < 256) s_hist[threadIdx.x] = 0;
    stage_systems(kc, s_sys, s_raw);         // (its barrier also orders the histogram's zeroing)
    const bool slot_free0 = gp ? gather_slot_free(gp, o.gather_seq, rel0) : true;
    if (o.packed && o.packed_seq && blockIdx.x == 0 && threadIdx.x == 0)
        *reinterpret_cast<uint4 *>(o.packed + 4 * b.n) = make_uint4(o.packed_seq, 0u, 0u, 0u);
    if (blockIdx.x == 0) {
        if (o.gather_prev) gather_publish_lane(o.gather_prev, o.gather_prev_seq);
        if (gp) gather_release_lane(gp, o.gather_seq + 1u - (uint32_t)gp->depth);
    }
    const int sn = clamp_sys(s_in, kc.c.n_systems);
    set_action_substeps(s_sys[sn], kc.c.constrain_alpha != 0, kc.c.n_substeps, q, a_in);
    // rank by predicted work (a counting sort over 256 buckets, heaviest first, dead envs last):
    // the bucket histogram with one LDS atomic per env -- whose return value is the env's place in
    // its bucket (in atomic order: the deal, not any result, depends on it) -- then its prefix sums
    double lmax = 0.0;
    for (int k = 0; k < kc.c.n_systems; ++k) lmax = fmax(lmax, s_sys[k].L[1]);
#if defined(CTR_RK45_KEY_NSEG)
    const int bkt = !in_n ? 255 : MODE == 0 ? pair_work_bucket_rk45(s_sys[sn], q, 1.0 / (4.0 * lmax))
                                            : pair_work_bucket(s_sys[sn], q, 1.0 / (4.0 * lmax));
#else
    const int bkt = in_n ? pair_work_bucket(s_sys[sn], q, 1.0 / (4.0 * lmax)) : 255;
#endif
    int place = 0;
    if (!odd) {
        place = atomicAdd(&s_hist[bkt], 1);
        #pragma unroll
        for (int i = 0; i < 6; ++i) s_q[i][pr] = q[i];
        s_s[pr] = sn;
    }
    __syncthreads();
    if (threadIdx.x < 64) {                   // wave 0: exclusive prefix sums of the 256 counts
        const int4 c4 = reinterpret_cast<const int4 *>(s_hist)[threadIdx.x];
        const int tot = c4.x + c4.y + c4.z + c4.w;
        int incl = tot;
        #pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_up(incl, off);
            if ((int)threadIdx.x >= off) incl += v;
        }
        const int ex = incl - tot;
        reinterpret_cast<int4 *>(s_hist)[threadIdx.x] = make_int4(ex, ex + c4.x, ex + c4.x + c4.y,
                                                                  ex + c4.x + c4.y + c4.z);
    }
    __syncthreads();
    const int rank = s_hist[bkt] + place;
    const int chunk = rank >> 5;
#if defined(CTR_PAIR_DEAL_ADJ)          // A/B diagnostic: pair chunks onto waves 2k, 2k + 1 instead
    const int slot = (chunk < 4 ? 2 * chunk : 2 * (7 - chunk) + 1) * 32 + (rank & 31);
#elif defined(CTR_PAIR_NOSORT)          // A/B diagnostic: the natural env order
    const int slot = pr;
    (void)chunk;
#else
    const int slot = (chunk < 4 ? chunk : 11 - chunk) * 32 + (rank & 31);
#endif
    if (!odd) s_src[slot] = (uint16_t)pr;
    __syncthreads();
    const int src = s_src[pr];
    const int64_t e = base + src;
    const bool in = e < b.n;
    const bool live = in && !odd;
    #pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = s_q[i][src];
    const int s = s_s[src];
    const int64_t ee = in ? e : b.n - 1;
    const int32_t t_in = b.t[ee];
    const uint32_t ep_in = b.epoch[ee];
    StepFlags fl;
    float4 grow = make_float4(0.f, 0.f, 0.f, 0.f);
    PoolPre pp;
    // the time-limit resets' rows in flight during the FK (the others load theirs when done)
    if (MODE != 0 && in && j == (HER ? 0 : 1)) pool_prefetch(kc, b, e, autoreset, pp, t_in, ep_in);
    const SysK &sy = in ? episode_sys_at(kc, s_sys, s_raw, s, ep_in, (uint64_t)(b.env_base + e), pr) : s_sys[0];
    const double qd[6] = {(double)q[0], (double)q[1], (double)q[2], (double)q[3], (double)q[4], (double)q[5]};
    FkStats st = {0, 0, 0, 0, 0};
    double ag[3];
    if constexpr (MODE == 0) {
        if (fk_needs_careful_trig(qd)) fk_pair_rk45<true>(sy, qd, odd, ag, st);
        else fk_pair_rk45<false>(sy, qd, odd, ag, st);
    } else {
        if (fk_needs_careful_trig(qd)) fk_pair_rk4<true>(sy, qd, odd, ag, st, (double)kc.c.rk4_steps_per_m);
        else fk_pair_rk4<false>(sy, qd, odd, ag, st, (double)kc.c.rk4_steps_per_m);
    }
    if constexpr (HER) {
        if (live) {
            double dg_in[3];
            #pragma unroll
            for (int i = 0; i < 3; ++i) dg_in[i] = b.desired_goal[3 * e + i];
            step_finish(kc, b, o, e, s, q, ag, st, autoreset, fl, her, actions + 6 * e, pp, t_in, ep_in, dg_in, grow);
        }
    } else {
        step_finish_group<2>(kc, b, o, e, j, in, s, q, ag, st, autoreset, fl, pp, grow);
    }
    step_epilogue(b, o, autoreset, fl, e, live, gp, slot_free0, grow);
}

template <int MODE>
__global__ __launch_bounds__(step_block<MODE>()) void k_step(KCfg kc, ctr_batch_t b, const float *__restrict__ actions,
                                                                ctr_step_out_t o, int32_t autoreset)
{
    if constexpr (pair_mode<MODE>()) step_body_pair<MODE, false>(kc, b, actions, o, autoreset, HerK{});
    else step_body<MODE, false>(kc, b, actions, o, autoreset, HerK{});
}

template <int MODE>
__global__ __launch_bounds__(step_block<MODE>()) void k_step_her(KCfg kc, ctr_batch_t b,
                                                                    const float *__restrict__ actions,
                                                                    ctr_step_out_t o, int32_t autoreset, HerK hk)
{
    if constexpr (pair_mode<MODE>()) step_body_pair<MODE, true>(kc, b, actions, o, autoreset, hk);
    else step_body<MODE, true>(kc, b, actions, o, autoreset, hk);
}

// ------------------------------------------------------------------------------------------
// One reset (reset number r of global env genv) computed by a lane PAIR: the even lane draws the
// desired joints and runs the goal FK (ctr_reach_env.py:100-101), the odd lane draws the start
// joints and runs the start FK (:104-112); results are swapped with lane shuffles.  With the rigid
// model and fixed-step RK4 (the 8-lane group FK of k_step, fk_group_rigid4) each FK runs on an
// 8-lane group instead, and a reset takes 16 lanes: lanes 0-7 the goal FK, 8-15 the start FK (the
// groups' lead lanes draw) -- so pooled and swept resets are the same arithmetic as each other.
// Every lane of the wave must call this (inactive lanes with active = false).
struct ResetOut {
    float qd[6], q0[6];
    double dg[3], ag[3];
    int sys;
    uint32_t stat;
};

template <int MODE>
struct ResetLanes {
    static constexpr bool GROUP = (MODE & 6) == 6;
    static constexpr int U = GROUP ? 2 * SEG_GROUP : 2;     // lanes per reset
    static constexpr int PX = GROUP ? SEG_GROUP : 1;        // lane xor: the other FK's lane
    // this lane's FK (0 goal, 1 start), its place in the FK's group, and whether it writes
    __device__ static bool odd() { return ((threadIdx.x & 63) / PX) & 1; }
    __device__ static int j() { return GROUP ? (int)(threadIdx.x & (SEG_GROUP - 1)) : 0; }
    __device__ static bool writer() { return odd() && j() == 0; }
};

template <int MODE>
__device__ __forceinline__ ResetOut reset_pair(const KCfg &kc, const SysK *s_sys, const ctr_tube_raw_t *s_raw,
                                               bool active, bool odd,
                                               uint64_t genv, uint32_t r, const float *q_cur, const double *goal,
                                               int sys_fixed)
{
    using RL = ResetLanes<MODE>;
    constexpr int PX = RL::PX;
    const int j = RL::j();
    const int lead = (int)(threadIdx.x & 63) - j;          // the FK group's lead lane
    const uint64_t seed = kc.c.seed;
    const int ns = kc.c.n_systems;
    const int s = !active ? 0 : (sys_fixed >= 0 ? sys_fixed : sample_system(seed, r, genv, ns));
    const SysK &sy = s_sys[s];
    uint32_t stat = 0;
    float qv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    double tip[3] = {0.0, 0.0, 0.0};
    const bool drew = active && (odd ? (kc.c.resample_joints != 0) : (goal == nullptr));
    // the whole wave samples together (sample_joints_wave): every lane calls it
    if (sample_joints_wave(sy, seed, r, odd ? 1u : 0u, genv, drew && j == 0, qv) > 1000) stat |= CTR_STATUS_SAMPLER_STUCK;
    if constexpr (RL::GROUP) {
        #pragma unroll
        for (int k = 0; k < 6; ++k) qv[k] = __shfl(qv[k], lead);
        stat = (uint32_t)__shfl((int)stat, lead);
    }
    if (active && !drew && odd) {
        #pragma unroll
        for (int k = 0; k < 6; ++k) qv[k] = q_cur[k];
    }
    if constexpr (RL::GROUP) {
        // every lane runs the group FK (DPP joins); the tip is valid on the group's lead lane
        const SysK &esy = active ? episode_sys(kc, s_sys, s_raw, s, r, genv) : s_sys[0];
        const double qd[6] = {(double)qv[0], (double)qv[1], (double)qv[2], (double)qv[3], (double)qv[4], (double)qv[5]};
        FkStats st = {0, 0, 0, 0, 0};
        if (fk_needs_careful_trig(qd))
            fk_group_rigid4<(MODE & 1) != 0, true>(esy, qd, j, tip, st, (double)kc.c.rk4_steps_per_m);
        else
            fk_group_rigid4<(MODE & 1) != 0, false>(esy, qd, j, tip, st, (double)kc.c.rk4_steps_per_m);
        #pragma unroll
        for (int k = 0; k < 3; ++k) tip[k] = __shfl(tip[k], lead);
        const uint32_t fst = (uint32_t)__shfl((int)st.status, lead);
        if (active && !odd && goal) {
            #pragma unroll
            for (int k = 0; k < 3; ++k) tip[k] = goal[k];
        } else if (active) {
            stat |= fst;
        }
    } else if (active) {
        if (!odd && goal) {
            #pragma unroll
            for (int k = 0; k < 3; ++k) tip[k] = goal[k];
        } else {
            FkStats st = {0, 0, 0, 0, 0};
            fk_dispatch<MODE>(kc, episode_sys(kc, s_sys, s_raw, s, r, genv), qv, tip, st);
            stat |= st.status;
        }
    }
    ResetOut ro;
    #pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double other = __shfl_xor(tip[k], PX);
        ro.dg[k] = odd ? other : tip[k];
        ro.ag[k] = odd ? tip[k] : other;
    }
    #pragma unroll
    for (int k = 0; k < 6; ++k) {
        const float other = __shfl_xor(qv[k], PX);
        ro.qd[k] = odd ? other : qv[k];
        ro.q0[k] = odd ? qv[k] : other;
    }
    ro.stat = stat | __shfl_xor(stat, PX);
    ro.sys = s;
    return ro;
}

// Synchronous reset.  mode 0: envs queued in b.work by k_step (pool misses / no pool), swept
// grid-stride by a small grid; it also zeroes the miss counter of the next step.
// mode 1: all envs (or mask).  The pair's odd lane writes the env.
template <int MODE>
__global__ __launch_bounds__(BLOCK) void k_reset(KCfg kc, ctr_batch_t b, int mode, const uint8_t *__restrict__ mask,
                                                    const double *__restrict__ goal,
                                                    const int32_t *__restrict__ sys_in, void *__restrict__ obs,
                                                    uint32_t *__restrict__ status, HerK hk, int32_t her_on)
{
    __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
    __shared__ ctr_tube_raw_t s_raw[CTR_MAX_SYSTEMS];
    __shared__ int s_count;
    if (mode == 0) {
        // launched after every auto-reset step; with the reset pool the miss list is almost always
        // empty, so leave before staging the tables (the launch then costs ~1.5 us, not ~4.7)
        const int32_t c = min(*miss_counter(b), (int32_t)b.n);
        if (threadIdx.x == 0 && blockIdx.x == 0) b.work[(b.work_parity & 1) ^ 1] = 0;   // next step's counter
        if (c == 0) return;                              // block-uniform: no barrier is skipped
        if (threadIdx.x == 0) s_count = c;
    } else if (threadIdx.x == 0) {
        s_count = 0;
    }
    stage_systems(kc, s_sys, s_raw);
    using RL = ResetLanes<MODE>;
    constexpr int PER_WG = BLOCK / RL::U;                 // resets per workgroup and pass
    const int64_t stride = (mode == 0) ? (int64_t)gridDim.x * PER_WG : (int64_t)1 << 62;
    for (int64_t base = (int64_t)blockIdx.x * PER_WG; mode != 0 || base < s_count; base += stride) {
    const int64_t slot = base + threadIdx.x / RL::U;
    const bool odd = RL::odd();
    int64_t e = -1;
    if (mode == 0) {
        if (slot < s_count) e = miss_items(b)[slot];
    } else if (slot < b.n && (!mask || mask[slot])) {
        e = slot;
    }
    const bool active = e >= 0;
    const int64_t ee = active ? e : 0;
    const uint32_t r = active ? b.epoch[ee] + 1 : 0;
    float qc[6];
    #pragma unroll
    for (int k = 0; k < 6; ++k) qc[k] = active ? b.joints[6 * ee + k] : 0.f;
    const int sf = (active && sys_in) ? clamp_sys(sys_in[ee], kc.c.n_systems) : -1;
    const ResetOut ro = reset_pair<MODE>(kc, s_sys, s_raw, active, odd, (uint64_t)(b.env_base + ee), r, qc,
                                           goal ? goal + 3 * ee : nullptr, sf);
    bool queue = false;
    if (active && RL::writer()) {
        #pragma unroll
        for (int k = 0; k < 6; ++k) b.joints[6 * e + k] = ro.q0[k];
        #pragma unroll
        for (int k = 0; k < 3; ++k) { b.desired_goal[3 * e + k] = ro.dg[k]; b.achieved_goal[3 * e + k] = ro.ag[k]; }
        b.t[e] = 0;
        b.system[e] = ro.sys;
        b.epoch[e] = r;
        if (b.desired_joints)
            #pragma unroll
            for (int k = 0; k < 6; ++k) b.desired_joints[6 * e + k] = ro.qd[k];
        if (b.starting_joints)
            #pragma unroll
            for (int k = 0; k < 6; ++k) b.starting_joints[6 * e + k] = ro.q0[k];
        if (b.starting_position)
            #pragma unroll
            for (int k = 0; k < 3; ++k) b.starting_position[3 * e + k] = ro.ag[k];
        const bool multi = kc.c.n_systems > 1;
        double ob[14];
        obs_lane(ro.q0, ro.dg, ro.ag, kc.c.tol, ro.sys, multi, kc.c.egocentric != 0, ob);   // :114
        write_obs(obs, e, ob, multi, kc.c.obs_f64 != 0);
        if (status) status[e] |= ro.stat;
        // ctr_step_her: a swept auto-reset miss opens the env's next HER episode here
        if (her_on && mode == 0) {
            float obf[14];
            obs_to_f32(ob, obf);
            her_reopen(hk.h, e, r, obf, ro.ag, ro.dg);
        }
        queue = b.pool_depth > 0;
    }
    if (b.pool_depth > 0) {
        // keep the pool P resets deep: mode 0 replaces the reset just taken (r + P); mode 1
        // (re)queues r+1 .. r+P, skipping slots already holding the right reset
        if (mode == 0) {
            const int32_t two[2] = {(int32_t)ee, (int32_t)(r + (uint32_t)b.pool_depth)};
            wave_append(b.refill, b.refill + 1, b.refill_cap, queue, two, 2);
        } else {
            for (int j = 1; j <= b.pool_depth; ++j) {
                const uint32_t rr = r + (uint32_t)j;
                const bool need = queue && b.pool[(int64_t)(rr % (uint32_t)b.pool_depth) * b.n + ee].r != rr;
                const int32_t two[2] = {(int32_t)ee, (int32_t)rr};
                wave_append(b.refill, b.refill + 1, b.refill_cap, need, two, 2);
            }
        }
    }
    if (mode != 0) break;
    }
}

// Resumable refill (ctr_batch_t.carry): a header, then two lists of resets whose FKs a refill
// suspended.  Refill k reads list `parity` (resuming every reset on it) and appends to the other;
// its last workgroup empties the list it read and flips `parity`, so HIP-graph replays of the
// refill alternate the lists without host involvement.  Each list is CARRY_SUBS sub-lists with
// their own counters (workgroup b appends to sub-list b mod nsub, nsub = min(CARRY_SUBS, grid)): the waves of a refill
// all suspend at about the same time, and one counter for all 1 024 of them serialised their
// atomics (~7 us of the refill's tail, clock-stamped build); 64 sub-lists put 16 waves on each.
struct CarryRec {
    FkSuspend fk[2];          // the suspended goal FK (even lane) / start FK (odd lane)
    double tip[2][3];         // the tip of an FK that has finished
    float qd[6], q0[6];       // the reset's sampled joints
    int32_t e;
    uint32_t r;
    int32_t sys;
    uint32_t stat;            // the pair's sampling status
    uint32_t fstat[2];        // the status of an FK that has finished
    uint32_t done;            // bit 0: goal FK finished, bit 1: start FK finished
    uint32_t pad;
};
static_assert(sizeof(CarryRec) == 640, "CarryRec layout");

constexpr int CARRY_SUBS = 64;

struct CarryHdr {
    int32_t count[2][CARRY_SUBS];   // resets on each sub-list of each list
    int32_t parity;                 // the list the next refill reads
    int32_t pad[127];
};
static_assert(sizeof(CarryHdr) == 1024, "CarryHdr layout");

// One FK of a refill: the scipy-RK45 FK (either model) runs at most `budget` iterations (the
// compliant RK4 FK at most `budget` RK4 steps) and can start from a suspended state (fk_lane /
// fk_lane_rk4 RESUME); the rigid model's fixed-step RK4 (segment maps on 8-lane groups) always
// runs to the end.
template <int MODE>
constexpr bool refill_resumable() { return (MODE & 6) != 6; }

template <int MODE>
__device__ __forceinline__ bool fk_refill(const KCfg &kc, const SysK &sy, const float q[6], double tip[3], FkStats &st,
                                          const FkSuspend *from, FkSuspend *to, int budget)
{
    if constexpr (!refill_resumable<MODE>()) {
        fk_dispatch<MODE>(kc, sy, q, tip, st);
        return true;
    } else if constexpr ((MODE & 2) != 0) {
        constexpr bool UY = (MODE & 1) != 0;
        const double qd[6] = {(double)q[0], (double)q[1], (double)q[2], (double)q[3], (double)q[4], (double)q[5]};
        const double spm = (double)kc.c.rk4_steps_per_m;
        if (fk_needs_careful_trig(qd)) return fk_lane_rk4<UY, false, true, true>(sy, qd, tip, st, spm, from, to, budget);
        return fk_lane_rk4<UY, false, false, true>(sy, qd, tip, st, spm, from, to, budget);
    } else {
        constexpr bool UY = (MODE & 1) != 0, RG = (MODE & 4) != 0;
        const double qd[6] = {(double)q[0], (double)q[1], (double)q[2], (double)q[3], (double)q[4], (double)q[5]};
        if (fk_needs_careful_trig(qd)) return fk_lane<UY, RG, false, true, true>(sy, qd, tip, st, nullptr, from, to, budget);
        return fk_lane<UY, RG, false, false, true>(sy, qd, tip, st, nullptr, from, to, budget);
    }
}

// Pool refill: the resets suspended by the previous refill (finished here), then the entries
// (env, reset number) queued in b.refill; two lanes per reset, as reset_pair: the even lane draws
// the desired joints and runs the goal FK, the odd lane draws the start joints and runs the start
// FK (ctr_reach_env.py:100-112).
template <int MODE>
__global__ __launch_bounds__(BLOCK) void k_refill(KCfg kc, ctr_batch_t b)
{
    constexpr bool RESUMABLE = refill_resumable<MODE>();  // all but the rigid model's RK4
    __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
    __shared__ ctr_tube_raw_t s_raw[CTR_MAX_SYSTEMS];
    __shared__ int64_t s_count, s_carried;
    __shared__ int s_par, s_budget;
    __shared__ int32_t s_pref[CARRY_SUBS + 1];           // sub-list starts of the list read
    // the table inputs' loads first (stage_load), the queue and list counts behind them: one
    // latency for both before the staging stores them
    StageRegs stg;
    stage_load(kc, stg);
    __builtin_amdgcn_sched_barrier(0);
    CarryHdr *ch = static_cast<CarryHdr *>(b.carry);
    // sub-lists in use: one per dealing workgroup up to CARRY_SUBS (the grid is the same every
    // refill of a batch, so writer and reader agree), each carry_cap / nsub records long
    const int nsub = (int)min((int64_t)CARRY_SUBS, min((int64_t)gridDim.x, (int64_t)256));
    const bool carry_on = RESUMABLE && ch != nullptr && b.carry_cap >= nsub;
    const int64_t sub_cap = b.carry_cap / nsub;
    // the list's parity and sub-list counts: loaded by wave 0 now, used after the staging below
    // (its barriers do not wait for them)
    // (both lists' counts: no load waits for the parity)
    static_assert(CARRY_SUBS == 64, "one count of each list per lane of wave 0");
    int par_l = 0;
    int32_t cnt_a = 0, cnt_b = 0;
    if (threadIdx.x < 64 && carry_on) {
        par_l = ch->parity & 1;
        cnt_a = ch->count[0][threadIdx.x];
        cnt_b = ch->count[1][threadIdx.x];
    }
    if (threadIdx.x == 0) s_count = min((int64_t)b.refill[0], b.refill_cap);
    // (the rigid model's FK never reads the segment LUT: no staging of it)
    stage_systems<(MODE & 4) == 0>(kc, s_sys, s_raw, &stg);
    if (threadIdx.x < 64) {                               // wave 0: prefix sums of the counts read
        int32_t incl = (int32_t)min((int64_t)(par_l ? cnt_b : cnt_a), sub_cap);
        #pragma unroll
        for (int off = 1; off < CARRY_SUBS; off <<= 1) {
            const int32_t v = __shfl_up(incl, off);
            if ((int)threadIdx.x >= off) incl += v;
        }
        if (threadIdx.x < CARRY_SUBS) s_pref[threadIdx.x + 1] = incl;
        if (threadIdx.x == 0) {
            s_pref[0] = 0;
            s_par = par_l;
        }
        if (threadIdx.x == CARRY_SUBS - 1) {
            s_carried = incl;
            // a budget only while every sub-list can take all the pairs its workgroups may suspend
            const int64_t G = min((int64_t)gridDim.x, (int64_t)256);
            const int64_t per_pass = G * (BLOCK / 64) * 32;
            const int64_t passes = (s_count + incl + per_pass - 1) / per_pass;
            const int64_t inflow = (G + nsub - 1) / nsub * (BLOCK / 64) * 32 * passes;
            s_budget = (carry_on && b.refill_budget > 0 && inflow <= sub_cap) ? b.refill_budget : 0;
        }
    }
    __syncthreads();
    CarryRec *recs = carry_on ? reinterpret_cast<CarryRec *>(reinterpret_cast<char *>(ch) + sizeof(CarryHdr)) : nullptr;
    const int par = s_par;
    const int64_t c = s_carried;
    const CarryRec *in_list = recs ? recs + par * b.carry_cap : nullptr;
    CarryRec *out_list = recs ? recs + (par ^ 1) * b.carry_cap : nullptr;
    // entries are dealt round-robin over the waves of the first (at most) 256 workgroups, one
    // wave per SIMD of the chip: a typical refill (~10 k entries) then puts ~10 resets on every
    // wave instead of 32 on a third of them, and a wave lasts as long as its slowest lane
    using RL = ResetLanes<MODE>;
    const int64_t G = min((int64_t)gridDim.x, (int64_t)256);
    const int64_t waves = G * (BLOCK / 64);
    const int64_t per_pass = waves * (64 / RL::U);        // 32 lane pairs (4 lane groups) per wave
    const int64_t my_wave = (int64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6);
    const int64_t my_pair = (threadIdx.x & 63) / RL::U;
    const int64_t total = s_count + c;
    const int64_t count = blockIdx.x < G ? total : 0;
    const int lane = threadIdx.x & 63;
    const bool odd = RL::odd();
    for (int64_t base = 0; base < count; base += per_pass) {
        const int64_t i = base + my_pair * waves + my_wave;
        if constexpr (!RESUMABLE) {
            // fixed-step RK4: every FK runs to its end (reset_pair; 8-lane group FKs for the rigid model)
            const bool queued = i < total;
            const int64_t e = queued ? b.refill[1 + 2 * i] : 0;
            const uint32_t r = queued ? (uint32_t)b.refill[2 + 2 * i] : 0u;
            const int64_t ps = queued ? (int64_t)(r % (uint32_t)b.pool_depth) * b.n + e : 0;
            // only the resets the env can still take from its ring (see below)
            const bool fresh = queued && b.pool[ps].r != r && r - (uint32_t)b.epoch[e] - 1u < (uint32_t)b.pool_depth;
            // every queued entry draws and integrates (a reset is a pure function of (seed, env,
            // r): an entry that is not fresh computes what it would discard), so the pool_r /
            // epoch loads behind `fresh` overlap the sampling instead of preceding it
            const ResetOut ro = reset_pair<MODE>(kc, s_sys, s_raw, queued, odd, (uint64_t)(b.env_base + e), r, nullptr,
                                                   nullptr, -1);
            if (fresh && RL::writer()) pool_store(b.pool + ps, ro.qd, ro.q0, ro.dg, ro.ag, ro.sys, ro.stat, r);
            continue;
        }
        const bool carried = i < c;                       // pair-uniform, as everything below
        const bool queued = !carried && i < total;
        const CarryRec *rin = nullptr;
        if (carried) {                                    // sub-list k: s_pref[k] <= i < s_pref[k + 1]
            int lo = 0;
            #pragma unroll
            for (int step = CARRY_SUBS / 2; step >= 1; step >>= 1)
                if (s_pref[lo + step] <= (int32_t)i) lo += step;
            rin = in_list + lo * sub_cap + (i - s_pref[lo]);
        }
        int64_t e = 0;
        uint32_t r = 0;
        if (carried) {
            e = rin->e;
            r = rin->r;
        } else if (queued) {
            e = b.refill[1 + 2 * (i - c)];
            r = (uint32_t)b.refill[2 + 2 * (i - c)];
        }
        const int64_t ps = (carried || queued) ? (int64_t)(r % (uint32_t)b.pool_depth) * b.n + e : 0;
        // only the resets the env can still take from its ring, epoch + 1 .. epoch + P.  With a
        // ring shallower than the refill interval one period can queue both r + P (the env took
        // reset r from the ring) and r + 2P (the miss sweep took r + P when the ring ran dry):
        // the two map to one slot, and writing both would race (fields of two resets mixed)
        const uint32_t lead = (queued || carried) ? r - (uint32_t)b.epoch[e] - 1u : 0u;   // resets before r
        // (queued or carried alike: a suspended reset the env has passed meanwhile -- a miss sweep
        // took it -- or whose slot already holds it is dropped, not finished into a stale slot)
        const bool fresh = (queued || carried) && b.pool[ps].r != r && lead < (uint32_t)b.pool_depth;
        const uint64_t genv = (uint64_t)(b.env_base + e);
        // every queued entry draws (draws are a pure function of (seed, env, r); one that is not
        // fresh discards its joints), so the pool_r / epoch loads behind `fresh` overlap the
        // sampling instead of preceding it
        const int s = queued ? sample_system(kc.c.seed, r, genv, kc.c.n_systems) : (carried ? rin->sys : 0);
        float qv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        uint32_t stat = 0;
        // the wave's new resets draw together (sample_joints_wave): every lane calls it
        if (sample_joints_wave(s_sys[s], kc.c.seed, r, odd ? 1u : 0u, genv, queued, qv) > 1000)
            stat |= CTR_STATUS_SAMPLER_STUCK;
        stat |= __shfl_xor(stat, 1);                      // the pair's sampling status
        bool had = false;                                 // this lane's FK finished in an earlier refill
        if (carried) {
            #pragma unroll
            for (int k = 0; k < 6; ++k) qv[k] = odd ? rin->q0[k] : rin->qd[k];
            stat = rin->stat;
            had = ((rin->done >> (odd ? 1 : 0)) & 1u) != 0;
        }
        double tip[3] = {0.0, 0.0, 0.0};
        uint32_t fst = 0;                                 // this lane's FK status
        bool fin = true;
        FkSuspend sv;
        if (had) {
            #pragma unroll
            for (int k = 0; k < 3; ++k) tip[k] = rin->tip[odd][k];
            fst = rin->fstat[odd];
        } else if (fresh) {
            // a reset at least refill_lead resets ahead of its env runs on the budget (again, if it
            // was suspended before); a nearer one finishes here, before the env can need it
            const int budget = (s_budget > 0 && lead >= (uint32_t)b.refill_lead) ? s_budget : 0x7fffffff;
            FkStats st = {0, 0, 0, 0, 0};
            fin = fk_refill<MODE>(kc, episode_sys(kc, s_sys, s_raw, s, r, genv), qv, tip, st,
                                  carried ? &rin->fk[odd] : nullptr, &sv, budget);
            fst = st.status;
        }
        const bool active = fresh;
        const bool ofin = __shfl_xor((int)fin, 1) != 0;
        double otip[3];
        float oq[6];
        #pragma unroll
        for (int k = 0; k < 3; ++k) otip[k] = __shfl_xor(tip[k], 1);
        #pragma unroll
        for (int k = 0; k < 6; ++k) oq[k] = __shfl_xor(qv[k], 1);
        const uint32_t ofst = __shfl_xor(fst, 1);
        if (active && fin && ofin && odd)                 // both FKs done: the pool slot
            pool_store(b.pool + ps, oq, qv, otip, tip, s, stat | fst | ofst, r);
        if constexpr (RESUMABLE) {
            // a pair with a suspended FK goes onto the other list (one atomic per wave)
            const bool keep = active && !(fin && ofin);
            const uint64_t m = __ballot(keep && odd);
            if (m) {
                const int leader = __builtin_ctzll(m);
                int slot = 0;
                const int sub = blockIdx.x % nsub;
                if (lane == leader) slot = atomicAdd(&ch->count[par ^ 1][sub], __popcll(m));
                slot = __shfl(slot, leader) + __popcll(m & ((1ull << (lane | 1)) - 1ull));
                if (keep && slot < sub_cap) {
                    CarryRec *ro = out_list + sub * sub_cap + slot;
                    if (fin) {
                        #pragma unroll
                        for (int k = 0; k < 3; ++k) ro->tip[odd][k] = tip[k];
                        ro->fstat[odd] = fst;
                    } else {
                        ro->fk[odd] = sv;
                    }
                    if (odd) {
                        #pragma unroll
                        for (int k = 0; k < 6; ++k) { ro->qd[k] = oq[k]; ro->q0[k] = qv[k]; }
                        ro->e = (int32_t)e;
                        ro->r = r;
                        ro->sys = s;
                        ro->stat = stat;
                        ro->done = (ofin ? 1u : 0u) | (fin ? 2u : 0u);
                    }
                }
            }
        }
    }
    // the last workgroup to finish clears the queue and the list it read, and flips the lists
    // (every workgroup read the counts at its start): a ticket at refill[1 + 2 cap] instead of a
    // clearing launch
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t *ticket = b.refill + 1 + 2 * b.refill_cap;
        if (atomicAdd(ticket, 1) == (int32_t)gridDim.x - 1) {
            b.refill[0] = 0;
            if (carry_on) {
                for (int k = 0; k < CARRY_SUBS; ++k) ch->count[par][k] = 0;
                ch->parity = par ^ 1;
            }
            *ticket = 0;
        }
    }
}

// Requeue: every env's resets epoch + 1 .. epoch + P that its pool slots do not hold (after a seed
// change or a restore).  One atomic per wave: each lane counts its missing resets (a bit mask over
// j), an exclusive prefix sum over the wave places them.  The refill's suspended resets are among
// them (not in the pool), so both carry lists are emptied (wave 0 of workgroup 0).
__global__ __launch_bounds__(BLOCK) void k_pool_requeue(ctr_batch_t b)
{
    if (blockIdx.x == 0 && threadIdx.x < CARRY_SUBS && b.carry) {
        CarryHdr *ch = static_cast<CarryHdr *>(b.carry);
        ch->count[0][threadIdx.x] = 0;
        ch->count[1][threadIdx.x] = 0;
        if (threadIdx.x == 0) ch->parity = 0;
    }
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    const bool in = e < b.n;
    const uint32_t r = in ? b.epoch[e] : 0u;
    const int P = b.pool_depth;
    // bit j of word w: reset r + 1 + 64 w + j missing (P <= CTR_POOL_MAX = 3 x 64)
    uint64_t miss[CTR_POOL_MAX / 64];
    #pragma unroll
    for (int w = 0; w < CTR_POOL_MAX / 64; ++w) {
        uint64_t m = 0;
        for (int j = 0; j < 64 && 64 * w + j < P && in; ++j) {
            const uint32_t rr = r + 1u + (uint32_t)(64 * w + j);
            if (b.pool[(int64_t)(rr % (uint32_t)P) * b.n + e].r != rr) m |= 1ull << j;
        }
        miss[w] = m;
    }
    int cnt = 0;
    #pragma unroll
    for (int w = 0; w < CTR_POOL_MAX / 64; ++w) cnt += __popcll(miss[w]);
    const int lane = threadIdx.x & 63;
    int incl = cnt;                    // inclusive prefix sum over the wave
    #pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
    }
    const int total = __shfl(incl, 63);
    if (total == 0) return;
    int base = 0;
    if (lane == 0) base = atomicAdd(b.refill, total);
    base = __shfl(base, 0) + (incl - cnt);
    #pragma unroll
    for (int w = 0; w < CTR_POOL_MAX / 64; ++w) {
        for (uint64_t m = miss[w]; m && base < b.refill_cap; m &= m - 1, ++base) {
            b.refill[1 + 2 * base] = (int32_t)e;
            b.refill[2 + 2 * base] = (int32_t)(r + 1u + (uint32_t)(64 * w + __builtin_ctzll(m)));
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_domain_params(KCfg kc, ctr_batch_t b, ctr_system_t *__restrict__ sys_out,
                                                            ctr_tube_raw_t *__restrict__ raw_out)
{
    __shared__ SysK s_sys[CTR_MAX_SYSTEMS];
    __shared__ ctr_tube_raw_t s_raw[CTR_MAX_SYSTEMS];
    stage_systems(kc, s_sys, s_raw);
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= b.n) return;
    const int s = clamp_sys(b.system[e], kc.c.n_systems);
    const uint32_t ep = b.epoch[e];
    ctr_system_t sy;
    ctr_tube_raw_t raw;
    if (kc.c.domain_rand != 0.0 && ep != 0) {
        domain_system(s_sys[s], s_raw[s], kc.c.domain_rand, kc.c.seed, ep, (uint64_t)(b.env_base + e), sy, &raw);
    } else {
        sy = s_sys[s];
        raw = s_raw[s];
    }
    if (sys_out) sys_out[e] = sy;
    if (raw_out) raw_out[e] = raw;
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
    if (cfg->integrator != CTR_INTEGRATOR_RK45_SCIPY && cfg->integrator != CTR_INTEGRATOR_RK4)
        return fail(CTR_EINVAL, "unknown integrator");
    if (cfg->integrator == CTR_INTEGRATOR_RK4 && cfg->rk4_steps_per_m <= 0)
        return fail(CTR_EINVAL, "RK4 needs rk4_steps_per_m > 0");
    if (cfg->model != CTR_MODEL_COMPLIANT && cfg->model != CTR_MODEL_RIGID) return fail(CTR_EINVAL, "unknown model");
    if (!isfinite(cfg->domain_rand)) return fail(CTR_EINVAL, "domain_rand must be finite");
    return 0;
}

int check_batch(const ctr_batch_t &b, const char *who)
{
    if (b.n < 0 || b.n > 0x7fffffff) return fail(CTR_EINVAL, "batch size out of range");
    if (b.n == 0) return 0;
    if (!b.joints || !b.desired_goal || !b.achieved_goal || !b.t || !b.system || !b.epoch)
        return fail(CTR_EINVAL, who);
    if (b.pool_depth < 0 || b.pool_depth > CTR_POOL_MAX)
        return fail(CTR_EINVAL, "pool_depth out of range (0..CTR_POOL_MAX = 192)");
    if (b.pool_depth > 0 && (!b.pool || !b.refill || b.refill_cap <= 0))
        return fail(CTR_EINVAL, "pool_depth > 0 needs the pool and a refill queue");
    if (b.pool_depth > 0 && ((uintptr_t)b.pool & 127u) != 0)
        return fail(CTR_EINVAL, "the reset pool must be 128-B aligned (one cache line per slot)");
    if (b.carry && (b.carry_cap <= 0 || b.carry_cap > 0x3fffffff || b.refill_budget < 0 || b.refill_lead < 0))
        return fail(CTR_EINVAL, "carry needs carry_cap in 1..2^30 and refill_budget, refill_lead >= 0");
    return 0;
}

KCfg make_kcfg(const ctr_env_config_t *cfg)
{
    KCfg kc;
    memcpy(&kc.c, cfg, sizeof *cfg);
    memset(kc.sysk, 0, sizeof kc.sysk);
    for (int s = 0; s < cfg->n_systems && s < CTR_MAX_SYSTEMS; ++s) {
        // sysk_derive's arithmetic (kz_j = EI_j / GJ_j, model.py:97; inv[m] = 1 / sum of the EI
        // present in mask m, model.py:83): one correctly rounded operation at a time
        const ctr_system_t &y = cfg->systems[s];
        for (int j = 0; j < 3; ++j) kc.sysk[s][j] = y.EI[j] / y.GJ[j];
        for (int m = 0; m < 8; ++m) {
            const double e0 = (m & 1) ? y.EI[0] : 0.0, e1 = (m & 2) ? y.EI[1] : 0.0, e2 = (m & 4) ? y.EI[2] : 0.0;
            kc.sysk[s][3 + m] = 1.0 / ((e0 + e1) + e2);
        }
    }
    int has_uy = 0;
    for (int s = 0; s < cfg->n_systems; ++s)
        for (int i = 0; i < 3; ++i)
            if (cfg->systems[s].Uy[i] != 0.0) has_uy = 1;
    kc.mode = has_uy | (cfg->integrator == CTR_INTEGRATOR_RK4 ? 2 : 0) | (cfg->model == CTR_MODEL_RIGID ? 4 : 0);
    return kc;
}

inline unsigned grid_for(int64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }

// lanes k_reset / k_refill spend on one reset (ResetLanes<MODE>::U)
inline int64_t reset_lanes(const KCfg &kc) { return (kc.mode & 6) == 6 ? 2 * SEG_GROUP : 2; }

// Launch kernel template K<MODE> for the runtime mode (8 instantiations).
#define CTR_LAUNCH(K, MODE, GRID, SHM, STREAM, ...)                                                     \
    do {                                                                                           \
        switch (MODE) {                                                                            \
        case 0: hipLaunchKernelGGL(K<0>, GRID, dim3(BLOCK), SHM, STREAM, __VA_ARGS__); break;        \
        case 1: hipLaunchKernelGGL(K<1>, GRID, dim3(BLOCK), SHM, STREAM, __VA_ARGS__); break;        \
        case 2: hipLaunchKernelGGL(K<2>, GRID, dim3(BLOCK), SHM, STREAM, __VA_ARGS__); break;        \
        case 3: hipLaunchKernelGGL(K<3>, GRID, dim3(BLOCK), SHM, STREAM, __VA_ARGS__); break;        \
        case 4: hipLaunchKernelGGL(K<4>, GRID, dim3(BLOCK), SHM, STREAM, __VA_ARGS__); break;        \
        case 5: hipLaunchKernelGGL(K<5>, GRID, dim3(BLOCK), SHM, STREAM, __VA_ARGS__); break;        \
        case 6: hipLaunchKernelGGL(K<6>, GRID, dim3(BLOCK), SHM, STREAM, __VA_ARGS__); break;        \
        default: hipLaunchKernelGGL(K<7>, GRID, dim3(BLOCK), SHM, STREAM, __VA_ARGS__); break;       \
        }                                                                                          \
    } while (0)

}  // namespace

extern "C" {

int ctr_abi_version(void) { return CTR_ABI_VERSION; }

const char *ctr_last_error(void) { return g_err; }

static int fk_impl(const float *joints, const int32_t *sys_idx, const ctr_system_t *tables, int64_t n,
                   const ctr_env_config_t *cfg, double *tip, uint32_t *stats, uint32_t *status, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (n < 0 || (n > 0 && (!joints || !tip))) return fail(CTR_EINVAL, "ctr_fk: bad buffers");
    if (n == 0) return 0;
    KCfg kc = make_kcfg(cfg);
    if (tables) kc.mode |= 1;     // per-row tables may carry y pre-curvature
    CTR_LAUNCH(k_fk, kc.mode, dim3(grid_for(n)), tables ? (size_t)BLOCK * sizeof(SysK) : 0, (hipStream_t)stream, kc,
               joints, sys_idx, tables, n, tip, stats, status);
    return hip_check("ctr_fk launch");
}

int ctr_fk(const float *joints, const int32_t *sys_idx, int64_t n, const ctr_env_config_t *cfg, double *tip,
           uint32_t *stats, uint32_t *status, void *stream)
{
    return fk_impl(joints, sys_idx, nullptr, n, cfg, tip, stats, status, stream);
}

int ctr_fk_tables(const float *joints, const ctr_system_t *tables, int64_t n, const ctr_env_config_t *cfg,
                  double *tip, uint32_t *stats, uint32_t *status, void *stream)
{
    if (n > 0 && !tables) return fail(CTR_EINVAL, "ctr_fk_tables: tables is NULL");
    return fk_impl(joints, nullptr, tables, n, cfg, tip, stats, status, stream);
}

int ctr_fk_shape(const float *joints, const int32_t *sys_idx, const ctr_system_t *tables, int64_t n,
                 const ctr_env_config_t *cfg, int32_t cap, double *tip, double *r, double *s, int32_t *npts,
                 uint32_t *status, void *stream)
{
    if (int rc = check_cfg(cfg)) return rc;
    if (cfg->integrator != CTR_INTEGRATOR_RK45_SCIPY)
        return fail(CTR_EINVAL, "ctr_fk_shape: the backbone dense output needs integrator rk45_scipy");
    if (n < 0 || cap < 0 || (n > 0 && (!joints || !tip || !npts || (cap > 0 && (!r || !s)))))
        return fail(CTR_EINVAL, "ctr_fk_shape: bad buffers");
    if (n == 0) return 0;
    KCfg kc = make_kcfg(cfg);
    if (tables) kc.mode |= 1;
    CTR_LAUNCH(k_fk_shape, kc.mode, dim3(grid_for(n)), tables ? (size_t)BLOCK * sizeof(SysK) : 0, (hipStream_t)stream,
               kc, joints, sys_idx, tables, n, cap, tip, r, s, npts, status);
    return hip_check("ctr_fk_shape launch");
}

int ctr_jacobian(const double *joints, const int32_t *sys_idx, int64_t n, const ctr_env_config_t *cfg, double eps,
                 double *tip, double *jac, uint32_t *status, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (n < 0 || (n > 0 && (!joints || !jac))) return fail(CTR_EINVAL, "ctr_jacobian: bad buffers");
    if (!(eps != 0.0) || !isfinite(eps)) return fail(CTR_EINVAL, "ctr_jacobian: eps must be finite and nonzero");
    if (n == 0) return 0;
    KCfg kc = make_kcfg(cfg);
    const unsigned grid = (unsigned)((n + JAC_ENVS - 1) / JAC_ENVS);
    CTR_LAUNCH(k_jacobian, kc.mode, dim3(grid), 0, (hipStream_t)stream, kc, joints, sys_idx, n, eps, tip, jac, status);
    return hip_check("ctr_jacobian launch");
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

}  // extern "C"

namespace {

// ctr_step / ctr_step_her: her != NULL records the step into the HER store inside k_step (and the
// miss sweep opens the next episodes of the envs it resets).
int step_launch(const ctr_env_config_t *cfg, const ctr_batch_t *batch, const float *actions, const ctr_step_out_t *out,
                int32_t autoreset, const ctr_her_t *her, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (!batch || !out || !actions) return fail(CTR_EINVAL, "ctr_step: NULL argument");
    const ctr_batch_t b = *batch;
    const ctr_step_out_t o = *out;
    if (int r = check_batch(b, "ctr_step: batch buffer missing")) return r;
    if (b.n == 0) return 0;
    if (!o.obs || !o.reward || !o.done || !o.success || !o.error) return fail(CTR_EINVAL, "ctr_step: output missing");
    if (autoreset < CTR_AUTORESET_OFF || autoreset > CTR_AUTORESET_POOLED) return fail(CTR_EINVAL, "ctr_step: bad autoreset");
    if (autoreset && !b.work) return fail(CTR_EINVAL, "ctr_step: autoreset needs batch->work");
    if (autoreset == CTR_AUTORESET_POOLED && b.pool_depth <= 0)
        return fail(CTR_EINVAL, "ctr_step: CTR_AUTORESET_POOLED needs a reset pool");
    if (b.pool_depth > 0 && !cfg->resample_joints) return fail(CTR_EINVAL, "the reset pool needs resample_joints");
    KCfg kc = make_kcfg(cfg);
    hipStream_t s = (hipStream_t)stream;
    HerK hk = {};
    if (her) hk.h = *her;
    const int32_t her_on = her != nullptr;
    if ((kc.mode == 2 && pair_mode<2>()) || (kc.mode == 0 && pair_mode<0>())) {
        // configs[4]: 256 envs per 512-lane workgroup (step_body_pair); dynamic LDS: one domain table per env
        const dim3 g((unsigned)((b.n + BLOCK - 1) / BLOCK)), blk(2 * BLOCK);
        if (kc.mode == 0) {
            if (her) hipLaunchKernelGGL(k_step_her<0>, g, blk, lane_lds_bytes(kc), s, kc, b, actions, o, autoreset, hk);
            else hipLaunchKernelGGL(k_step<0>, g, blk, lane_lds_bytes(kc), s, kc, b, actions, o, autoreset);
        } else {
            if (her) hipLaunchKernelGGL(k_step_her<2>, g, blk, lane_lds_bytes(kc), s, kc, b, actions, o, autoreset, hk);
            else hipLaunchKernelGGL(k_step<2>, g, blk, lane_lds_bytes(kc), s, kc, b, actions, o, autoreset);
        }
    } else {
        const int64_t lanes = (kc.mode & 6) == 6 ? SEG_GROUP * b.n : b.n;      // k_step's lanes per env
        if (her)
            CTR_LAUNCH(k_step_her, kc.mode, dim3(grid_for(lanes)), lane_lds_bytes(kc), s, kc, b, actions, o, autoreset, hk);
        else
            CTR_LAUNCH(k_step, kc.mode, dim3(grid_for(lanes)), lane_lds_bytes(kc), s, kc, b, actions, o, autoreset);
    }
    if (int r = hip_check("ctr_step launch")) return r;
    if (autoreset == CTR_AUTORESET_SWEEP) {
        // misses are rare with a pool: a small grid sweeps the list grid-stride
        const unsigned g = b.pool_depth > 0 ? std::min(grid_for(reset_lanes(kc) * b.n), 64u)
                                            : grid_for(reset_lanes(kc) * b.n);
        CTR_LAUNCH(k_reset, kc.mode, dim3(g), lane_lds_bytes(kc), s, kc, b, 0, (const uint8_t *)nullptr, (const double *)nullptr,
                   (const int32_t *)nullptr, o.obs, o.status, hk, her_on);
        return hip_check("ctr_step reset launch");
    }
    return 0;
}

}  // namespace

extern "C" {

int ctr_step(const ctr_env_config_t *cfg, const ctr_batch_t *batch, const float *actions, const ctr_step_out_t *out,
             int32_t autoreset, void *stream)
{
    return step_launch(cfg, batch, actions, out, autoreset, nullptr, stream);
}

int ctr_reset(const ctr_env_config_t *cfg, const ctr_batch_t *batch, const uint8_t *mask, const double *goal,
              const int32_t *system, void *obs, uint32_t *status, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (!batch || !obs) return fail(CTR_EINVAL, "ctr_reset: NULL argument");
    const ctr_batch_t b = *batch;
    if (int r = check_batch(b, "ctr_reset: batch buffer missing")) return r;
    if (b.n == 0) return 0;
    if (b.pool_depth > 0 && !cfg->resample_joints) return fail(CTR_EINVAL, "the reset pool needs resample_joints");
    KCfg kc = make_kcfg(cfg);
    CTR_LAUNCH(k_reset, kc.mode, dim3(grid_for(reset_lanes(kc) * b.n)), lane_lds_bytes(kc), (hipStream_t)stream, kc, b, 1, mask,
               goal, system, obs,
               status, HerK{}, 0);
    return hip_check("ctr_reset launch");
}

int ctr_pool_refill(const ctr_env_config_t *cfg, const ctr_batch_t *batch, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (!batch) return fail(CTR_EINVAL, "ctr_pool_refill: NULL argument");
    const ctr_batch_t b = *batch;
    if (int r = check_batch(b, "ctr_pool_refill: batch buffer missing")) return r;
    if (b.n == 0 || b.pool_depth == 0) return 0;
    if (!cfg->resample_joints) return fail(CTR_EINVAL, "the reset pool needs resample_joints");
    KCfg kc = make_kcfg(cfg);
    hipStream_t s = (hipStream_t)stream;
    // at most 256 workgroups (one wave per SIMD): the queued entries are dealt over their waves
    CTR_LAUNCH(k_refill, kc.mode, dim3(std::min(grid_for(reset_lanes(kc) * b.n), 256u)), lane_lds_bytes(kc), s, kc, b);
    return hip_check("ctr_pool_refill launch");
}

int64_t ctr_refill_carry_bytes(int64_t carry_cap)
{
    if (carry_cap < 0) return 0;
    return (int64_t)sizeof(CarryHdr) + 2 * carry_cap * (int64_t)sizeof(CarryRec);
}

int ctr_pool_requeue(const ctr_env_config_t *cfg, const ctr_batch_t *batch, void *stream)
{
    if (int r = check_cfg(cfg)) return r;
    if (!batch) return fail(CTR_EINVAL, "ctr_pool_requeue: NULL argument");
    const ctr_batch_t b = *batch;
    if (int r = check_batch(b, "ctr_pool_requeue: batch buffer missing")) return r;
    if (b.n == 0 || b.pool_depth == 0) return 0;
    hipLaunchKernelGGL(k_pool_requeue, dim3(grid_for(b.n)), dim3(BLOCK), 0, (hipStream_t)stream, b);
    return hip_check("ctr_pool_requeue launch");
}

int ctr_domain_params(const ctr_env_config_t *cfg, const ctr_batch_t *batch, ctr_system_t *sys_out,
                      ctr_tube_raw_t *raw_out, void *stream)
{
    if (int rc = check_cfg(cfg)) return rc;
    if (!batch) return fail(CTR_EINVAL, "batch is NULL");
    const ctr_batch_t b = *batch;
    if (b.n < 0 || b.n > 0x7fffffff) return fail(CTR_EINVAL, "batch size out of range");
    if (b.n == 0 || (!sys_out && !raw_out)) return 0;
    if (!b.system || !b.epoch) return fail(CTR_EINVAL, "ctr_domain_params: batch needs system and epoch");
    const KCfg kc = make_kcfg(cfg);
    hipLaunchKernelGGL(k_domain_params, dim3(grid_for(b.n)), dim3(BLOCK), 0, (hipStream_t)stream, kc, b, sys_out,
                       raw_out);
    return hip_check("ctr_domain_params launch");
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

#include "ctr_her.inc"
#include "ctr_gather.inc"
