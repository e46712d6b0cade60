// ctr_device.hpp -- per-lane device math of the batched CTR reach environment (gfx950).
//
// One environment per lane.  Everything here is written for one lane's registers:
// fixed-size arrays are only ever indexed with compile-time constants (fully unrolled)
// so they stay in VGPRs; runtime-indexed lookups go through select chains.
//
// Reference behaviour restated (paths relative to /root/reference/ctr_reach_envs):
//   seg_build          envs/CTR_Python/Segment.py:6-61
//   rhs                envs/model.py:72-117
//   fk_lane            envs/model.py:30-70, 119-164 + scipy solve_ivp(RK45) (rk.py, common.py)
//   set_action_lane    envs/obs.py:166-183
//   obs_lane           envs/obs.py:136-164, envs/obs_utils.py:41-53,69-80
//   sample_joints_wave envs/obs.py:185-207 (Philox4x32-10 stream instead of numpy MT19937)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ctr_reach_amd.h"
#include "ctr_math.hpp"

namespace ctr {

constexpr int NS = 18;  // [u_z(3), alpha(3), r(3), R row-major(9)]   (model.py:136)
constexpr int CTR_BLOCK = 256;   // every kernel runs 256-lane workgroups (per-lane LDS slots below)
constexpr int RK4_MAX_STEPS = 1 << 20;   // fixed-step RK4: more steps in one segment -> CTR_STATUS_TOO_LONG

// ------------------------------------------------------------------------------------------
// Segmentation (Segment.py:6-61).  Ten transition points [0, beta, d_c, d_tip] are sorted,
// the gaps floored to 10 um, and per-gap tube presence / curvature decided.  The result is
// kept "raw" (9 gaps in sorted order, many of which are dropped later) so that every array
// index is static; integration walks the gaps with a cursor.
// ------------------------------------------------------------------------------------------
// The 9 gap end points (cumsum(len[0..k]) + min(beta)) live in LDS, one column per lane
// (s_end[k][lane]: conflict-free, dynamically indexable, off the VGPR budget).
// Tube presence and curvature per gap are 9-bit masks (bit k = gap k): tube i is present on the
// gaps [a_i, c_i) and curved on [b_i, c_i) (Segment.py:29-44), so each mask is one range.
// One column per lane of a 256-lane workgroup, shared by every FK variant a kernel instantiates
// (a function-scope __shared__ array would be allocated once per template instantiation).
__shared__ double s_seg_end[9][CTR_BLOCK];

struct Seg {
    uint32_t kept;     // bit k: gap k has non-zero length and ends after s = 0 (kept in S)
    uint64_t pc;       // bits 9i + k: tube i present on gap k; bits 27 + 9i + k: tube i curved
};

// The 6-bit (present 0-2 | curved 3-5) description of gap k that seg_par takes.
__device__ __forceinline__ uint32_t seg_bits(const Seg &sg, int k)
{
    const uint64_t x = sg.pc >> k;
    uint32_t b = 0;
    #pragma unroll
    for (int j = 0; j < 6; ++j) b |= (uint32_t)((x >> (9 * j)) & 1u) << j;
    return b;
}

__device__ __forceinline__ void cswap(double &a, double &b, int &ia, int &ib)
{
    // Stable compare-exchange: swap only when strictly out of order.
    bool s = b < a;
    double ta = s ? b : a, tb = s ? a : b;
    int ja = s ? ib : ia, jb = s ? ia : ib;
    a = ta; b = tb; ia = ja; ib = jb;
}

// COLSHIFT: the LDS column is threadIdx.x >> COLSHIFT (1: the two lanes of an env pair share one
// column and store the same values into it, fk_pair_rk4).
template <int STRIDE = CTR_BLOCK, int COLSHIFT = 0>   // LDS column stride of end_lds (lanes of the workgroup)
__device__ __forceinline__ Seg seg_build(const ctr_system_t &sy, const double beta[3], double *end_lds)
{
#pragma clang fp contract(off)
    // per-lane LDS column: the sorted position of each point (argsort), so the runtime-indexed
    // lookups below are one LDS read instead of a 10-way select chain; zero-length gaps as a mask
    __shared__ uint8_t s_pos[10][STRIDE];
    const int col = (int)(threadIdx.x >> COLSHIFT) % STRIDE;
    double v[10];
    int id[10];
    v[0] = 0.0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        double dtip = sy.L[i] + beta[i];      // Segment.py:11
        double dc = dtip - sy.Lc[i];          // Segment.py:12
        v[1 + i] = beta[i];
        v[4 + i] = dc;
        v[7 + i] = dtip;
    }
    #pragma unroll
    for (int i = 0; i < 10; ++i) id[i] = i;
    // Odd-even transposition network (10 rounds) -- stable, static indices only.
    #pragma unroll
    for (int r = 0; r < 10; ++r) {
        #pragma unroll
        for (int i = (r & 1); i + 1 < 10; i += 2) cswap(v[i], v[i + 1], id[i], id[i + 1]);
    }
    double len[9];
    uint32_t zero = 0;                    // bit k: gap k floored to zero length
    #pragma unroll
    for (int k = 0; k < 9; ++k) {
        len[k] = 1e-5 * floor(1e5 * (v[k + 1] - v[k]));   // :16
        zero |= (len[k] == 0.0) ? (1u << k) : 0u;
    }
    #pragma unroll
    for (int k = 0; k < 10; ++k) s_pos[id[k]][col] = (uint8_t)k;   // inverse permutation (argsort positions)
    // len_at(x) == 0 (index 9 is never zero-tested by the reference)
    auto zero_at = [&](int x) { return ((zero >> x) & 1u) != 0u; };
    uint64_t pc = 0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        int a = s_pos[i + 1][col], b = s_pos[i + 4][col], c = s_pos[i + 7][col];
        if (zero_at(a)) a += 1;           // :29-36
        if (zero_at(b)) b += 1;
        if (zero_at(a)) a += 1;
        if (c <= 8 && zero_at(c)) c += 1;
        const uint32_t upto_c = (1u << c) - 1u;          // gaps < c (c <= 9)
        const uint32_t pres = upto_c & ~((1u << a) - 1u) & 0x1FFu;
        const uint32_t curv = upto_c & ~((1u << b) - 1u) & 0x1FFu;
        pc |= ((uint64_t)pres << (9 * i)) | ((uint64_t)curv << (27 + 9 * i));
    }
    double bmin = fmin(fmin(beta[0], beta[1]), beta[2]);
    Seg sg;
    sg.kept = 0;
    sg.pc = pc;
    double cum = 0.0;
    #pragma unroll
    for (int k = 0; k < 9; ++k) {         // :46-55 (adding a zero gap is an exact no-op)
        cum += len[k];
        end_lds[k * STRIDE] = cum + bmin;
        sg.kept |= ((len[k] != 0.0) && (cum + bmin > 0.0)) ? (1u << k) : 0u;
    }
    return sg;
}

// A tube system as staged in LDS: the table plus the per-segment divisions precomputed once per
// workgroup (kz_j = EI_j / GJ_j, model.py:97; inv[m] = 1 / sum of the EI present in mask m,
// model.py:83), so segment starts never divide.
struct SysK : ctr_system_t {
    double kz[3];
    double inv[8];
    const double *lut;   // [64][8]: seg_par of every 6-bit gap description (wx, g, inv, present),
                         // staged per workgroup by stage_systems, or nullptr (per-lane tables)
};

__device__ __forceinline__ void sysk_derive(SysK &s, int j)
{
    if (j < 3) s.kz[j] = s.EI[j] / s.GJ[j];
    else if (j < 11) {
        const int m = j - 3;
        const double e0 = (m & 1) ? s.EI[0] : 0.0, e1 = (m & 2) ? s.EI[1] : 0.0, e2 = (m & 4) ? s.EI[2] : 0.0;
        s.inv[m] = 1.0 / ((e0 + e1) + e2);
    }
}

// Per-segment RHS constants.  w* = EI_j * U*_j exactly as the reference's left-to-right
// product ei[j] * ux_0[j] (model.py:85-90); kz = EI/GJ (model.py:97).
struct SegPar {
    double wx[3], wy[3], ux0[3], uy0[3], kz[3], inv;
    double g[3];       // no y pre-curvature: du_z,j/ds = g_j * (sum_k wx_k sin(alpha_k - alpha_j))
    uint32_t present;  // bit j: tube j present (EI_j != 0)
};

// inv: 1 / the EI sum of the present tubes, sy.inv[bits6 & 7] (seg_par) -- passed in by a caller
// whose SysK is a private copy, where that dynamic index would place the copy in scratch memory.
__device__ __forceinline__ SegPar seg_par_inv(const SysK &sy, uint32_t bits6, bool rigid, double inv)
{
    SegPar p;
    #pragma unroll
    for (int j = 0; j < 3; ++j) {
        const bool pres = (bits6 >> j) & 1u;
        const bool curv = (bits6 >> (3 + j)) & 1u;
        const double ei = pres ? sy.EI[j] : 0.0;
        p.ux0[j] = curv ? sy.Ux[j] : 0.0;
        p.uy0[j] = curv ? sy.Uy[j] : 0.0;
        p.wx[j] = ei * p.ux0[j];
        p.wy[j] = ei * p.uy0[j];
        p.kz[j] = (pres && !rigid) ? sy.kz[j] : 0.0;   // torsionally rigid: GJ -> infinity
    }
    p.inv = inv;
    #pragma unroll
    for (int j = 0; j < 3; ++j) p.g[j] = (p.kz[j] * p.ux0[j]) * p.inv;
    p.present = (uint32_t)(bits6 & 7u);
    return p;
}

__device__ __forceinline__ SegPar seg_par(const SysK &sy, uint32_t bits6, bool rigid = false)
{
    return seg_par_inv(sy, bits6, rigid, sy.inv[bits6 & 7u]);
}

// No y pre-curvature: the RHS uses inv only as a factor of every wx product, so fold it in
// (wx <- inv wx, and g = kz ux0 inv becomes kz ux0): two fewer products per RHS.
__device__ __forceinline__ void seg_fold_inv(SegPar &p)
{
    #pragma unroll
    for (int j = 0; j < 3; ++j) {
        p.wx[j] = p.wx[j] * p.inv;
        p.g[j] = p.kz[j] * p.ux0[j];
    }
}

// seg_par from the workgroup's table when the RHS needs only (wx, g, inv, present): no y
// pre-curvature, compliant model, a shared system row (per-lane tables have lut == nullptr).
// Four LDS reads instead of the per-tube selects and products at every segment start.
template <bool HAS_UY, bool RIGID>
__device__ __forceinline__ SegPar seg_par_at(const SysK &sy, uint32_t bits6)
{
    if (!HAS_UY && !RIGID && sy.lut) {
        SegPar p = {};
        const double *e = sy.lut + 8 * bits6;
        #pragma unroll
        for (int j = 0; j < 3; ++j) { p.wx[j] = e[j]; p.g[j] = e[3 + j]; }
        p.inv = e[6];
        p.present = (uint32_t)e[7];
        return p;
    }
    SegPar p = seg_par(sy, bits6, RIGID);
    if (!HAS_UY) seg_fold_inv(p);
    return p;
}

// ------------------------------------------------------------------------------------------
// RHS of the torsionally compliant model (model.py:72-117), split in two parts:
//   trig_of(alpha)          the three relative-angle sin/cos pairs (the transcendental part;
//                           depends on the alpha components only)
//   rhs_core(p, trig, y)    d(u_z)/ds and dR/ds for one segment's constants
// The remaining derivative components are copies and are never materialised:
//   d(alpha_j)/ds = u_z,j if tube j is present else 0          (model.py:98)
//   dr/ds = R e3 = column 3 of R                               (model.py:104-109)
// ------------------------------------------------------------------------------------------
struct Trig {
    double c10, s10, c20, s20, c21, s21;   // cos/sin(alpha_i - alpha_j)
};

// (sin, cos)(k pi/256) table for sincos_tab, one copy per workgroup in LDS; every kernel that
// integrates calls trig_table_fill() before its first barrier.
__shared__ double s_trig_tab[512][2];

__device__ __forceinline__ void trig_table_fill()
{
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) (&s_trig_tab[0][0])[i] = (&ctr_math::TRIG_TAB[0][0])[i];
}

// The same copy in two halves, for a 256-lane workgroup: this lane's four table entries loaded
// into registers (trig_table_load), stored to LDS later (trig_table_store), so that loads the
// kernel issues in between overlap the table's latency instead of queueing behind its stores.
struct TrigRegs {
    double v[4];
};

__device__ __forceinline__ void trig_table_load(TrigRegs &t)
{
    #pragma unroll
    for (int k = 0; k < 4; ++k) t.v[k] = (&ctr_math::TRIG_TAB[0][0])[threadIdx.x + k * CTR_BLOCK];
}

__device__ __forceinline__ void trig_table_store(const TrigRegs &t)
{
    #pragma unroll
    for (int k = 0; k < 4; ++k) (&s_trig_tab[0][0])[threadIdx.x + k * CTR_BLOCK] = t.v[k];
}

// CAREFUL: a wave-uniform ballot sends huge / non-finite angle differences (|d| >= 2^20) to the
// exact out-of-line path.  The branch splits the stage code into basic blocks the scheduler
// cannot interleave (measured +6 % on k_step), so the FK checks its joint angles once
// (fk_needs_careful_trig) and runs the CAREFUL variant only when some lane of the wave needs it.
template <bool CAREFUL = true>
__device__ __forceinline__ Trig trig_of(const double al[3])
{
    Trig t;
    const double d10 = al[1] - al[0], d20 = al[2] - al[0];
    ctr_math::sincos_tab2(d10, d20, s_trig_tab, t.s10, t.c10, t.s20, t.c20);
    if (CAREFUL &&
        __builtin_expect(__ballot(ctr_math::sincos_needs_slow(d10) || ctr_math::sincos_needs_slow(d20)) != 0, 0)) {
        if (ctr_math::sincos_needs_slow(d10)) {
            const ctr_math::SinCos r = ctr_math::sincos_slow(d10);
            t.s10 = r.s;
            t.c10 = r.c;
        }
        if (ctr_math::sincos_needs_slow(d20)) {
            const ctr_math::SinCos r = ctr_math::sincos_slow(d20);
            t.s20 = r.s;
            t.c20 = r.c;
        }
    }
    // alpha_2 - alpha_1 = (alpha_2 - alpha_0) - (alpha_1 - alpha_0): angle-difference identity
    t.c21 = t.c20 * t.c10 + t.s20 * t.s10;
    t.s21 = t.s20 * t.c10 - t.c20 * t.s10;
    return t;
}

// One sincos from the workgroup's LDS table (<= 2 ulp like sincos_cw), the exact path beyond the
// table's |x| < 2^20 range.
__device__ __forceinline__ void sincos_lds(double x, double &s, double &c)
{
    ctr_math::sincos_tab(x, s_trig_tab, s, c);
    if (__builtin_expect(__ballot(ctr_math::sincos_needs_slow(x)) != 0, 0) && ctr_math::sincos_needs_slow(x)) {
        const ctr_math::SinCos r = ctr_math::sincos_slow(x);
        s = r.s;
        c = r.c;
    }
}

// Wave-uniform: does some lane start the FK with an angle of magnitude >= 2^18 (or non-finite)?
// Otherwise every angle difference met during the FK stays below 2^20: the twist integrated over
// a backbone (<= ~0.5 m) moves an angle by orders of magnitude less than 2^18 rad.
__device__ __forceinline__ bool fk_needs_careful_trig(const double q[6])
{
    const double lim = 262144.0;
    const bool ok = fabs(q[3]) < lim && fabs(q[4]) < lim && fabs(q[5]) < lim;
    return __ballot(!ok) != 0;
}

template <bool HAS_UY>
__device__ __forceinline__ void rhs_core(const SegPar &p, const Trig &t, const double uz[3], const double R[9],
                                         double duz[3], double dR[9])
{
    if constexpr (!HAS_UY) {
        // No tube has y pre-curvature (U_y = 0, the registered systems): model.py:86-102 reduce to
        //   uy_i = inv * sum_{k != i} wx_k sin(alpha_k - alpha_i)      (the sign folded per row)
        //   du_z,i/ds = -kz_i ux0_i uy_i = g_i * sum_{k != i} wx_k sin(alpha_i - alpha_k)
        // and only ux_0 of the x curvatures is used (the frame).  Same quantities as the general
        // form below with the known zero / unit terms dropped (a few ulp apart).
        const double sy1 = fma(p.wx[2], t.s20, p.wx[1] * t.s10);         // = -sum_k wx_k s[0][k]
        const double sy2 = fma(p.wx[2], t.s21, -(p.wx[0] * t.s10));       // = -sum_k wx_k s[1][k]
        const double sy3 = fma(p.wx[1], t.s21, p.wx[0] * t.s20);          // = +sum_k wx_k s[2][k]
        duz[0] = -(p.g[0] * sy1);
        duz[1] = -(p.g[1] * sy2);
        duz[2] = p.g[2] * sy3;
        const double a = fma(p.wx[2], t.c20, fma(p.wx[1], t.c10, p.wx[0]));   // ux_0 (wx = inv EI Ux)
        const double b = sy1;                                                 // uy_0
        const double u0 = uz[0];
        #pragma unroll
        for (int r = 0; r < 3; ++r) {                             // dR = R [u]x  (model.py:103-110)
            const double r0 = R[3 * r], r1 = R[3 * r + 1], r2 = R[3 * r + 2];
            dR[3 * r + 0] = r1 * u0 - r2 * b;
            dR[3 * r + 1] = r2 * a - r0 * u0;
            dR[3 * r + 2] = r0 * b - r1 * a;
        }
        return;
    }
    const double c[3][3] = {{1.0, t.c10, t.c20}, {t.c10, 1.0, t.c21}, {t.c20, t.c21, 1.0}};
    const double s[3][3] = {{0.0, -t.s10, -t.s20}, {t.s10, 0.0, -t.s21}, {t.s20, t.s21, 0.0}};
    double ux[3], uy[3];
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        double sx = 0.0, sy = 0.0;
        #pragma unroll
        for (int j = 0; j < 3; ++j) {
            sx += p.wx[j] * c[i][j];
            sy += -p.wx[j] * s[i][j];
            if (HAS_UY) {
                sx += p.wy[j] * s[i][j];
                sy += p.wy[j] * c[i][j];
            }
        }
        ux[i] = p.inv * sx;
        uy[i] = p.inv * sy;
    }
    #pragma unroll
    for (int j = 0; j < 3; ++j) {
        const double tz = HAS_UY ? (ux[j] * p.uy0[j] - uy[j] * p.ux0[j]) : (-uy[j] * p.ux0[j]);
        duz[j] = p.kz[j] * tz;                                   // model.py:97 (0 if absent)
    }
    const double u0 = uz[0], a = ux[0], b = uy[0];
    #pragma unroll
    for (int r = 0; r < 3; ++r) {                                 // dR = R [u]x  (model.py:103-110)
        const double r0 = R[3 * r], r1 = R[3 * r + 1], r2 = R[3 * r + 2];
        dR[3 * r + 0] = r1 * u0 - r2 * b;
        dR[3 * r + 1] = r2 * a - r0 * u0;
        dR[3 * r + 2] = r0 * b - r1 * a;
    }
}

// ------------------------------------------------------------------------------------------
// Tube levels (no y pre-curvature, compliant model).  Tube i is present on [beta_i, beta_i + L_i]
// with beta_i <= 0, so along a backbone the present set only shrinks: level 3 (tube 2 present),
// level 2 (tube 1 present, tube 2 absent), level 1 (tube 0 alone).  An absent tube has wx = g = 0
// and a parked u_z = 0 (fk_lane), so at level 2 every term of rhs_core with alpha_2 is an exact
// zero (only sin/cos(alpha_1 - alpha_0) is needed, u_z,2 and alpha_2 stay constant), and at level 1
// u' = 0 and the frame turns about (wx_0, 0, u_z,0) with no trig at all.  The level-L forms below
// drop those zero terms and give the same values as rhs_core (up to the sign of zero results, which
// no later operation can turn into a non-zero difference); fk_lane runs an attempt at the highest
// level any active lane of the wave needs.
// ------------------------------------------------------------------------------------------
// Trig at level LV < 3: 2 = sin/cos(alpha_1 - alpha_0) only; 1 = none.  Entries a level does not
// compute are 0 (finite: a level-3 RHS of a lower-level lane multiplies them by exact zeros).
template <int LV, bool CAREFUL>
__device__ __forceinline__ Trig trig_lv(const double al[3])
{
    static_assert(LV == 1 || LV == 2, "level 3 is trig_of");
    Trig t;
    t.c20 = t.s20 = t.c21 = t.s21 = 0.0;
    t.c10 = t.s10 = 0.0;
    if constexpr (LV == 2) {
        const double d10 = al[1] - al[0];
        ctr_math::sincos_tab(d10, s_trig_tab, t.s10, t.c10);
        if (CAREFUL && __builtin_expect(__ballot(ctr_math::sincos_needs_slow(d10)) != 0, 0) &&
            ctr_math::sincos_needs_slow(d10)) {
            const ctr_math::SinCos r = ctr_math::sincos_slow(d10);
            t.s10 = r.s;
            t.c10 = r.c;
        }
    }
    return t;
}

// rhs_core<false> at level LV < 3 (see above).
template <int LV>
__device__ __forceinline__ void rhs_core_lv(const SegPar &p, const Trig &t, const double uz[3], const double R[9],
                                            double duz[3], double dR[9])
{
    static_assert(LV == 1 || LV == 2, "level 3 is rhs_core");
    if constexpr (LV == 2) {
        const double sy1 = p.wx[1] * t.s10;              // rhs_core's sy1 with wx_2 = 0
        const double sy2 = -(p.wx[0] * t.s10);
        duz[0] = -(p.g[0] * sy1);
        duz[1] = -(p.g[1] * sy2);
        duz[2] = 0.0;
        const double a = fma(p.wx[1], t.c10, p.wx[0]);
        const double b = sy1;
        const double u0 = uz[0];
        #pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double r0 = R[3 * r], r1 = R[3 * r + 1], r2 = R[3 * r + 2];
            dR[3 * r + 0] = r1 * u0 - r2 * b;
            dR[3 * r + 1] = r2 * a - r0 * u0;
            dR[3 * r + 2] = r0 * b - r1 * a;
        }
    } else {
        duz[0] = duz[1] = duz[2] = 0.0;
        const double a = p.wx[0], u0 = uz[0];         // uy_0 = 0
        #pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double r0 = R[3 * r], r1 = R[3 * r + 1], r2 = R[3 * r + 2];
            dR[3 * r + 0] = r1 * u0;
            dR[3 * r + 1] = r2 * a - r0 * u0;
            dR[3 * r + 2] = -(r1 * a);
        }
    }
}

// ------------------------------------------------------------------------------------------
// scipy RK45 (Dormand-Prince 5(4)) with scipy's step-size controller.
// ------------------------------------------------------------------------------------------
namespace rk {
constexpr double A10 = 1.0 / 5;
constexpr double A20 = 3.0 / 40, A21 = 9.0 / 40;
constexpr double A30 = 44.0 / 45, A31 = -56.0 / 15, A32 = 32.0 / 9;
constexpr double A40 = 19372.0 / 6561, A41 = -25360.0 / 2187, A42 = 64448.0 / 6561, A43 = -212.0 / 729;
constexpr double A50 = 9017.0 / 3168, A51 = -355.0 / 33, A52 = 46732.0 / 5247, A53 = 49.0 / 176,
                 A54 = -5103.0 / 18656;
constexpr double B0 = 35.0 / 384, B2 = 500.0 / 1113, B3 = 125.0 / 192, B4 = -2187.0 / 6784, B5 = 11.0 / 84;
constexpr double E0 = -71.0 / 57600, E2 = 71.0 / 16695, E3 = -71.0 / 1920, E4 = 17253.0 / 339200,
                 E5 = -22.0 / 525, E6 = 1.0 / 40;
constexpr double RTOL = 1e-3, ATOL = 1e-6;
constexpr double INV_SQRT18 = 0.23570226039551584;
// dense-output matrix P (scipy rk.py RK45.P), rows = stages 0..6, columns = powers x^1..x^4
constexpr double P0[4] = {1.0, -8048581381.0 / 2820520608, 8663915743.0 / 2820520608, -12715105075.0 / 11282082432};
constexpr double P1[4] = {0.0, 0.0, 0.0, 0.0};
constexpr double P2[4] = {0.0, 131558114200.0 / 32700410799, -68118460800.0 / 10900136933,
                          87487479700.0 / 32700410799};
constexpr double P3[4] = {0.0, -1754552775.0 / 470086768, 14199869525.0 / 1410260304, -10690763975.0 / 1880347072};
constexpr double P4[4] = {0.0, 127303824393.0 / 49829197408, -318862633887.0 / 49829197408,
                          701980252875.0 / 199316789632};
constexpr double P5[4] = {0.0, -282668133.0 / 205662961, 2019193451.0 / 616988883, -1453857185.0 / 822651844};
constexpr double P6[4] = {0.0, 40617522.0 / 29380423, -110615467.0 / 29380423, 69997945.0 / 29380423};
constexpr int SHAPE_PTS = 30;          // t_eval points per segment (model.py:141 linspace num=30)
}  // namespace rk

// Backbone-shape output of one lane (model.py:66-68,141-164): r at the 30 sorted linspace
// points of every integrated segment (RK45 dense output, scipy rk.py RkDenseOutput), and the
// arclength of each point (ctr_model's Length).  Points beyond `cap` are counted, not stored.
struct ShapeOut {
    double *r;        // [cap][3]
    double *s;        // [cap]
    int cap;
    int count;
};

// numpy.linspace(a, b, 30) element i (numpy 2: i * step + a, step = (b - a) / 29; last = b),
// without contraction.
__device__ __forceinline__ double linspace30(double a, double b, double step, int i)
{
    return i == rk::SHAPE_PTS - 1 ? b : __dadd_rn(__dmul_rn((double)i, step), a);
}

__device__ __forceinline__ void shape_put(ShapeOut *so, double s, const double r[3])
{
    if (so->count < so->cap) {
        so->s[so->count] = s;
        so->r[3 * so->count + 0] = r[0];
        so->r[3 * so->count + 1] = r[1];
        so->r[3 * so->count + 2] = r[2];
    }
    so->count++;
}

// nrej: rejected RK45 attempts.  Fixed-step RK4 never rejects; there it counts the segments run as
// segment maps (matrix powers: every segment of the rigid model, the tube-0-alone tail of the
// compliant one) in bits 16-31 and their square-and-multiply compositions in bits 0-15, and
// nstep counts only the steps taken stage by stage (nfev still counts 4 per RK4 step, mapped or not).
struct FkStats {
    uint32_t nfev, nstep, nrej, nseg, status;
};

// An RK45 FK suspended at the top of its attempt loop (fk_lane<..., RESUME = true>): the state y,
// the parked u_z of tubes 1-2, the controller and the segment cursor.  The FSAL derivative f and
// the trig of y are not stored: both are recomputed from y on resume with the same arithmetic
// that produced them (f = K6 of the accepted step = rhs(y); a rejection leaves f at rhs(y)), so a
// suspended-and-resumed FK is bit-identical to an uninterrupted one.  256 B.
struct FkSuspend {
    double yu[3], ya[3], yr[3], yR[9], uzf[3];
    double t, tb, ha, min_step, prev_end;
    uint32_t remaining, k, flags, pad0;   // flags: 1 need_init, 2 new_step, 4 rejected
    FkStats st;
    uint32_t pad1[3];
};
static_assert(sizeof(FkSuspend) == 256, "FkSuspend layout");

#if defined(CTR_ASM_MARKERS)
// asm-listing build: a comment + scheduling barrier at each block boundary (instruction counts)
#define CTR_STAMP(var)                                   \
    do {                                                 \
        __builtin_amdgcn_sched_barrier(0);               \
        asm volatile(";CTR_MARK " #var ::: "memory");    \
        __builtin_amdgcn_sched_barrier(0);               \
    } while (0)
#else
#define CTR_STAMP(var)
#endif

// Stage derivative storage: u_z' (3), alpha' (3), R' (9).  r' = column 3 of the stage input
// R is folded straight into the B / E accumulators instead of being stored.
struct Stage {
    double uz[3], al[3], R[9];
};

// Full derivative at a state y whose (u_z, R) derivatives are d: builds alpha' and r'.
// MASKED = false: the caller keeps u_z of absent tubes 1 and 2 at 0 (fk_lane), so alpha'_1,2 = u_z
// as is; tube 0 is always masked (its u_z drives the frame even where the tube is absent).
template <bool MASKED = true>
__device__ __forceinline__ void stage_at(const SegPar &p, const Trig &t, const double *uz, const double *R, Stage &k,
                                         double rcol[3])
{
    #pragma unroll
    for (int j = 0; j < 3; ++j) k.al[j] = ((!MASKED && j > 0) || ((p.present >> j) & 1u)) ? uz[j] : 0.0;
    rcol[0] = R[2]; rcol[1] = R[5]; rcol[2] = R[8];
}


// One attempt of RungeKutta._step_impl (rk.py:111-175) from y over h (tnew = t + h) at tube level
// LV < 3 ("Tube levels"; no y pre-curvature, compliant model, no dense output): only the NU u_z and
// NA alpha components the level changes are integrated -- the others keep y's value, their
// derivatives and error terms being exact zeros -- and only the level's trig is evaluated.  Same
// values as fk_lane's own (level-3) attempt for every lane at level LV or below; the error norm's
// partial sums skip only +0 terms, in the same order.
template <int LV, bool CAREFUL>
__device__ __forceinline__ void rk45_attempt_lv(const SegPar &p, double yu[3], double ya[3], double yr[3],
                                                double yR[9], Stage &f, Trig &ty, double &t, double tb, double &ha,
                                                double h, double tnew, bool &rejected, bool &new_step,
                                                bool &need_init, FkStats &st)
{
    using namespace rk;
    static_assert(LV == 1 || LV == 2, "level 3 is fk_lane's own attempt");
    constexpr int NU = LV == 2 ? 2 : 0;      // u_z components that change
    constexpr int NA = LV == 2 ? 2 : 1;      // alpha components that change
    constexpr int NT = LV == 2 ? 2 : 0;      // alpha stage inputs the trig reads
#define CTR_FAL(i) ((i) == 0 ? (((p.present & 1u) != 0u) ? yu[0] : 0.0) : yu[i])
    // f's implied parts: alpha' = masked u_z(y), r' = R(y) e3
    const double fr[3] = {yR[2], yR[5], yR[8]};
    double br[3], er[3];                     // B / E accumulators for r (never an RHS input)
    #pragma unroll
    for (int i = 0; i < 3; ++i) { br[i] = fr[i] * B0; er[i] = fr[i] * E0; }
    Stage K1, K2, K3, K4, K5;
    double ui[3], ai[3], Ri[9], rc[3];
    // stage coefficients pre-multiplied by h: y + sum_j K_j (a_sj h)
    const double a10 = A10 * h;
    const double a20 = A20 * h, a21 = A21 * h;
    const double a30 = A30 * h, a31 = A31 * h, a32 = A32 * h;
    const double a40 = A40 * h, a41 = A41 * h, a42 = A42 * h, a43 = A43 * h;
    const double a50 = A50 * h, a51 = A51 * h, a52 = A52 * h, a53 = A53 * h, a54 = A54 * h;
    auto c1 = [&](double k0, double y) { return fma(k0, a10, y); };
    auto c2 = [&](double k0, double k1, double y) { return fma(k1, a21, fma(k0, a20, y)); };
    auto c3 = [&](double k0, double k1, double k2, double y) { return fma(k2, a32, fma(k1, a31, fma(k0, a30, y))); };
    auto c4 = [&](double k0, double k1, double k2, double k3, double y) {
        return fma(k3, a43, fma(k2, a42, fma(k1, a41, fma(k0, a40, y))));
    };
    auto c5 = [&](double k0, double k1, double k2, double k3, double k4, double y) {
        return fma(k4, a54, fma(k3, a53, fma(k2, a52, fma(k1, a51, fma(k0, a50, y)))));
    };
#define CTR_STAGE(KOUT, EXPR_U, EXPR_A, EXPR_R, BCOEF, ECOEF)                                   \
    {                                                                                          \
        _Pragma("unroll") for (int i = 0; i < 3; ++i) {                                        \
            ui[i] = (i < NU) ? (EXPR_U) : yu[i];                                               \
            if (i < NT) ai[i] = EXPR_A;                                                        \
        }                                                                                      \
        _Pragma("unroll") for (int i = 0; i < 9; ++i) Ri[i] = EXPR_R;                          \
        const Trig tt = trig_lv<LV, CAREFUL>(ai);                                              \
        rhs_core_lv<LV>(p, tt, ui, Ri, KOUT.uz, KOUT.R);                                       \
        stage_at<false>(p, tt, ui, Ri, KOUT, rc);                                              \
        _Pragma("unroll") for (int i = 0; i < 3; ++i) {                                        \
            br[i] += rc[i] * (BCOEF);                                                          \
            er[i] += rc[i] * (ECOEF);                                                          \
        }                                                                                      \
    }
    CTR_STAGE(K1, c1(f.uz[i], yu[i]), c1(CTR_FAL(i), ya[i]), c1(f.R[i], yR[i]), 0.0, 0.0)
    CTR_STAGE(K2, c2(f.uz[i], K1.uz[i], yu[i]), c2(CTR_FAL(i), K1.al[i], ya[i]), c2(f.R[i], K1.R[i], yR[i]), B2, E2)
    CTR_STAGE(K3, c3(f.uz[i], K1.uz[i], K2.uz[i], yu[i]), c3(CTR_FAL(i), K1.al[i], K2.al[i], ya[i]),
              c3(f.R[i], K1.R[i], K2.R[i], yR[i]), B3, E3)
    CTR_STAGE(K4, c4(f.uz[i], K1.uz[i], K2.uz[i], K3.uz[i], yu[i]), c4(CTR_FAL(i), K1.al[i], K2.al[i], K3.al[i], ya[i]),
              c4(f.R[i], K1.R[i], K2.R[i], K3.R[i], yR[i]), B4, E4)
    CTR_STAGE(K5, c5(f.uz[i], K1.uz[i], K2.uz[i], K3.uz[i], K4.uz[i], yu[i]),
              c5(CTR_FAL(i), K1.al[i], K2.al[i], K3.al[i], K4.al[i], ya[i]),
              c5(f.R[i], K1.R[i], K2.R[i], K3.R[i], K4.R[i], yR[i]), B5, E5)
#undef CTR_STAGE
    // y_new (rk.py rk_step) and the error sums without K6
    double nu[3], na[3], nr[3], nR[9];
    double eu[3], ea[3], eR[9];
    const double b0 = B0 * h, b2 = B2 * h, b3 = B3 * h, b4 = B4 * h, b5 = B5 * h;
    auto cb = [&](double k0, double k2, double k3, double k4, double k5, double y) {
        return fma(k5, b5, fma(k4, b4, fma(k3, b3, fma(k2, b2, fma(k0, b0, y)))));
    };
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        nu[i] = (i < NU) ? cb(f.uz[i], K2.uz[i], K3.uz[i], K4.uz[i], K5.uz[i], yu[i]) : yu[i];
        na[i] = (i < NA) ? cb(CTR_FAL(i), K2.al[i], K3.al[i], K4.al[i], K5.al[i], ya[i]) : ya[i];
        nr[i] = yr[i] + h * br[i];
        eu[i] = (i < NU) ? f.uz[i] * E0 + K2.uz[i] * E2 + K3.uz[i] * E3 + K4.uz[i] * E4 + K5.uz[i] * E5 : 0.0;
        ea[i] = (i < NA) ? CTR_FAL(i) * E0 + K2.al[i] * E2 + K3.al[i] * E3 + K4.al[i] * E4 + K5.al[i] * E5 : 0.0;
    }
    #pragma unroll
    for (int i = 0; i < 9; ++i) {
        nR[i] = cb(f.R[i], K2.R[i], K3.R[i], K4.R[i], K5.R[i], yR[i]);
        eR[i] = f.R[i] * E0 + K2.R[i] * E2 + K3.R[i] * E3 + K4.R[i] * E4 + K5.R[i] * E5;
    }
    Stage K6;
    double k6r[3];
    Trig tn = trig_lv<LV, CAREFUL>(na);
    rhs_core_lv<LV>(p, tn, nu, nR, K6.uz, K6.R);
    stage_at<false>(p, tn, nu, nR, K6, k6r);
    st.nfev += 6;
    // error norm as fk_lane's attempt (three partial sums), without the +0 terms
    double acc[3] = {0.0, 0.0, 0.0};
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i < NU) {
            const double xu = fma(K6.uz[i], E6, eu[i]) * ctr_math::rcp_est(fma(ctr_math::absmax(yu[i], nu[i]), RTOL, ATOL));
            acc[0] = fma(xu, xu, acc[0]);
        }
        if (i < NA) {
            const double xa = fma(K6.al[i], E6, ea[i]) * ctr_math::rcp_est(fma(ctr_math::absmax(ya[i], na[i]), RTOL, ATOL));
            acc[1] = fma(xa, xa, acc[1]);
        }
        const double xr = fma(k6r[i], E6, er[i]) * ctr_math::rcp_est(fma(ctr_math::absmax(yr[i], nr[i]), RTOL, ATOL));
        acc[2] = fma(xr, xr, acc[2]);
    }
    #pragma unroll
    for (int i = 0; i < 9; ++i) {
        const double xR = fma(K6.R[i], E6, eR[i]) * ctr_math::rcp_est(fma(ctr_math::absmax(yR[i], nR[i]), RTOL, ATOL));
        acc[i / 3] = fma(xR, xR, acc[i / 3]);
    }
    double en2 = (acc[0] + acc[1]) + acc[2];
    en2 *= h * h;                           // = 18 error_norm^2
    const double en2n = en2 * (1.0 / 18);   // error_norm^2
    // unguarded: for en2n >= 1e300 (or inf / NaN) the root is < 2e-30 (or NaN) and only enters
    // fmax(0.2, fpow) of a rejection, which is 0.2 either way (rk.py:171)
    const double fpow = 0.9 * ctr_math::inv_root10(en2n);
    // accept / reject (fk_lane's attempt does the same)
    const bool ok = en2n < 1.0;
    double factor = (en2n == 0.0) ? 10.0 : fmin(10.0, fpow);
    if (rejected) factor = fmin(1.0, factor);
    ha *= ok ? factor : fmax(0.2, fpow);
    if (__builtin_expect(__ballot(!ok) != 0, 0)) {
        // a lane rejects (rare: the env workload rejects ~1e-3 attempts per FK): its "new" state
        // becomes its old one, so every lane takes the plain assignments below, which cost the
        // allocator at most a copy where per-dword selects on the accept path cost a v_cndmask each
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            nu[i] = ok ? nu[i] : yu[i];
            na[i] = ok ? na[i] : ya[i];
            nr[i] = ok ? nr[i] : yr[i];
            K6.uz[i] = ok ? K6.uz[i] : f.uz[i];
            K6.al[i] = ok ? K6.al[i] : f.al[i];
        }
        #pragma unroll
        for (int i = 0; i < 9; ++i) {
            nR[i] = ok ? nR[i] : yR[i];
            K6.R[i] = ok ? K6.R[i] : f.R[i];
        }
        tn.c10 = ok ? tn.c10 : ty.c10; tn.s10 = ok ? tn.s10 : ty.s10;
        tn.c20 = ok ? tn.c20 : ty.c20; tn.s20 = ok ? tn.s20 : ty.s20;
        tn.c21 = ok ? tn.c21 : ty.c21; tn.s21 = ok ? tn.s21 : ty.s21;
        tnew = ok ? tnew : t;
    }
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i < NU) yu[i] = nu[i];
        if (i < NA) ya[i] = na[i];
        yr[i] = nr[i];
    }
    #pragma unroll
    for (int i = 0; i < 9; ++i) yR[i] = nR[i];
    f = K6;
    ty = tn;
    t = tnew;
    st.nstep += ok ? 1u : 0u;
    st.nrej += ok ? 0u : 1u;
    new_step = ok;
    rejected = ok ? rejected : true;
    if (ok && t - tb >= 0.0) need_init = true;    // segment finished (status 'finished')
#undef CTR_FAL
}

// Forward kinematics of one lane, scipy-RK45 integrator: joints (f64; the env's float32 joints
// promoted exactly as model.py:51 does) -> tip (f64).  RIGID: torsionally rigid variant (GJ -> inf:
// u_z stays 0, the tube angles stay at their joint values, so the trig is computed once).
// RESUME (the pool refill): start from *from when it is non-null, and after `budget` loop
// iterations (segment start + attempt) suspend into *to and return false; true = tip written.
template <bool HAS_UY, bool RIGID, bool SHAPE = false, bool CAREFUL = true, bool RESUME = false>
__device__ bool fk_lane(const SysK &sy, const double q[6], double tip[3], FkStats &st, ShapeOut *so = nullptr,
                        const FkSuspend *from = nullptr, FkSuspend *to = nullptr, int budget = 0)
{
    using namespace rk;
    // f's alpha part is the masked u_z of y (stage_at, and K6 -> f on acceptance): it is read
    // from y instead of being carried in f (three fewer loop-carried doubles)
#define CTR_FAL(i) ((i) == 0 ? (((p.present & 1u) != 0u) ? yu[0] : 0.0) : yu[i])
    const double beta[3] = {(double)q[0], (double)q[1], (double)q[2]};
    double *end_lds = &s_seg_end[0][threadIdx.x];
    const Seg sg = seg_build(sy, beta, end_lds);

    // state y = [u_z(3), alpha(3), r(3), R(9)]
    double yu[3] = {0.0, 0.0, 0.0};
    // u_z of an absent tube (EI = 0) has zero derivative and alpha' = 0 there (model.py:97-102).
    // A tube is present on one contiguous run of segments, so u_z stays 0 before its run; when the
    // run of tube 1 or 2 ends its value is parked in uzf and the live u_z is zeroed, so
    // alpha' = u_z needs no mask in the stages.  The parked value only enters select_initial_step's
    // d0 (common.py:104-106).  Tube 0 keeps its u_z: the frame rotates with u_z,0 even past the
    // tube's tip (model.py:104-107), which set_action's unchecked nesting pass can produce (Q8).
    double uzf[3] = {0.0, 0.0, 0.0};
    double ya[3] = {(double)q[3], (double)q[4], (double)q[5]};
    double yr[3] = {0.0, 0.0, 0.0};
    double yR[9];
    {
        double s0, c0;
        ctr_math::sincos_cw(ya[0], &s0, &c0);                    // R0 = Rz(alpha_0)  model.py:57-60
        yR[0] = c0; yR[1] = -s0; yR[2] = 0.0;
        yR[3] = s0; yR[4] = c0;  yR[5] = 0.0;
        yR[6] = 0.0; yR[7] = 0.0; yR[8] = 1.0;
    }
    Trig ty = trig_of<CAREFUL>(ya);          // trig of the current state's alphas (reused at segment starts)
    Stage f;                        // FSAL derivative at y (alpha' and r' implied by y)
    SegPar p;
    double t = 0.0, tb = 0.0, ha = 0.0, min_step = 0.0, prev_end = 0.0;
    uint32_t remaining = sg.kept;   // kept gaps not yet integrated, in arclength order
    bool need_init = true, new_step = true, rejected = false;
    double sh_a = 0.0, sh_b = 0.0, sh_step = 0.0;   // SHAPE: the segment's t_eval linspace
    bool sh_rev = false;
    int sh_j = 0;                                   // SHAPE: next t_eval point of the segment
    int kcur = 0, iters = 0;                        // RESUME: segment cursor, iterations run
    if constexpr (RESUME) {
        if (from) {
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                yu[i] = from->yu[i]; ya[i] = from->ya[i]; yr[i] = from->yr[i]; uzf[i] = from->uzf[i];
            }
            #pragma unroll
            for (int i = 0; i < 9; ++i) yR[i] = from->yR[i];
            t = from->t; tb = from->tb; ha = from->ha; min_step = from->min_step; prev_end = from->prev_end;
            remaining = from->remaining;
            kcur = (int)from->k;
            need_init = (from->flags & 1u) != 0;
            new_step = (from->flags & 2u) != 0;
            rejected = (from->flags & 4u) != 0;
            st = from->st;
            ty = trig_of<CAREFUL>(ya);
            if (!need_init) {                     // mid-segment: the segment's constants and f = rhs(y)
                p = seg_par_at<HAS_UY, RIGID>(sy, seg_bits(sg, kcur));
                rhs_core<HAS_UY>(p, ty, yu, yR, f.uz, f.R);
            }
        }
    }

    for (;;) {
        CTR_STAMP(ts0);
        if constexpr (RESUME) {
            if (iters >= budget && !(need_init && remaining == 0)) {
                #pragma unroll
                for (int i = 0; i < 3; ++i) {
                    to->yu[i] = yu[i]; to->ya[i] = ya[i]; to->yr[i] = yr[i]; to->uzf[i] = uzf[i];
                }
                #pragma unroll
                for (int i = 0; i < 9; ++i) to->yR[i] = yR[i];
                to->t = t; to->tb = tb; to->ha = ha; to->min_step = min_step; to->prev_end = prev_end;
                to->remaining = remaining;
                to->k = (uint32_t)kcur;
                to->flags = (need_init ? 1u : 0u) | (new_step ? 2u : 0u) | (rejected ? 4u : 0u);
                to->st = st;
                return false;
            }
            ++iters;
        }
        if (need_init) {
            if (remaining == 0) break;
            const int k = __builtin_ctz(remaining);
            remaining &= remaining - 1u;
            if constexpr (RESUME) kcur = k;
            p = seg_par_at<HAS_UY, RIGID>(sy, seg_bits(sg, k));
            #pragma unroll
            for (int j = 1; j < 3; ++j) {
                const bool absent = !((p.present >> j) & 1u);
                uzf[j] = (absent && yu[j] != 0.0) ? yu[j] : uzf[j];
                yu[j] = absent ? 0.0 : yu[j];
            }
            const double endk = end_lds[k * CTR_BLOCK];
            const double a = prev_end, b = endk - 1e-6;          // model.py:141 linspace endpoints
            const double t0 = fmin(a, b);
            tb = fmax(a, b);                                      // :145-151 sorted span
            prev_end = endk;
            if (SHAPE) {
                // t_eval = sorted(linspace(a, b, 30)) (model.py:141-147)
                sh_a = a;
                sh_b = b;
                sh_step = (b - a) / 29.0;
                sh_rev = a > b;
                sh_j = 0;
            }
            // RungeKutta.__init__: f = fun(t0, y0) -- the trig of y is already known
            rhs_core<HAS_UY>(p, ty, yu, yR, f.uz, f.R);
            double fr[3];
            stage_at<false>(p, ty, yu, yR, f, fr);
            st.nfev++;
            st.nseg++;
            const double interval = tb - t0;
            if (interval == 0.0) {                                // OdeSolver.step: t == t_bound
                if (SHAPE)                                        // ConstantDenseOutput(y)
                    for (int j = 0; j < SHAPE_PTS; ++j)
                        shape_put(so, linspace30(sh_a, sh_b, sh_step, sh_rev ? SHAPE_PTS - 1 - j : j), yr);
                continue;
            }
            if (p.present == 0u) {
                // a gap with no tube (joints outside the nesting constraints): the reference's
                // RHS is NaN (1/sum EI = inf, model.py:87-93) and scipy's step loop never ends
                // on the NaN step size; stop with a NaN tip
                yr[0] = yr[1] = yr[2] = NAN;
                st.status |= CTR_STATUS_NAN;
                break;
            }
            // select_initial_step (common.py:68-140), order 4, direction +1
            double isc_u[3], isc_a[3], isc_r[3], isc_R[9], yuref[3];
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                yuref[i] = (i == 0 || ((p.present >> i) & 1u)) ? yu[i] : uzf[i];   // the reference's u_z
                isc_u[i] = ctr_math::rcp_est(ATOL + fabs(yuref[i]) * RTOL);
                isc_a[i] = ctr_math::rcp_est(ATOL + fabs(ya[i]) * RTOL);
                isc_r[i] = ctr_math::rcp_est(ATOL + fabs(yr[i]) * RTOL);
            }
            #pragma unroll
            for (int i = 0; i < 9; ++i) isc_R[i] = ctr_math::rcp_est(ATOL + fabs(yR[i]) * RTOL);
            double s0 = 0.0, s1 = 0.0;
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                s0 += (yuref[i] * isc_u[i]) * (yuref[i] * isc_u[i]) + (ya[i] * isc_a[i]) * (ya[i] * isc_a[i]) +
                      (yr[i] * isc_r[i]) * (yr[i] * isc_r[i]);
                s1 += (f.uz[i] * isc_u[i]) * (f.uz[i] * isc_u[i]) + (CTR_FAL(i) * isc_a[i]) * (CTR_FAL(i) * isc_a[i]) +
                      (fr[i] * isc_r[i]) * (fr[i] * isc_r[i]);
            }
            #pragma unroll
            for (int i = 0; i < 9; ++i) {
                s0 += (yR[i] * isc_R[i]) * (yR[i] * isc_R[i]);
                s1 += (f.R[i] * isc_R[i]) * (f.R[i] * isc_R[i]);
            }
            // d0 = ||y/sc||_rms, d1 = ||f/sc||_rms kept squared (no sqrt on the hot path)
            const double d0sq = s0 * (1.0 / 18), d1sq = s1 * (1.0 / 18);
            // branch-free selects (both sides are cheap; a branch would split the scheduling region)
            const double h0n = 0.01 * ctr_math::sqrt_rsq(s0 * ctr_math::rcp1(s1));
            double h0 = (d0sq < 1e-10 || d1sq < 1e-10) ? 1e-6 : h0n;
            h0 = fmin(h0, interval);
            double u1[3], a1[3], R1[9];
            #pragma unroll
            for (int i = 0; i < 3; ++i) { u1[i] = yu[i] + h0 * f.uz[i]; a1[i] = ya[i] + h0 * CTR_FAL(i); }
            #pragma unroll
            for (int i = 0; i < 9; ++i) R1[i] = yR[i] + h0 * f.R[i];
            Stage f1;
            double f1r[3];
            {
                const Trig t1 = RIGID ? ty : trig_of<CAREFUL>(a1);
                rhs_core<HAS_UY>(p, t1, u1, R1, f1.uz, f1.R);
                stage_at<false>(p, t1, u1, R1, f1, f1r);
            }
            st.nfev++;
            double s2 = 0.0;
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                const double du = (f1.uz[i] - f.uz[i]) * isc_u[i], da = (f1.al[i] - CTR_FAL(i)) * isc_a[i],
                             dr = (f1r[i] - fr[i]) * isc_r[i];
                s2 += du * du + da * da + dr * dr;
            }
            #pragma unroll
            for (int i = 0; i < 9; ++i) {
                const double dR = (f1.R[i] - f.R[i]) * isc_R[i];
                s2 += dR * dR;
            }
            const double ih0 = ctr_math::rcp1(h0);
            const double d2sq = s2 * (1.0 / 18) * ih0 * ih0;            // d2^2
            double h1;
            const double h1a = fmax(1e-6, h0 * 1e-3);
            const double h1b = 0.3981071705534972 * ctr_math::inv_root10(fmax(d1sq, d2sq));   // (0.01/max(d1,d2))^(1/5)
            h1 = (d1sq <= 1e-30 && d2sq <= 1e-30) ? h1a : h1b;
            ha = fmin(fmin(100.0 * h0, h1), interval);
            t = t0;
            need_init = false;
            new_step = true;
        }

        CTR_STAMP(ts1);
        // ---- one attempt of RungeKutta._step_impl (rk.py:111-175) ----
        {
            // new step: min_step = 10 |nextafter(t, inf) - t| and h_abs >= min_step (rk.py:114-119)
            const double ms = 10.0 * ctr_math::gap_up(t);       // = 10 |nextafter(t, inf) - t|
            min_step = new_step ? ms : min_step;
            ha = (new_step && ha < ms) ? ms : ha;
            rejected = new_step ? false : rejected;
            new_step = false;
        }
        if (!(ha >= min_step)) {                     // TOO_SMALL_STEP -> solver failed
            if (ha < min_step) {
                st.status |= CTR_STATUS_STEP_UNDERFLOW;
            } else {                                 // NaN step size (NaN joints): scipy would
                yr[0] = yr[1] = yr[2] = NAN;         // loop forever (as in the gap case)
                st.status |= CTR_STATUS_NAN;
            }
            break;
        }
        double tnew = t + ha;
        if (tnew - tb > 0.0) tnew = tb;
        const double h = tnew - t;
        ha = fabs(h);

        if constexpr (!HAS_UY && !RIGID && !SHAPE) {
            // no active lane of the wave has tube 2 (level 3): the attempt at the wave's tube level
            // ("Tube levels"); the level-3 attempt below stays as it is
            if (__ballot((p.present & 4u) != 0) == 0) {
                if (__ballot((p.present & 2u) != 0) != 0)
                    rk45_attempt_lv<2, CAREFUL>(p, yu, ya, yr, yR, f, ty, t, tb, ha, h, tnew, rejected, new_step,
                                                need_init, st);
                else
                    rk45_attempt_lv<1, CAREFUL>(p, yu, ya, yr, yR, f, ty, t, tb, ha, h, tnew, rejected, new_step,
                                                need_init, st);
                continue;
            }
        }
        // f's implied parts: alpha' = masked u_z(y), r' = R(y) e3
        double fr[3] = {yR[2], yR[5], yR[8]};
        // B / E accumulators for r (never an RHS input)
        double br[3], er[3];
        #pragma unroll
        for (int i = 0; i < 3; ++i) { br[i] = fr[i] * B0; er[i] = fr[i] * E0; }
        double qr[3][4];                             // SHAPE: Q = K^T P for the r components
        if (SHAPE)
            #pragma unroll
            for (int i = 0; i < 3; ++i)
                #pragma unroll
                for (int j = 0; j < 4; ++j) qr[i][j] = fr[i] * P0[j];

        Stage K1, K2, K3, K4, K5;
        double ui[3], ai[3], Ri[9], rc[3];
        // stage coefficients pre-multiplied by h: y + sum_j K_j (a_sj h)
        const double a10 = A10 * h;
        const double a20 = A20 * h, a21 = A21 * h;
        const double a30 = A30 * h, a31 = A31 * h, a32 = A32 * h;
        const double a40 = A40 * h, a41 = A41 * h, a42 = A42 * h, a43 = A43 * h;
        const double a50 = A50 * h, a51 = A51 * h, a52 = A52 * h, a53 = A53 * h, a54 = A54 * h;
        auto c1 = [&](double k0, double y) { return fma(k0, a10, y); };
        auto c2 = [&](double k0, double k1, double y) { return fma(k1, a21, fma(k0, a20, y)); };
        auto c3 = [&](double k0, double k1, double k2, double y) { return fma(k2, a32, fma(k1, a31, fma(k0, a30, y))); };
        auto c4 = [&](double k0, double k1, double k2, double k3, double y) {
            return fma(k3, a43, fma(k2, a42, fma(k1, a41, fma(k0, a40, y))));
        };
        auto c5 = [&](double k0, double k1, double k2, double k3, double k4, double y) {
            return fma(k4, a54, fma(k3, a53, fma(k2, a52, fma(k1, a51, fma(k0, a50, y)))));
        };
#define CTR_STAGE(KOUT, EXPR_U, EXPR_A, EXPR_R, BCOEF, ECOEF, PROW)                            \
        {                                                                                      \
            _Pragma("unroll") for (int i = 0; i < 3; ++i) {                                    \
                ui[i] = EXPR_U;                                                                \
                ai[i] = EXPR_A;                                                                \
            }                                                                                  \
            _Pragma("unroll") for (int i = 0; i < 9; ++i) Ri[i] = EXPR_R;                      \
            const Trig tt = RIGID ? ty : trig_of<CAREFUL>(ai);                                \
            rhs_core<HAS_UY>(p, tt, ui, Ri, KOUT.uz, KOUT.R);                                  \
            stage_at<false>(p, tt, ui, Ri, KOUT, rc);                                          \
            _Pragma("unroll") for (int i = 0; i < 3; ++i) {                                    \
                br[i] += rc[i] * (BCOEF);                                                      \
                er[i] += rc[i] * (ECOEF);                                                      \
            }                                                                                  \
            if (SHAPE)                                                                         \
                _Pragma("unroll") for (int i = 0; i < 3; ++i)                                  \
                    _Pragma("unroll") for (int j = 0; j < 4; ++j) qr[i][j] += rc[i] * PROW[j]; \
        }
        CTR_STAGE(K1, c1(f.uz[i], yu[i]), c1(CTR_FAL(i), ya[i]), c1(f.R[i], yR[i]), 0.0, 0.0, P1)
        CTR_STAGE(K2, c2(f.uz[i], K1.uz[i], yu[i]), c2(CTR_FAL(i), K1.al[i], ya[i]), c2(f.R[i], K1.R[i], yR[i]),
                  B2, E2, P2)
        CTR_STAGE(K3, c3(f.uz[i], K1.uz[i], K2.uz[i], yu[i]), c3(CTR_FAL(i), K1.al[i], K2.al[i], ya[i]),
                  c3(f.R[i], K1.R[i], K2.R[i], yR[i]), B3, E3, P3)
        CTR_STAGE(K4, c4(f.uz[i], K1.uz[i], K2.uz[i], K3.uz[i], yu[i]), c4(CTR_FAL(i), K1.al[i], K2.al[i], K3.al[i], ya[i]),
                  c4(f.R[i], K1.R[i], K2.R[i], K3.R[i], yR[i]), B4, E4, P4)
        CTR_STAGE(K5, c5(f.uz[i], K1.uz[i], K2.uz[i], K3.uz[i], K4.uz[i], yu[i]),
                  c5(CTR_FAL(i), K1.al[i], K2.al[i], K3.al[i], K4.al[i], ya[i]),
                  c5(f.R[i], K1.R[i], K2.R[i], K3.R[i], K4.R[i], yR[i]), B5, E5, P5)
#undef CTR_STAGE
        CTR_STAMP(ts2);
        // y_new (rk.py rk_step) and the error sums without K6
        double nu[3], na[3], nr[3], nR[9];
        double eu[3], ea[3], eR[9];
        const double b0 = B0 * h, b2 = B2 * h, b3 = B3 * h, b4 = B4 * h, b5 = B5 * h;
        auto cb = [&](double k0, double k2, double k3, double k4, double k5, double y) {
            return fma(k5, b5, fma(k4, b4, fma(k3, b3, fma(k2, b2, fma(k0, b0, y)))));
        };
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            nu[i] = cb(f.uz[i], K2.uz[i], K3.uz[i], K4.uz[i], K5.uz[i], yu[i]);
            na[i] = cb(CTR_FAL(i), K2.al[i], K3.al[i], K4.al[i], K5.al[i], ya[i]);
            nr[i] = yr[i] + h * br[i];
            eu[i] = f.uz[i] * E0 + K2.uz[i] * E2 + K3.uz[i] * E3 + K4.uz[i] * E4 + K5.uz[i] * E5;
            ea[i] = CTR_FAL(i) * E0 + K2.al[i] * E2 + K3.al[i] * E3 + K4.al[i] * E4 + K5.al[i] * E5;
        }
        #pragma unroll
        for (int i = 0; i < 9; ++i) {
            nR[i] = cb(f.R[i], K2.R[i], K3.R[i], K4.R[i], K5.R[i], yR[i]);
            eR[i] = f.R[i] * E0 + K2.R[i] * E2 + K3.R[i] * E3 + K4.R[i] * E4 + K5.R[i] * E5;
        }
        Stage K6;
        double k6r[3];
        Trig tn = RIGID ? ty : trig_of<CAREFUL>(na);
        rhs_core<HAS_UY>(p, tn, nu, nR, K6.uz, K6.R);
        stage_at<false>(p, tn, nu, nR, K6, k6r);
        st.nfev += 6;
        // error norm: RMS of h * (K^T E) / (atol + max(|y|, |y_new|) rtol); |h| factored out
        // three independent partial sums: one wave per SIMD exposes the FMA latency of a single
        // 18-long accumulation chain at the end of the attempt, where little else can issue
        double acc[3] = {0.0, 0.0, 0.0};
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double xu = fma(K6.uz[i], E6, eu[i]) * ctr_math::rcp_est(fma(ctr_math::absmax(yu[i], nu[i]), RTOL, ATOL));
            const double xa = fma(K6.al[i], E6, ea[i]) * ctr_math::rcp_est(fma(ctr_math::absmax(ya[i], na[i]), RTOL, ATOL));
            const double xr = fma(k6r[i], E6, er[i]) * ctr_math::rcp_est(fma(ctr_math::absmax(yr[i], nr[i]), RTOL, ATOL));
            acc[0] = fma(xu, xu, acc[0]);
            acc[1] = fma(xa, xa, acc[1]);
            acc[2] = fma(xr, xr, acc[2]);
        }
        #pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double xR = fma(K6.R[i], E6, eR[i]) * ctr_math::rcp_est(fma(ctr_math::absmax(yR[i], nR[i]), RTOL, ATOL));
            acc[i / 3] = fma(xR, xR, acc[i / 3]);
        }
        double en2 = (acc[0] + acc[1]) + acc[2];
        en2 *= h * h;                       // = 18 error_norm^2
        const double en2n = en2 * (1.0 / 18);   // error_norm^2
        // error_norm ** -0.2 = (error_norm^2) ** -0.1
        // unguarded: for en2n >= 1e300 (or inf / NaN) the root is < 2e-30 (or NaN) and only enters
        // fmax(0.2, fpow) of a rejection, which is 0.2 either way (rk.py:171)
        const double fpow = 0.9 * ctr_math::inv_root10(en2n);
        CTR_STAMP(ts3);
        if constexpr (!SHAPE) {
            // accept / reject (rk.py:160-175): every lane takes the new state by plain assignment;
            // a rejecting lane (rare, see rk45_attempt_lv) first sets its new state to its old one
            // inside a wave-uniform branch (DESIGN.md 4.5 log: -2.6 us, bit-equal)
            const bool ok = en2n < 1.0;
            double factor = (en2n == 0.0) ? 10.0 : fmin(10.0, fpow);
            if (rejected) factor = fmin(1.0, factor);
            ha *= ok ? factor : fmax(0.2, fpow);
            if (__builtin_expect(__ballot(!ok) != 0, 0)) {
                // a lane rejects (rare): its "new" state becomes its old one (rk45_attempt_lv)
                #pragma unroll
                for (int i = 0; i < 3; ++i) {
                    nu[i] = ok ? nu[i] : yu[i];
                    na[i] = ok ? na[i] : ya[i];
                    nr[i] = ok ? nr[i] : yr[i];
                    K6.uz[i] = ok ? K6.uz[i] : f.uz[i];
                    K6.al[i] = ok ? K6.al[i] : f.al[i];
                }
                #pragma unroll
                for (int i = 0; i < 9; ++i) {
                    nR[i] = ok ? nR[i] : yR[i];
                    K6.R[i] = ok ? K6.R[i] : f.R[i];
                }
                tn.c10 = ok ? tn.c10 : ty.c10; tn.s10 = ok ? tn.s10 : ty.s10;
                tn.c20 = ok ? tn.c20 : ty.c20; tn.s20 = ok ? tn.s20 : ty.s20;
                tn.c21 = ok ? tn.c21 : ty.c21; tn.s21 = ok ? tn.s21 : ty.s21;
                tnew = ok ? tnew : t;
            }
            #pragma unroll
            for (int i = 0; i < 3; ++i) { yu[i] = nu[i]; ya[i] = na[i]; yr[i] = nr[i]; }
            #pragma unroll
            for (int i = 0; i < 9; ++i) yR[i] = nR[i];
            f = K6;
            ty = tn;
            t = tnew;
            st.nstep += ok ? 1u : 0u;
            st.nrej += ok ? 0u : 1u;
            new_step = ok;
            rejected = ok ? rejected : true;
            if (ok && t - tb >= 0.0) need_init = true;    // segment finished (status 'finished')
        } else if (en2n < 1.0) {
            double factor = (en2n == 0.0) ? 10.0 : fmin(10.0, fpow);
            if (rejected) factor = fmin(1.0, factor);
            ha *= factor;
            if (SHAPE) {
                // ivp.py t_eval: the points in (t_old, t_new] (and t0 itself on the first step)
                // from this step's dense output y_old + h Q [x, x^2, x^3, x^4], x = (s - t_old)/h
                #pragma unroll
                for (int i = 0; i < 3; ++i)
                    #pragma unroll
                    for (int j = 0; j < 4; ++j) qr[i][j] += k6r[i] * P6[j];
                while (sh_j < SHAPE_PTS) {
                    const double te = linspace30(sh_a, sh_b, sh_step, sh_rev ? SHAPE_PTS - 1 - sh_j : sh_j);
                    if (te > tnew) break;
                    const double x = (te - t) / h;
                    const double x2 = x * x, x3 = x2 * x, x4 = x3 * x;
                    double rp[3];
                    #pragma unroll
                    for (int i = 0; i < 3; ++i)
                        rp[i] = h * (qr[i][0] * x + qr[i][1] * x2 + qr[i][2] * x3 + qr[i][3] * x4) + yr[i];
                    shape_put(so, te, rp);
                    ++sh_j;
                }
            }
            #pragma unroll
            for (int i = 0; i < 3; ++i) { yu[i] = nu[i]; ya[i] = na[i]; yr[i] = nr[i]; }
            #pragma unroll
            for (int i = 0; i < 9; ++i) yR[i] = nR[i];
            f = K6;
            ty = tn;
            t = tnew;
            st.nstep++;
            new_step = true;
            if (t - tb >= 0.0) need_init = true;    // segment finished (status 'finished')
        } else {
            ha *= fmax(0.2, fpow);
            rejected = true;
            st.nrej++;
        }
    }
    tip[0] = yr[0]; tip[1] = yr[1]; tip[2] = yr[2];
    if (isnan(tip[0]) || isnan(tip[1]) || isnan(tip[2])) st.status |= CTR_STATUS_NAN;
    return true;
#undef CTR_FAL
}

// ------------------------------------------------------------------------------------------
// Fixed-step classical RK4 of the same ODE (throughput / convergence mode, BASELINE configs 2
// and 5).  Each kept segment span [t0, tb] (the same spans as the RK45 path) is split into
// n = max(1, ceil((tb - t0) * steps_per_m)) equal steps.  Lanes stay in lock-step: one loop
// iteration = one RK4 step of whichever segment the lane is in, at the wave's tube level; the
// segments of constant curvature (all of them for the rigid model, the trailing tube-0-alone ones
// for the compliant model) run afterwards as segment maps (fk_lane_rk4).
// ------------------------------------------------------------------------------------------
// Torsionally rigid model: u_z stays 0 and the tube angles keep their joint values, so on a
// segment the curvature u is constant and the ODE is linear, Y' = Y A with Y = [[R, r], [0, 1]]
// and A = [[W, e3], [0, 0]], W = [u]x.  One classical RK4 step of a linear autonomous ODE is
// exactly Y <- Y T(hA), T(X) = I + X + X^2/2 + X^3/6 + X^4/24 (its stages collapse to the degree-4
// Taylor polynomial), i.e. R <- R Q, r <- R m + r with
//   P = I + (hW/2)(I + (hW/3)(I + hW/4)),  Q = I + hW P,  m = h P e3,
// and the segment's n steps are M^n, computed by square-and-multiply on the coefficients of
// polynomials in W (rigid_segment_map below); results agree with stepping the stages to rounding.
// Affine maps applied to row vectors, Y -> Y [[Q, m], [0, 1]]: (Q1, m1) <- (Q1 Q2, Q1 m2 + m1).
__device__ __forceinline__ void affine_compose(double Q1[9], double m1[3], const double Q2[9], const double m2[3])
{
    double Q[9], m[3];
    #pragma unroll
    for (int r = 0; r < 3; ++r) {
        #pragma unroll
        for (int c = 0; c < 3; ++c)
            Q[3 * r + c] = fma(Q1[3 * r + 2], Q2[6 + c], fma(Q1[3 * r + 1], Q2[3 + c], Q1[3 * r] * Q2[c]));
        m[r] = fma(Q1[3 * r + 2], m2[2], fma(Q1[3 * r + 1], m2[1], fma(Q1[3 * r], m2[0], m1[r])));
    }
    #pragma unroll
    for (int i = 0; i < 9; ++i) Q1[i] = Q[i];
    #pragma unroll
    for (int i = 0; i < 3; ++i) m1[i] = m[i];
}

// The powers M^n of a segment's one-step map, without 3x3 products.  W = [w]x with w = (u_x0,
// u_y0, u_z0) satisfies W^3 = -theta^2 W (theta^2 = |w|^2), so every polynomial in W is
// a I + b W + c W^2: the step map is Q = I + (h - h^3 th^2/6) W + (h^2/2 - h^4 th^2/24) W^2 and
// m = h P e3 with P = I + (h/2 - h^3 th^2/24) W + (h^2/6) W^2 (the Q and P above with W^3
// reduced), and composing two maps of the same segment, (Q1 Q2, Q1 m2 + m1), is two products of
// such triples (10 flop each).  Square-and-multiply on the triples, then one expansion to the
// 3 x 4 map (W^2 = w w^T - theta^2 I).  Equal to stepping the RK4 stages up to rounding.
struct WPoly {
    double a, b, c;    // a I + b W + c W^2
};

__device__ __forceinline__ WPoly wpoly_mul(const WPoly &x, const WPoly &y, double th2)
{
    WPoly r;
    r.a = x.a * y.a;
    r.b = fma(x.a, y.b, fma(x.b, y.a, -th2 * fma(x.b, y.c, x.c * y.b)));
    r.c = fma(x.a, y.c, fma(x.c, y.a, fma(x.b, y.b, -th2 * (x.c * y.c))));
    return r;
}

// (Q, m) <- (Q Q2, Q m2 + m) on the triples
__device__ __forceinline__ void wmap_compose(WPoly &q, WPoly &m, const WPoly &q2, const WPoly &m2, double th2)
{
    const WPoly qm = wpoly_mul(q, m2, th2);
    q = wpoly_mul(q, q2, th2);
    m.a += qm.a;
    m.b += qm.b;
    m.c += qm.c;
}

// The segment's n RK4 steps of size h (curvature triple w from the segment's constants) as one
// 3 x 4 map Q [9], m [3].  Returns the number of triple compositions executed.
template <bool HAS_UY>
__device__ __forceinline__ int rigid_segment_map(const SegPar &p, const Trig &t, const double uz[3], double h, int n,
                                                 double Q[9], double m[3])
{
    const double I3[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};
    double W[9], dz[3];
    rhs_core<HAS_UY>(p, t, uz, I3, dz, W);            // I [w]x = W
    const double wx = W[7], wy = W[2], wz = W[3];
    const double th2 = fma(wx, wx, fma(wy, wy, wz * wz));
    const double h2 = h * h, h3 = h2 * h;
    WPoly sq = {1.0, fma(-h3 * th2, 1.0 / 6.0, h), fma(-h2 * h2 * th2, 1.0 / 24.0, 0.5 * h2)};
    WPoly sm = {h, h * fma(-h3 * th2, 1.0 / 24.0, 0.5 * h), h * (h2 * (1.0 / 6.0))};
    WPoly aq = {1.0, 0.0, 0.0}, am = {0.0, 0.0, 0.0};
    int ncomp = 0;
    for (int e = n;;) {
        if (e & 1) { wmap_compose(aq, am, sq, sm, th2); ++ncomp; }   // acc <- acc M^(2^j)
        e >>= 1;
        if (!e) break;
        const WPoly q2 = sq, m2 = sm;
        wmap_compose(sq, sm, q2, m2, th2);
        ++ncomp;
    }
    const double w[3] = {wx, wy, wz};
    const double d = fma(-aq.c, th2, aq.a);
    #pragma unroll
    for (int r = 0; r < 3; ++r)
        #pragma unroll
        for (int c = 0; c < 3; ++c)
            Q[3 * r + c] = fma(aq.c * w[r], w[c], fma(aq.b, W[3 * r + c], r == c ? d : 0.0));
    // m = am.a e3 + am.b W e3 + am.c (w w_z - theta^2 e3), W e3 = (w_y, -w_x, 0)
    m[0] = fma(am.b, wy, am.c * (wx * wz));
    m[1] = fma(-am.b, wx, am.c * (wy * wz));
    m[2] = fma(am.c, fma(wz, wz, -th2), am.a);
    return ncomp;
}

// One classical RK4 step of the compliant model over h at tube level LV ("Tube levels": 3 = the
// full RHS; 2 = tube 2 absent, so u_z,2 and alpha_2 keep their values -- their derivatives are
// exact zeros, alpha' being masked by presence -- and only sin/cos(alpha_1 - alpha_0) is needed).
// The level-2 form gives rhs_core's values up to the sign of zero results, so a lane at level 2
// gets the same bits from either form; a wave runs the highest level one of its active lanes needs.
template <int LV, bool HAS_UY, bool CAREFUL>
__device__ __forceinline__ void rk4_step(const SegPar &p, double h, double yu[3], double ya[3], double yr[3],
                                         double yR[9])
{
    static_assert(LV == 2 || LV == 3, "level 1 runs in closed form (rk4_tail_maps)");
    static_assert(LV == 3 || !HAS_UY, "tube levels assume no y pre-curvature");
    constexpr int N = LV == 3 ? 3 : 2;          // u_z / alpha components that change
    auto rhs = [&](const double u[3], const double a[3], const double R[9], Stage &k, double rc[3]) {
        if constexpr (LV == 3) {
            const Trig tt = trig_of<CAREFUL>(a);
            rhs_core<HAS_UY>(p, tt, u, R, k.uz, k.R);
            stage_at(p, tt, u, R, k, rc);
        } else {
            const Trig tt = trig_lv<2, CAREFUL>(a);
            rhs_core_lv<2>(p, tt, u, R, k.uz, k.R);
            stage_at(p, tt, u, R, k, rc);
        }
    };
    Stage k1, k2, k3, k4;
    double r1[3], r2[3], r3[3], r4[3];
    double ui[3], ai[3], Ri[9];
    rhs(yu, ya, yR, k1, r1);
    const double h2 = 0.5 * h;
#define CTR_RK4_STAGE(KIN, KOUT, ROUT, C)                                                      \
    {                                                                                          \
        _Pragma("unroll") for (int i = 0; i < 3; ++i) {                                        \
            ui[i] = (i < N) ? fma(KIN.uz[i], C, yu[i]) : yu[i];                                \
            ai[i] = (i < N) ? fma(KIN.al[i], C, ya[i]) : ya[i];                                \
        }                                                                                      \
        _Pragma("unroll") for (int i = 0; i < 9; ++i) Ri[i] = fma(KIN.R[i], C, yR[i]);         \
        rhs(ui, ai, Ri, KOUT, ROUT);                                                           \
    }
    CTR_RK4_STAGE(k1, k2, r2, h2)
    CTR_RK4_STAGE(k2, k3, r3, h2)
    CTR_RK4_STAGE(k3, k4, r4, h)
#undef CTR_RK4_STAGE
    const double h6 = h * (1.0 / 6.0);
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i < N) {
            yu[i] = fma(h6, k1.uz[i] + 2.0 * (k2.uz[i] + k3.uz[i]) + k4.uz[i], yu[i]);
            ya[i] = fma(h6, k1.al[i] + 2.0 * (k2.al[i] + k3.al[i]) + k4.al[i], ya[i]);
        }
        yr[i] = fma(h6, r1[i] + 2.0 * (r2[i] + r3[i]) + r4[i], yr[i]);
    }
    #pragma unroll
    for (int i = 0; i < 9; ++i) yR[i] = fma(h6, k1.R[i] + 2.0 * (k2.R[i] + k3.R[i]) + k4.R[i], yR[i]);
}

// The plan of a fixed-step RK4 FK, computed for every kept gap before any integration (one
// convergent block instead of a division and a ceil at every segment start, which run under
// exec masks whenever some lane of the wave starts a segment): step count n_k and size h_k per
// gap in this lane's LDS columns, the gaps with steps to take, and the gaps integrated in closed
// form.  Gap k spans [S_k, S_{k+1} - 1e-6] (model.py:141, reversed spans sorted as :145-151) with
// n = max(1, ceil(len * steps_per_m)) equal steps (oracle rk4_span).  A segment whose RHS has a
// constant curvature runs as one segment map (rigid_segment_map): every gap of the rigid model,
// and with the compliant model (no y pre-curvature) the trailing gaps where tube 0 is alone ("Tube
// levels": u' = 0 there; the present set only shrinks along a backbone, so they come last).  A gap
// over RK4_MAX_STEPS steps ends the plan there (CTR_STATUS_TOO_LONG, NaN tip), as the oracle stops.
__shared__ int s_seg_n[9][CTR_BLOCK];

struct Rk4Plan {
    uint32_t step;     // kept gaps integrated stage by stage, in arclength order
    uint32_t tail;     // kept gaps after them, each as one segment map
    bool too_long;
};

template <bool LEVELS, bool RIGID>
__device__ __forceinline__ Rk4Plan rk4_plan(const Seg &sg, double *end_lds, int *n_lds, double steps_per_m)
{
    Rk4Plan pl = {0u, 0u, false};
    double prev_end = 0.0;
    uint32_t live = 0u;                       // gaps with at least one step
    #pragma unroll
    for (int k = 0; k < 9; ++k) {
        if (!((sg.kept >> k) & 1u) || pl.too_long) continue;
        const double endk = end_lds[k * CTR_BLOCK];
        const double a = prev_end, b = endk - 1e-6;
        const double len = fmax(a, b) - fmin(a, b);
        prev_end = endk;
        if (!(len > 0.0)) continue;
        const double nf = ceil(len * steps_per_m);
        if (!(nf <= (double)RK4_MAX_STEPS)) {  // joints far outside the Box
            pl.too_long = true;
            continue;
        }
        const int n = max(1, (int)nf);
        end_lds[k * CTR_BLOCK] = len / n;      // h_k replaces the gap's end (not read again)
        n_lds[k * CTR_BLOCK] = n;
        live |= 1u << k;
    }
    if (RIGID) {
        pl.tail = live;
    } else if (LEVELS) {
        // tube 0 alone on gap k: present bits (pc bits 9 i + k) = {0}
        const uint32_t t0 = (uint32_t)(sg.pc & 0x1FFu), t1 = (uint32_t)((sg.pc >> 9) & 0x1FFu),
                       t2 = (uint32_t)((sg.pc >> 18) & 0x1FFu);
        const uint32_t notalone = live & ~(t0 & ~t1 & ~t2);
        const uint32_t upto = notalone ? (2u << (31 - __builtin_clz(notalone))) - 1u : 0u;
        pl.step = live & upto;
        pl.tail = live & ~upto;
    } else {
        pl.step = live;
    }
    return pl;
}

// RESUME (the pool refill, compliant model): start from *from when it is non-null, and after
// `budget` RK4 steps suspend into *to and return false (true = tip written).  The suspended state
// is y, the gap cursor (the remaining stepped gaps, the current one and its steps left) and the
// counters; the plan is a pure function of the joints and is rebuilt on resume, so a suspended-
// and-resumed FK is bit-identical to an uninterrupted one (FkSuspend: remaining, k, flags = steps
// left).
template <bool HAS_UY, bool RIGID, bool CAREFUL = true, bool RESUME = false>
__device__ bool fk_lane_rk4(const SysK &sy, const double q[6], double tip[3], FkStats &st, double steps_per_m,
                            const FkSuspend *from = nullptr, FkSuspend *to = nullptr, int budget = 0)
{
    constexpr bool LEVELS = !HAS_UY && !RIGID;
    static_assert(!RESUME || !RIGID, "the rigid model's FKs run as segment maps, nothing to suspend");
    const double beta[3] = {q[0], q[1], q[2]};
    double *end_lds = &s_seg_end[0][threadIdx.x];
    int *n_lds = &s_seg_n[0][threadIdx.x];
    const Seg sg = seg_build(sy, beta, end_lds);
    const Rk4Plan pl = rk4_plan<LEVELS, RIGID>(sg, end_lds, n_lds, steps_per_m);
    double yu[3] = {0.0, 0.0, 0.0};
    double ya[3] = {q[3], q[4], q[5]};
    double yr[3] = {0.0, 0.0, 0.0};
    double yR[9];
    const bool resumed = RESUME && from != nullptr;
    if (!resumed) {
        st.nseg += (uint32_t)__builtin_popcount(sg.kept);
        double s0, c0;
        sincos_lds(ya[0], s0, c0);
        yR[0] = c0; yR[1] = -s0; yR[2] = 0.0;
        yR[3] = s0; yR[4] = c0;  yR[5] = 0.0;
        yR[6] = 0.0; yR[7] = 0.0; yR[8] = 1.0;
    }
    if constexpr (!RIGID) {
        // stepped gaps: one RK4 step per iteration (lanes in lock-step, each in its own gap); the
        // step runs at the wave's tube level
        SegPar p;
        double h = 0.0;
        int left = 0;                         // steps left in the current gap
        bool lv3 = true;
        uint32_t rem = pl.step;
        int kcur = 0, iters = 0;              // RESUME: the current gap, steps run here
        if constexpr (RESUME) {
            if (resumed) {
                #pragma unroll
                for (int i = 0; i < 3; ++i) { yu[i] = from->yu[i]; ya[i] = from->ya[i]; yr[i] = from->yr[i]; }
                #pragma unroll
                for (int i = 0; i < 9; ++i) yR[i] = from->yR[i];
                rem = from->remaining;
                kcur = (int)from->k;
                left = (int)from->flags;
                st = from->st;
                if (left > 0) {
                    p = seg_par_at<HAS_UY, false>(sy, seg_bits(sg, kcur));
                    h = end_lds[kcur * CTR_BLOCK];
                    lv3 = (p.present & 4u) != 0u || p.present == 0u;
                }
            }
        }
        for (;;) {
            if constexpr (RESUME) {
                if (iters >= budget && (left > 0 || rem != 0u)) {
                    #pragma unroll
                    for (int i = 0; i < 3; ++i) { to->yu[i] = yu[i]; to->ya[i] = ya[i]; to->yr[i] = yr[i]; }
                    #pragma unroll
                    for (int i = 0; i < 9; ++i) to->yR[i] = yR[i];
                    to->remaining = rem;
                    to->k = (uint32_t)kcur;
                    to->flags = (uint32_t)left;
                    to->st = st;
                    return false;
                }
                ++iters;
            }
            if (left == 0) {
                if (rem == 0u) break;
                const int k = __builtin_ctz(rem);
                rem &= rem - 1u;
                if constexpr (RESUME) kcur = k;
                p = seg_par_at<HAS_UY, false>(sy, seg_bits(sg, k));
                h = end_lds[k * CTR_BLOCK];
                left = n_lds[k * CTR_BLOCK];
                lv3 = (p.present & 4u) != 0u || p.present == 0u;
            }
            bool lower = false;
            if constexpr (LEVELS) lower = __ballot(lv3) == 0;
            if constexpr (LEVELS) {
                if (lower) rk4_step<2, false, CAREFUL>(p, h, yu, ya, yr, yR);
                else rk4_step<3, false, CAREFUL>(p, h, yu, ya, yr, yR);
            } else {
                rk4_step<3, HAS_UY, CAREFUL>(p, h, yu, ya, yr, yR);
            }
            st.nfev += 4;
            st.nstep++;
            --left;
        }
    }
    // closed-form gaps (every lane of the wave together): [R | r] M^n per gap (rigid_segment_map).
    // Rigid: the tube angles keep their joint values.  Compliant level 1: u = (u_x,0, 0, u_z,0) is
    // constant (wx_1 = wx_2 = 0 make the trig irrelevant); alpha is not advanced, nothing reads it.
    const Trig tc = RIGID ? trig_of<CAREFUL>(ya) : Trig{0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    uint32_t tail = pl.tail;
    while (__ballot(tail != 0u) != 0) {
        if (tail != 0u) {
            const int k = __builtin_ctz(tail);
            tail &= tail - 1u;
            const SegPar p = seg_par_at<HAS_UY, RIGID>(sy, seg_bits(sg, k));
            const int n = n_lds[k * CTR_BLOCK];
            double aq[9], am[3];
            const int ncomp = rigid_segment_map<HAS_UY>(p, tc, yu, end_lds[k * CTR_BLOCK], n, aq, am);
            double nR[9];
            #pragma unroll
            for (int r = 0; r < 3; ++r) {
                #pragma unroll
                for (int c = 0; c < 3; ++c)
                    nR[3 * r + c] = fma(yR[3 * r + 2], aq[6 + c], fma(yR[3 * r + 1], aq[3 + c], yR[3 * r] * aq[c]));
                yr[r] = fma(yR[3 * r + 2], am[2], fma(yR[3 * r + 1], am[1], fma(yR[3 * r], am[0], yr[r])));
            }
            #pragma unroll
            for (int i = 0; i < 9; ++i) yR[i] = nR[i];
            st.nfev += 4u * (uint32_t)n;      // the RK4 steps the map stands for (oracle nfev)
            st.nrej += (1u << 16) + (uint32_t)ncomp;   // one segment map + its compositions
        }
    }
    if (pl.too_long) {
        yr[0] = yr[1] = yr[2] = NAN;
        st.status |= CTR_STATUS_TOO_LONG | CTR_STATUS_NAN;
    }
    tip[0] = yr[0]; tip[1] = yr[1]; tip[2] = yr[2];
    if (isnan(tip[0]) || isnan(tip[1]) || isnan(tip[2])) st.status |= CTR_STATUS_NAN;
    return true;
}

// Rigid model + fixed-step RK4 with one env on a group of SEG_GROUP consecutive lanes (k_step for
// BASELINE configs[1]): every lane segments the same joints; lane j takes the env's j-th kept
// segment and raises its one-step map to the segment's step count (as fk_lane_rk4 does segment
// after segment), and the group forms the ordered product M_0 M_1 ... in log2 SEG_GROUP shuffle
// rounds.  Joints with beta <= 0 (the action Box) keep at most 6 segments: the four points
// 0, beta_0..2 are <= 0, so the first three gaps never end after s = 0.  Every lane of the wave
// must call it.  Tips agree with fk_lane_rk4 to rounding (the products associate differently).
constexpr int SEG_GROUP = 8;

// __shfl_down(x, OFF) inside a 16-lane DPP row (row_shl: lane i reads lane i + OFF of its row):
// one v_mov_dpp per dword instead of an LDS-crossbar ds_bpermute.  Lanes whose source lies past
// the row read 0; fk_group_rigid4 uses only lanes whose source is inside their own 8-lane group.
template <int OFF>
__device__ __forceinline__ int dpp_down(int x)
{
    return __builtin_amdgcn_update_dpp(0, x, 0x100 + OFF, 0xF, 0xF, true);
}

template <int OFF>
__device__ __forceinline__ double dpp_down(double x)
{
    const long long v = __double_as_longlong(x);
    const int lo = dpp_down<OFF>((int)(v & 0xffffffffll)), hi = dpp_down<OFF>((int)(v >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// seg_build for an 8-lane group that shares one env (Segment.py:6-61): the group ranks its 10
// points between its lanes (lane j ranks points j and j + 8) and passes the sorted values and the
// argsort positions through LDS, instead of every lane running the 45-comparator network.  The
// rank of point i by (value, index) is its place in the network's stable order, so the sorted
// values, positions and gap lengths are the network's bit for bit.  A NaN point (no total order)
// takes the network.  Every lane of the wave must call it.
__shared__ double s_gsort[CTR_BLOCK / SEG_GROUP][10];
__shared__ uint8_t s_gpos[CTR_BLOCK / SEG_GROUP][16];

__device__ __forceinline__ Seg seg_build_group(const ctr_system_t &sy, const double beta[3], double *end_lds, int j)
{
#pragma clang fp contract(off)
    double v[10];
    v[0] = 0.0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double dtip = sy.L[i] + beta[i];    // Segment.py:11-12
        v[1 + i] = beta[i];
        v[4 + i] = dtip - sy.Lc[i];
        v[7 + i] = dtip;
    }
    bool nan = false;
    #pragma unroll
    for (int i = 1; i < 10; ++i) nan |= v[i] != v[i];
    if (__ballot(nan) != 0) return seg_build(sy, beta, end_lds);
    const int g = threadIdx.x / SEG_GROUP;
    // point j (0..7) and point 8 + j (lanes 0 and 1)
    double va = v[0];
    #pragma unroll
    for (int m = 1; m < SEG_GROUP; ++m) va = (j == m) ? v[m] : va;
    const double vb = (j == 0) ? v[8] : v[9];
    int ra = 0, rb = 0;
    #pragma unroll
    for (int m = 0; m < 10; ++m) {
        ra += (v[m] < va || (v[m] == va && m < j)) ? 1 : 0;
        rb += (v[m] < vb || (v[m] == vb && m < 8 + j)) ? 1 : 0;
    }
    s_gsort[g][ra] = va;
    s_gpos[g][j] = (uint8_t)ra;
    if (j < 2) {
        s_gsort[g][rb] = vb;
        s_gpos[g][8 + j] = (uint8_t)rb;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    #pragma unroll
    for (int k = 0; k < 10; ++k) v[k] = s_gsort[g][k];
    double len[9];
    uint32_t zero = 0;                    // bit k: gap k floored to zero length
    #pragma unroll
    for (int k = 0; k < 9; ++k) {
        len[k] = 1e-5 * floor(1e5 * (v[k + 1] - v[k]));   // Segment.py:16
        zero |= (len[k] == 0.0) ? (1u << k) : 0u;
    }
    auto zero_at = [&](int x) { return ((zero >> x) & 1u) != 0u; };
    uint64_t pc = 0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {         // as seg_build (Segment.py:29-36)
        int a = s_gpos[g][i + 1], b = s_gpos[g][i + 4], c = s_gpos[g][i + 7];
        if (zero_at(a)) a += 1;
        if (zero_at(b)) b += 1;
        if (zero_at(a)) a += 1;
        if (c <= 8 && zero_at(c)) c += 1;
        const uint32_t upto_c = (1u << c) - 1u;
        const uint32_t pres = upto_c & ~((1u << a) - 1u) & 0x1FFu;
        const uint32_t curv = upto_c & ~((1u << b) - 1u) & 0x1FFu;
        pc |= ((uint64_t)pres << (9 * i)) | ((uint64_t)curv << (27 + 9 * i));
    }
    const double bmin = fmin(fmin(beta[0], beta[1]), beta[2]);
    Seg sg;
    sg.kept = 0;
    sg.pc = pc;
    double cum = 0.0;
    #pragma unroll
    for (int k = 0; k < 9; ++k) {         // Segment.py:46-55
        cum += len[k];
        end_lds[k * CTR_BLOCK] = cum + bmin;
        sg.kept |= ((len[k] != 0.0) && (cum + bmin > 0.0)) ? (1u << k) : 0u;
    }
    return sg;
}

template <bool HAS_UY, bool CAREFUL>
__device__ void fk_group_rigid4(const SysK &sy, const double q[6], int j, double tip[3], FkStats &st,
                                double steps_per_m)
{
    const double beta[3] = {q[0], q[1], q[2]};
    double *end_lds = &s_seg_end[0][threadIdx.x];
    const Seg sg = seg_build_group(sy, beta, end_lds, j);
    const double ya[3] = {q[3], q[4], q[5]};
    const double yu[3] = {0.0, 0.0, 0.0};
    const Trig tconst = trig_of<CAREFUL>(ya);
    // the lane's kept gap (the j-th set bit) and the end of the kept gap before it
    uint32_t rem = sg.kept;
    double prev_end = 0.0;
    for (int i = 0; i < j && rem != 0u; ++i) {
        prev_end = end_lds[__builtin_ctz(rem) * CTR_BLOCK];
        rem &= rem - 1u;
    }
    double aq[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0}, am[3] = {0.0, 0.0, 0.0};
    int nsteps = 0;
    bool too_long = false;
    if (rem != 0u) {
        const int k = __builtin_ctz(rem);
        SegPar p = seg_par(sy, seg_bits(sg, k), true);
        if (!HAS_UY) seg_fold_inv(p);
        const double endk = end_lds[k * CTR_BLOCK];
        const double a = prev_end, b = endk - 1e-6;
        const double len = fmax(a, b) - fmin(a, b);
        const double nf = ceil(len * steps_per_m);
        too_long = len > 0.0 && !(nf <= (double)RK4_MAX_STEPS);
        const int left = (len > 0.0 && !too_long) ? max(1, (int)nf) : 0;
        if (left > 0) {
            rigid_segment_map<HAS_UY>(p, tconst, yu, len / left, left, aq, am);
            nsteps = left;
        }
    }
    if (too_long) am[0] = NAN;                       // the product (and the tip) turns NaN
    int any_long = too_long ? 1 : 0;
    #pragma unroll
    for (int off = 1; off < SEG_GROUP; off <<= 1) any_long |= __shfl_xor(any_long, off, SEG_GROUP);
    // ordered product onto the group's lane 0: round r joins lane j with lane j + 2^r (DPP row
    // shifts: the 8-lane groups sit inside 16-lane rows)
    static_assert(SEG_GROUP == 8, "the DPP rounds below are written for 8-lane groups");
    auto join = [&](auto off_tag) {
        constexpr int off = decltype(off_tag)::value;
        double oq[9], om[3];
        #pragma unroll
        for (int i = 0; i < 9; ++i) oq[i] = dpp_down<off>(aq[i]);
        #pragma unroll
        for (int i = 0; i < 3; ++i) om[i] = dpp_down<off>(am[i]);
        const int on = dpp_down<off>(nsteps);
        if ((j & (2 * off - 1)) == 0) {
            affine_compose(aq, am, oq, om);
            nsteps += on;
        }
    };
    join(std::integral_constant<int, 1>{});
    join(std::integral_constant<int, 2>{});
    join(std::integral_constant<int, 4>{});
    // Y = [Rz(alpha_0) | 0] times the product: r = Rz(alpha_0) m  (model.py:57-60)
    double s0, c0;
    sincos_lds(ya[0], s0, c0);
    tip[0] = fma(-s0, am[1], c0 * am[0]);
    tip[1] = fma(c0, am[1], s0 * am[0]);
    tip[2] = am[2];
    st.nfev += 4u * (uint32_t)nsteps;
    st.nstep += (uint32_t)nsteps;
    st.nseg += (uint32_t)__builtin_popcount(sg.kept);
    if (any_long) st.status |= CTR_STATUS_TOO_LONG;
    if (isnan(tip[0]) || isnan(tip[1]) || isnan(tip[2])) st.status |= CTR_STATUS_NAN;
}

// ------------------------------------------------------------------------------------------
// Fixed-step RK4 of the compliant model (no y pre-curvature) with one env on an adjacent lane PAIR
// (k_step for BASELINE configs[4], 512-lane workgroups).  Both lanes run one
// instruction stream on different state slots:
//   lane 0: A = R row 0, B = R row 1, rA = r_0, rB = r_1
//   lane 1: A = R row 2,              rA = r_2                 (B, rB idle, kept at 0)
// and each lane carries tube 0's twist (u_z,0, alpha_0) and that of its own tube "a" (lane 0:
// tube 1, lane 1: tube 2; the other is tube "b").  Per RHS each lane evaluates ONE table sincos,
// of alpha_a - alpha_0 (x = V[1] - V[0] on both lanes: no select), and receives the partner's, of
// alpha_b - alpha_0, with one quad_perm DPP swap: so neither alpha_b nor u_z,b is needed locally.
// The twist derivatives are written in (a, b) form with per-lane constants (wx_a, wx_b, g_a), and
// the frame rows use the lane's own u = (u_x,0, u_y,0, u_z,0).  The stage combinations and the
// update run on 10 slots + 2 r instead of 18 values, the RHS on one sincos and two rows instead of
// two and three.  tube 0's twist runs on both lanes, rounded in different orders (the lanes are
// rounding-level apart from each other and from fk_lane_rk4's one-lane arithmetic).
// ------------------------------------------------------------------------------------------
// quad_perm DPP on a 64-bit value: lane i of each quad reads lane P[i] (one v_mov_dpp per dword)
template <int CTRL>
__device__ __forceinline__ double dpp_qp(double x)
{
    const long long v = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_mov_dpp((int)(v & 0xffffffffll), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp((int)(v >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int DPP_FROM_ODD = 0xF5;     // quad_perm [1, 1, 3, 3]: both lanes of a pair read the odd one
constexpr int DPP_FROM_EVEN = 0xA0;    // quad_perm [0, 0, 2, 2]
constexpr int DPP_SWAP = 0xB1;         // quad_perm [1, 0, 3, 2]

// ctr_math::sincos_tab of one angle in two halves (the same operations, so the same bits): the
// reduction and the table loads (pair_trig_pre), issued a stage ahead of the polynomial work that
// consumes them (pair_trig_post), so the LDS latency of stage k + 1's table read runs under stage
// k's RHS.  The stage-(k + 1) angle exists that early: alpha' is the masked u_z of the stage input,
// whose value is formed before the stage's RHS.
struct PairTrig {
    double x, r, ts, tc;
};

__device__ __forceinline__ PairTrig pair_trig_pre(double x)
{
    PairTrig p;
    p.x = x;
    const double n = rint(x * 81.48733086305042);          // sincos_tab2_pre, angle 0
    const int k = ((int)n) & 511;
    p.ts = s_trig_tab[k][0];
    p.tc = s_trig_tab[k][1];
    p.r = fma(-n, 4.783776559169348e-19, fma(-n, 0.01227184630308513, x));
    return p;
}

template <bool CAREFUL>
__device__ __forceinline__ void pair_trig_post(const PairTrig &p, double &s, double &c)
{
    const double r = p.r, z = r * r;                        // sincos_tab2_post, angle 0
    const double sp = fma(z, 8.3333333333333332e-03, -1.6666666666666666e-01);
    const double cp = fma(z, 4.1666666666666664e-02, -0.5);
    const double sr = fma(r * z, sp, r), cr = fma(z, cp, 1.0);
    s = fma(p.ts, cr, p.tc * sr);
    c = fma(p.tc, cr, -(p.ts * sr));
    if (CAREFUL && __builtin_expect(__ballot(ctr_math::sincos_needs_slow(p.x)) != 0, 0) &&
        ctr_math::sincos_needs_slow(p.x)) {
        const ctr_math::SinCos q = ctr_math::sincos_slow(p.x);
        s = q.s;
        c = q.c;
    }
}

// The angle each lane evaluates at level LV from the stage input's alpha slots: alpha_a - alpha_0
// (level 3), or the even lane's alpha_1 - alpha_0 (level 2: the odd lane's tube a is tube 2)
template <int LV>
__device__ __forceinline__ double pair_angle(const double V[2])
{
    if constexpr (LV == 3) return V[1] - V[0];
    else return dpp_qp<DPP_FROM_EVEN>(V[1] - V[0]);
}

// A segment's RHS constants in the lane's tube order (SegPar, seg_fold_inv'ed: wx = inv EI Ux),
// and the alpha' presence masks of the twist slots 0 (tube 0) and 1 (tube a) (stage_at): alpha' =
// u_z of a present tube, 0 otherwise.  alpha' is never formed: the masks scale the step
// coefficients of the alpha slots instead (alpha_in = fma(u_z,in, C m, alpha), the update h/6 m),
// the same values for m = 1 and alpha kept for m = 0, at no cost per RHS.
constexpr int PAIR_NT = 2;          // twist slots per lane: tube 0, tube a
struct PairPar {
    double wx0, wx1, wxa, wxb, g0, ga;
    double ch2[PAIR_NT], ch[PAIR_NT], ch6[PAIR_NT];   // h/2 m, h m, h/6 m of the alpha slots (the gap's h)
};

__device__ __forceinline__ PairPar pair_par(const SegPar &p, bool odd, double h)
{
    PairPar q;
    q.wx0 = p.wx[0];
    q.wx1 = p.wx[1];
    q.wxa = odd ? p.wx[2] : p.wx[1];
    q.wxb = odd ? p.wx[1] : p.wx[2];
    q.g0 = p.g[0];
    q.ga = odd ? p.g[2] : p.g[1];
    const bool m[PAIR_NT] = {(p.present & 1u) != 0u, ((p.present >> (odd ? 2 : 1)) & 1u) != 0u};
    const double h2 = 0.5 * h, h6 = h * (1.0 / 6.0);   // rk4_step_pair's coefficients
    #pragma unroll
    for (int j = 0; j < PAIR_NT; ++j) {
        q.ch2[j] = m[j] ? h2 : 0.0;
        q.ch[j] = m[j] ? h : 0.0;
        q.ch6[j] = m[j] ? h6 : 0.0;
    }
    return q;
}

// The pair's derivative at stage input (A, B, U, V): dA, dB (rows of R [u]x) and dU (du_z of tube 0
// and tube a); r' = (A[2], B[2]) and alpha' (U masked, PairPar) are the caller's.
// Level 2 (tube 2 absent): sin/cos(alpha_1 - alpha_0) only, formed from the even lane's difference
// (the odd lane's tube a is tube 2, constant at this level: g_a = 0).
template <int LV, bool CAREFUL>
__device__ __forceinline__ void rhs_pair(const PairPar &p, const PairTrig &tg, const double A[3], const double B[3],
                                         const double U[PAIR_NT], double dA[3], double dB[3], double dU[PAIR_NT])
{
    double a, b;
    if constexpr (LV == 3) {
        double sa, ca;                                 // alpha_a - alpha_0
        pair_trig_post<CAREFUL>(tg, sa, ca);
        const double sb = dpp_qp<DPP_SWAP>(sa), cb = dpp_qp<DPP_SWAP>(ca);   // alpha_b - alpha_0
        const double sab = sa * cb - ca * sb;          // sin(alpha_a - alpha_b)
        const double sy1 = fma(p.wxb, sb, p.wxa * sa); // u_y,0 (wx_1 s10 + wx_2 s20)
        dU[0] = -(p.g0 * sy1);
        dU[1] = p.ga * fma(p.wxb, sab, p.wx0 * sa);
        a = fma(p.wxb, cb, fma(p.wxa, ca, p.wx0));
        b = sy1;
    } else {
        double s1, c1;                                 // alpha_1 - alpha_0 (the even lane's)
        pair_trig_post<CAREFUL>(tg, s1, c1);
        const double sy1 = p.wx1 * s1;                 // rhs_core_lv<2>
        const double sy2 = -(p.wx0 * s1);
        dU[0] = -(p.g0 * sy1);
        dU[1] = -(p.ga * sy2);                          // tube 1 on the even lane, tube 2 (g = 0) on the odd
        a = fma(p.wx1, c1, p.wx0);
        b = sy1;
    }
    const double u0 = U[0];
    #pragma unroll
    for (int r = 0; r < 2; ++r) {
        const double *X = r ? B : A;
        double *dX = r ? dB : dA;
        const double r0 = X[0], r1 = X[1], r2 = X[2];
        dX[0] = r1 * u0 - r2 * b;
        dX[1] = r2 * a - r0 * u0;
        dX[2] = r0 * b - r1 * a;
    }
}

// One classical RK4 step of the pair (rk4_step's combinations; a tube's zero derivatives keep its
// slots exactly, so level 2 runs every slot).
template <int LV, bool CAREFUL>
__device__ __forceinline__ void rk4_step_pair(const PairPar &p, double h, double A[3], double B[3], double U[PAIR_NT],
                                              double V[PAIR_NT], double &rA, double &rB)
{
    // kU: the stage derivatives of u_z; uU: the stage inputs of u_z (alpha' = m u_z,in)
    double kA[4][3], kB[4][3], kU[4][PAIR_NT], uU[4][PAIR_NT], qA[4], qB[4];
    double iA[3], iB[3], iV[PAIR_NT];
    const double h2 = 0.5 * h, h6 = h * (1.0 / 6.0);
    const double *ch2 = p.ch2, *ch = p.ch, *ch6 = p.ch6;   // the alpha slots' coefficients, masked
    // stage 0's table read, and stage 1's (its alpha input is fma(u_z, h/2 m, alpha)) behind it
    #pragma unroll
    for (int i = 0; i < PAIR_NT; ++i) uU[0][i] = U[i];
    PairTrig tg = pair_trig_pre(pair_angle<LV>(V));
    #pragma unroll
    for (int i = 0; i < PAIR_NT; ++i) iV[i] = fma(uU[0][i], ch2[i], V[i]);
    PairTrig tn = pair_trig_pre(pair_angle<LV>(iV));
    rhs_pair<LV, CAREFUL>(p, tg, A, B, U, kA[0], kB[0], kU[0]);
    qA[0] = A[2];
    qB[0] = B[2];
    #pragma unroll
    for (int st = 1; st < 4; ++st) {
        const double C = st < 3 ? h2 : h;
        tg = tn;
        #pragma unroll
        for (int i = 0; i < PAIR_NT; ++i) uU[st][i] = fma(kU[st - 1][i], C, U[i]);
        if (st < 3) {                                  // the next stage's angle and table read
            #pragma unroll
            for (int i = 0; i < PAIR_NT; ++i) iV[i] = fma(uU[st][i], st < 2 ? ch2[i] : ch[i], V[i]);
            tn = pair_trig_pre(pair_angle<LV>(iV));
        }
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            iA[i] = fma(kA[st - 1][i], C, A[i]);
            iB[i] = fma(kB[st - 1][i], C, B[i]);
        }
        rhs_pair<LV, CAREFUL>(p, tg, iA, iB, uU[st], kA[st], kB[st], kU[st]);
        qA[st] = iA[2];
        qB[st] = iB[2];
    }
    #pragma unroll
    for (int i = 0; i < PAIR_NT; ++i) {
        V[i] = fma(ch6[i], uU[0][i] + 2.0 * (uU[1][i] + uU[2][i]) + uU[3][i], V[i]);
        U[i] = fma(h6, kU[0][i] + 2.0 * (kU[1][i] + kU[2][i]) + kU[3][i], U[i]);
    }
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        A[i] = fma(h6, kA[0][i] + 2.0 * (kA[1][i] + kA[2][i]) + kA[3][i], A[i]);
        B[i] = fma(h6, kB[0][i] + 2.0 * (kB[1][i] + kB[2][i]) + kB[3][i], B[i]);
    }
    rA = fma(h6, qA[0] + 2.0 * (qA[1] + qA[2]) + qA[3], rA);
    rB = fma(h6, qB[0] + 2.0 * (qB[1] + qB[2]) + qB[3], rB);
}

// fk_lane_rk4<false, false, CAREFUL> on a lane pair (see above).  Both lanes of every pair of the
// wave must call it (in lock-step: the pair shares its segmentation and plan, one LDS column per
// pair); the tip and the counters are returned on both lanes.
template <bool CAREFUL>
__device__ void fk_pair_rk4(const SysK &sy, const double q[6], bool odd, double tip[3], FkStats &st, double steps_per_m)
{
    const double beta[3] = {q[0], q[1], q[2]};
    const int col = (int)(threadIdx.x >> 1);
    double *end_lds = &s_seg_end[0][col];
    int *n_lds = &s_seg_n[0][col];
    const Seg sg = seg_build<CTR_BLOCK, 1>(sy, beta, end_lds);
    const Rk4Plan pl = rk4_plan<true, false>(sg, end_lds, n_lds, steps_per_m);
    st.nseg += (uint32_t)__builtin_popcount(sg.kept);
    double s0, c0;
    sincos_lds(q[3], s0, c0);
    // R0 = Rz(alpha_0): rows (c0, -s0, 0), (s0, c0, 0), (0, 0, 1)
    double A[3], B[3], U[PAIR_NT], V[PAIR_NT];
    A[0] = odd ? 0.0 : c0;  A[1] = odd ? 0.0 : -s0;  A[2] = odd ? 1.0 : 0.0;
    B[0] = odd ? 0.0 : s0;  B[1] = odd ? 0.0 : c0;   B[2] = 0.0;
    U[0] = U[1] = 0.0;
    V[0] = q[3];
    V[1] = odd ? q[5] : q[4];             // tube a
    double rA = 0.0, rB = 0.0;
    PairPar p;
    double h = 0.0;
    int left = 0;
    bool lv3 = true;
    uint32_t rem = pl.step;
    for (;;) {
        if (left == 0) {
            if (rem == 0u) break;
            const int k = __builtin_ctz(rem);
            rem &= rem - 1u;
            const SegPar sp = seg_par_at<false, false>(sy, seg_bits(sg, k));
            h = end_lds[k * CTR_BLOCK];
            p = pair_par(sp, odd, h);
            left = n_lds[k * CTR_BLOCK];
            lv3 = (sp.present & 4u) != 0u || sp.present == 0u;
        }
        if (__ballot(lv3) == 0) rk4_step_pair<2, CAREFUL>(p, h, A, B, U, V, rA, rB);
        else rk4_step_pair<3, CAREFUL>(p, h, A, B, U, V, rA, rB);
        st.nfev += 4;
        st.nstep++;
        --left;
    }
    // the tube-0-alone tail as segment maps (fk_lane_rk4): u = (u_x,0, 0, u_z,0), u_z,0 from the odd lane
    const Trig tc = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    const double uzt[3] = {U[0], 0.0, 0.0};
    uint32_t tail = pl.tail;
    while (__ballot(tail != 0u) != 0) {
        if (tail != 0u) {
            const int k = __builtin_ctz(tail);
            tail &= tail - 1u;
            const SegPar pt = seg_par_at<false, false>(sy, seg_bits(sg, k));
            const int n = n_lds[k * CTR_BLOCK];
            double aq[9], am[3];
            const int ncomp = rigid_segment_map<false>(pt, tc, uzt, end_lds[k * CTR_BLOCK], n, aq, am);
            #pragma unroll
            for (int r = 0; r < 2; ++r) {
                double *X = r ? B : A;
                double &rr = r ? rB : rA;
                double nX[3];
                #pragma unroll
                for (int c = 0; c < 3; ++c) nX[c] = fma(X[2], aq[6 + c], fma(X[1], aq[3 + c], X[0] * aq[c]));
                rr = fma(X[2], am[2], fma(X[1], am[1], fma(X[0], am[0], rr)));
                #pragma unroll
                for (int c = 0; c < 3; ++c) X[c] = nX[c];
            }
            st.nfev += 4u * (uint32_t)n;
            st.nrej += (1u << 16) + (uint32_t)ncomp;
        }
    }
    double r3[3] = {dpp_qp<DPP_FROM_EVEN>(rA), dpp_qp<DPP_FROM_EVEN>(rB), dpp_qp<DPP_FROM_ODD>(rA)};
    if (pl.too_long) {
        r3[0] = r3[1] = r3[2] = NAN;
        st.status |= CTR_STATUS_TOO_LONG | CTR_STATUS_NAN;
    }
    tip[0] = r3[0]; tip[1] = r3[1]; tip[2] = r3[2];
    if (isnan(tip[0]) || isnan(tip[1]) || isnan(tip[2])) st.status |= CTR_STATUS_NAN;
}

// ------------------------------------------------------------------------------------------
// scipy RK45 of the compliant model (no y pre-curvature) on a lane PAIR: fk_lane<false, false,
// false, CAREFUL> in fk_pair_rk4's slots (A, B, U, V, rA, rB).  The controller (t, h, accept /
// reject, the segment cursor) runs on both lanes with the same values: every norm is the sum of
// the two lanes' partial sums, exchanged with one DPP swap (a + b == b + a exactly), so the pair
// takes every branch together.  As in fk_lane, u_z of an absent tube a is parked (uzf) and tube
// 0's alpha' is masked by its presence m0.  The FSAL derivative f is (fA, fB, fU); its alpha' and
// r' are implied by y.  Each stage's table read is issued a stage early (rk4_step_pair).
// An A/B experiment (CTR_RK45_PAIR, off in the product build): the step-path parity tests pass on
// it, but k_step takes 92.5-95.5 us against 72.3 us one env per lane -- 1.41x the VALU
// instructions at a 7 % better issue rate ("RK45 on lane pairs").
// ------------------------------------------------------------------------------------------
namespace rk {
constexpr double RKA[6][5] = {{0, 0, 0, 0, 0},
                              {A10, 0, 0, 0, 0},
                              {A20, A21, 0, 0, 0},
                              {A30, A31, A32, 0, 0},
                              {A40, A41, A42, A43, 0},
                              {A50, A51, A52, A53, A54}};
constexpr double RKB[6] = {B0, 0.0, B2, B3, B4, B5};
constexpr double RKE[6] = {E0, 0.0, E2, E3, E4, E5};
}  // namespace rk

// One attempt of RungeKutta._step_impl (rk.py:111-175) on the pair at tube level LV (3, or 2:
// no lane of the wave has tube 2); fk_lane's attempt in the pair's slots.
template <int LV, bool CAREFUL>
__device__ __forceinline__ void rk45_attempt_pair(const PairPar &p, bool m0, bool odd, double A[3], double B[3],
                                                  double U[PAIR_NT], double V[PAIR_NT], double &rA, double &rB,
                                                  double fA[3], double fB[3], double fU[PAIR_NT], double &t, double tb,
                                                  double &ha, double h, double tnew, bool &rejected, bool &new_step,
                                                  bool &need_init, FkStats &st)
{
    using namespace rk;
    // The stages are h-scaled (K_j = h f_j): rhs_pair at wx h and u_z,0 h gives h dA, h dB, h dU
    // directly, so every combination's coefficient is a tableau constant (no per-lane a_sj h).
    // Each K_j enters y_new (5th order) and the error sum as soon as it exists (fma chains from
    // stage 0 up, fk_lane's order), so a stage is dead after its last stage input.
    PairPar ph = p;
    ph.wx0 = p.wx0 * h; ph.wx1 = p.wx1 * h; ph.wxa = p.wxa * h; ph.wxb = p.wxb * h;
    double kA[3][5], kB[3][5], kU[PAIR_NT][5], al[PAIR_NT][5];   // al: h alpha' = h (masked u_z of the stage input)
    double nA[3], nB[3], nU[PAIR_NT], nV[PAIR_NT];
    double eA[3], eB[3], eU[PAIR_NT], eV[PAIR_NT];
    al[0][0] = m0 ? U[0] * h : 0.0;
    al[1][0] = U[1] * h;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        kA[i][0] = fA[i] * h; kB[i][0] = fB[i] * h;
        nA[i] = fma(kA[i][0], B0, A[i]); nB[i] = fma(kB[i][0], B0, B[i]);
        eA[i] = kA[i][0] * E0; eB[i] = kB[i][0] * E0;
    }
    #pragma unroll
    for (int i = 0; i < PAIR_NT; ++i) {
        kU[i][0] = fU[i] * h;
        nU[i] = fma(kU[i][0], B0, U[i]); eU[i] = kU[i][0] * E0;
        nV[i] = fma(al[i][0], B0, V[i]); eV[i] = al[i][0] * E0;
    }
    double br[2] = {A[2] * B0, B[2] * B0}, er[2] = {A[2] * E0, B[2] * E0};
    double iA[3], iB[3], iU[PAIR_NT], iV[PAIR_NT];
    #pragma unroll
    for (int i = 0; i < PAIR_NT; ++i) iV[i] = fma(al[i][0], A10, V[i]);
    PairTrig tg = pair_trig_pre(pair_angle<LV>(iV)), tn;
    #pragma unroll
    for (int s = 1; s < 6; ++s) {
        // stage s input: u_z first (alpha'_s), then the next angle's table read, then the rows
        #pragma unroll
        for (int i = 0; i < PAIR_NT; ++i) {
            double u = U[i];
            #pragma unroll
            for (int j = 0; j < s; ++j) u = fma(kU[i][j], RKA[s][j], u);
            iU[i] = u;
        }
        const double u0h = iU[0] * h;
        const double als[PAIR_NT] = {m0 ? u0h : 0.0, iU[1] * h};
        if (s < 5) {
            al[0][s] = als[0];
            al[1][s] = als[1];
            #pragma unroll
            for (int i = 0; i < PAIR_NT; ++i) {
                double v = V[i];
                #pragma unroll
                for (int j = 0; j <= s; ++j) v = fma(al[i][j], RKA[s + 1][j], v);
                iV[i] = v;
            }
            tn = pair_trig_pre(pair_angle<LV>(iV));
        }
        if (s > 1) {
            #pragma unroll
            for (int i = 0; i < PAIR_NT; ++i) { nV[i] = fma(als[i], RKB[s], nV[i]); eV[i] = fma(als[i], RKE[s], eV[i]); }
        }
        if (s == 5) tn = pair_trig_pre(pair_angle<LV>(nV));
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            double a = A[i], b = B[i];
            #pragma unroll
            for (int j = 0; j < s; ++j) { a = fma(kA[i][j], RKA[s][j], a); b = fma(kB[i][j], RKA[s][j], b); }
            iA[i] = a;
            iB[i] = b;
        }
        double dA[3], dB[3], dU[PAIR_NT];
        const double uh[PAIR_NT] = {u0h, 0.0};
        rhs_pair<LV, CAREFUL>(ph, tg, iA, iB, uh, dA, dB, dU);
        if (s < 5) {
            #pragma unroll
            for (int i = 0; i < 3; ++i) { kA[i][s] = dA[i]; kB[i][s] = dB[i]; }
            #pragma unroll
            for (int i = 0; i < PAIR_NT; ++i) kU[i][s] = dU[i];
        }
        if (s > 1) {
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                nA[i] = fma(dA[i], RKB[s], nA[i]); nB[i] = fma(dB[i], RKB[s], nB[i]);
                eA[i] = fma(dA[i], RKE[s], eA[i]); eB[i] = fma(dB[i], RKE[s], eB[i]);
            }
            #pragma unroll
            for (int i = 0; i < PAIR_NT; ++i) { nU[i] = fma(dU[i], RKB[s], nU[i]); eU[i] = fma(dU[i], RKE[s], eU[i]); }
            br[0] += iA[2] * RKB[s]; br[1] += iB[2] * RKB[s];
            er[0] += iA[2] * RKE[s]; er[1] += iB[2] * RKE[s];
        }
        tg = tn;
    }
    double nr[2];
    nr[0] = rA + h * br[0];
    nr[1] = rB + h * br[1];
    double k6A[3], k6B[3], k6U[PAIR_NT];       // f at y_new (unscaled: the next attempt's f)
    rhs_pair<LV, CAREFUL>(p, tg, nA, nB, nU, k6A, k6B, k6U);
    st.nfev += 6;
    // error norm: this lane's slots (tube 0's twist counted on the even lane only), then the pair's sum
    const double e6h = E6 * h;
    auto term = [&](double k6, double e, double y, double yn) {
        const double x = fma(k6, e6h, e) * ctr_math::rcp_est(fma(ctr_math::absmax(y, yn), RTOL, ATOL));
        return x * x;
    };
    double acc[3] = {0.0, 0.0, 0.0};
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        acc[0] += term(k6A[i], eA[i], A[i], nA[i]);
        acc[1] += term(k6B[i], eB[i], B[i], nB[i]);
    }
    acc[2] += term(nA[2], er[0] * h, rA, nr[0]);
    acc[2] += term(nB[2], er[1] * h, rB, nr[1]);
    {
        const double tu0 = term(k6U[0], eU[0], U[0], nU[0]);
        const double tv0 = term(m0 ? nU[0] : 0.0, eV[0], V[0], nV[0]);
        acc[0] += odd ? 0.0 : tu0;
        acc[1] += odd ? 0.0 : tv0;
        acc[2] += term(k6U[1], eU[1], U[1], nU[1]);
        acc[2] += term(nU[1], eV[1], V[1], nV[1]);
    }
    const double own = (acc[0] + acc[1]) + acc[2];
    const double en2 = own + dpp_qp<DPP_SWAP>(own);   // = 18 error_norm^2
    const double en2n = en2 * (1.0 / 18);
    const double fpow = 0.9 * ctr_math::inv_root10(en2n);
    const bool ok = en2n < 1.0;
    double factor = (en2n == 0.0) ? 10.0 : fmin(10.0, fpow);
    if (rejected) factor = fmin(1.0, factor);
    ha *= ok ? factor : fmax(0.2, fpow);
    if (__builtin_expect(__ballot(!ok) != 0, 0)) {
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            nA[i] = ok ? nA[i] : A[i];
            nB[i] = ok ? nB[i] : B[i];
            k6A[i] = ok ? k6A[i] : fA[i];
            k6B[i] = ok ? k6B[i] : fB[i];
        }
        #pragma unroll
        for (int i = 0; i < PAIR_NT; ++i) {
            nU[i] = ok ? nU[i] : U[i];
            nV[i] = ok ? nV[i] : V[i];
            k6U[i] = ok ? k6U[i] : fU[i];
        }
        nr[0] = ok ? nr[0] : rA;
        nr[1] = ok ? nr[1] : rB;
        tnew = ok ? tnew : t;
    }
    #pragma unroll
    for (int i = 0; i < 3; ++i) { A[i] = nA[i]; B[i] = nB[i]; fA[i] = k6A[i]; fB[i] = k6B[i]; }
    #pragma unroll
    for (int i = 0; i < PAIR_NT; ++i) { U[i] = nU[i]; V[i] = nV[i]; fU[i] = k6U[i]; }
    rA = nr[0];
    rB = nr[1];
    t = tnew;
    st.nstep += ok ? 1u : 0u;
    st.nrej += ok ? 0u : 1u;
    new_step = ok;
    rejected = ok ? rejected : true;
    if (ok && t - tb >= 0.0) need_init = true;
}

// fk_lane<false, false, false, CAREFUL> on a lane pair (see above).  Both lanes of every pair of
// the wave call it; the tip and the counters are returned on both lanes.
template <bool CAREFUL>
__device__ void fk_pair_rk45(const SysK &sy, const double q[6], bool odd, double tip[3], FkStats &st)
{
    using namespace rk;
    const double beta[3] = {q[0], q[1], q[2]};
    const int col = (int)(threadIdx.x >> 1);
    double *end_lds = &s_seg_end[0][col];
    const Seg sg = seg_build<CTR_BLOCK, 1>(sy, beta, end_lds);
    double A[3], B[3], U[PAIR_NT], V[PAIR_NT];
    {
        double s0, c0;
        ctr_math::sincos_cw(q[3], &s0, &c0);                  // R0 = Rz(alpha_0), as fk_lane
        A[0] = odd ? 0.0 : c0;  A[1] = odd ? 0.0 : -s0;  A[2] = odd ? 1.0 : 0.0;
        B[0] = odd ? 0.0 : s0;  B[1] = odd ? 0.0 : c0;   B[2] = 0.0;
    }
    U[0] = U[1] = 0.0;
    V[0] = q[3];
    V[1] = odd ? q[5] : q[4];             // tube a
    double rA = 0.0, rB = 0.0, uzf = 0.0;
    double fA[3], fB[3], fU[PAIR_NT];
    PairPar p;
    bool m0 = true, lv3 = true;
    double t = 0.0, tb = 0.0, ha = 0.0, min_step = 0.0, prev_end = 0.0;
    uint32_t remaining = sg.kept;
    bool need_init = true, new_step = true, rejected = false;
    for (;;) {
        if (need_init) {
            if (remaining == 0u) break;
            const int k = __builtin_ctz(remaining);
            remaining &= remaining - 1u;
            const SegPar sp = seg_par_at<false, false>(sy, seg_bits(sg, k));
            p = pair_par(sp, odd, 0.0);
            m0 = (sp.present & 1u) != 0u;
            const bool ma = ((sp.present >> (odd ? 2 : 1)) & 1u) != 0u;
            uzf = (!ma && U[1] != 0.0) ? U[1] : uzf;
            U[1] = ma ? U[1] : 0.0;
            lv3 = (sp.present & 4u) != 0u;
            const double endk = end_lds[k * CTR_BLOCK];
            const double a = prev_end, b = endk - 1e-6;          // model.py:141 linspace endpoints
            const double t0 = fmin(a, b);
            tb = fmax(a, b);
            prev_end = endk;
            // f = fun(t0, y0) (the level-3 form: the same values at every level)
            rhs_pair<3, CAREFUL>(p, pair_trig_pre(pair_angle<3>(V)), A, B, U, fA, fB, fU);
            st.nfev++;
            st.nseg++;
            const double interval = tb - t0;
            if (interval == 0.0) continue;
            if (sp.present == 0u) {                              // a gap with no tube (fk_lane)
                rA = rB = NAN;
                st.status |= CTR_STATUS_NAN;
                break;
            }
            // select_initial_step (common.py:68-140) on the pair's slots
            const double fV[PAIR_NT] = {m0 ? U[0] : 0.0, U[1]};
            const double yur1 = ma ? U[1] : uzf;                 // the reference's u_z of tube a
            double iscA[3], iscB[3], iscU[PAIR_NT], iscV[PAIR_NT], iscr[2];
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                iscA[i] = ctr_math::rcp_est(ATOL + fabs(A[i]) * RTOL);
                iscB[i] = ctr_math::rcp_est(ATOL + fabs(B[i]) * RTOL);
            }
            iscU[0] = ctr_math::rcp_est(ATOL + fabs(U[0]) * RTOL);
            iscU[1] = ctr_math::rcp_est(ATOL + fabs(yur1) * RTOL);
            #pragma unroll
            for (int i = 0; i < PAIR_NT; ++i) iscV[i] = ctr_math::rcp_est(ATOL + fabs(V[i]) * RTOL);
            iscr[0] = ctr_math::rcp_est(ATOL + fabs(rA) * RTOL);
            iscr[1] = ctr_math::rcp_est(ATOL + fabs(rB) * RTOL);
            auto sq = [](double x) { return x * x; };
            double s0 = 0.0, s1 = 0.0;
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                s0 += sq(A[i] * iscA[i]) + sq(B[i] * iscB[i]);
                s1 += sq(fA[i] * iscA[i]) + sq(fB[i] * iscB[i]);
            }
            s0 += sq(rA * iscr[0]) + sq(rB * iscr[1]) + sq(yur1 * iscU[1]) + sq(V[1] * iscV[1]);
            s1 += sq(A[2] * iscr[0]) + sq(B[2] * iscr[1]) + sq(fU[1] * iscU[1]) + sq(fV[1] * iscV[1]);
            s0 += odd ? 0.0 : sq(U[0] * iscU[0]) + sq(V[0] * iscV[0]);
            s1 += odd ? 0.0 : sq(fU[0] * iscU[0]) + sq(fV[0] * iscV[0]);
            s0 += dpp_qp<DPP_SWAP>(s0);
            s1 += dpp_qp<DPP_SWAP>(s1);
            const double d0sq = s0 * (1.0 / 18), d1sq = s1 * (1.0 / 18);
            const double h0n = 0.01 * ctr_math::sqrt_rsq(s0 * ctr_math::rcp1(s1));
            double h0 = (d0sq < 1e-10 || d1sq < 1e-10) ? 1e-6 : h0n;
            h0 = fmin(h0, interval);
            double A1[3], B1[3], U1[PAIR_NT], V1[PAIR_NT];
            #pragma unroll
            for (int i = 0; i < 3; ++i) { A1[i] = A[i] + h0 * fA[i]; B1[i] = B[i] + h0 * fB[i]; }
            #pragma unroll
            for (int i = 0; i < PAIR_NT; ++i) { U1[i] = U[i] + h0 * fU[i]; V1[i] = V[i] + h0 * fV[i]; }
            double gA[3], gB[3], gU[PAIR_NT];
            rhs_pair<3, CAREFUL>(p, pair_trig_pre(pair_angle<3>(V1)), A1, B1, U1, gA, gB, gU);
            st.nfev++;
            const double gV[PAIR_NT] = {m0 ? U1[0] : 0.0, U1[1]};
            double s2 = 0.0;
            #pragma unroll
            for (int i = 0; i < 3; ++i) s2 += sq((gA[i] - fA[i]) * iscA[i]) + sq((gB[i] - fB[i]) * iscB[i]);
            s2 += sq((A1[2] - A[2]) * iscr[0]) + sq((B1[2] - B[2]) * iscr[1]) + sq((gU[1] - fU[1]) * iscU[1]) +
                  sq((gV[1] - fV[1]) * iscV[1]);
            s2 += odd ? 0.0 : sq((gU[0] - fU[0]) * iscU[0]) + sq((gV[0] - fV[0]) * iscV[0]);
            s2 += dpp_qp<DPP_SWAP>(s2);
            const double ih0 = ctr_math::rcp1(h0);
            const double d2sq = s2 * (1.0 / 18) * ih0 * ih0;
            const double h1a = fmax(1e-6, h0 * 1e-3);
            const double h1b = 0.3981071705534972 * ctr_math::inv_root10(fmax(d1sq, d2sq));
            const double h1 = (d1sq <= 1e-30 && d2sq <= 1e-30) ? h1a : h1b;
            ha = fmin(fmin(100.0 * h0, h1), interval);
            t = t0;
            need_init = false;
            new_step = true;
        }
        {
            const double ms = 10.0 * ctr_math::gap_up(t);
            min_step = new_step ? ms : min_step;
            ha = (new_step && ha < ms) ? ms : ha;
            rejected = new_step ? false : rejected;
            new_step = false;
        }
        if (!(ha >= min_step)) {
            if (ha < min_step) {
                st.status |= CTR_STATUS_STEP_UNDERFLOW;
            } else {
                rA = rB = NAN;
                st.status |= CTR_STATUS_NAN;
            }
            break;
        }
        double tnew = t + ha;
        if (tnew - tb > 0.0) tnew = tb;
        const double h = tnew - t;
        ha = fabs(h);
        if (__ballot(lv3) == 0)
            rk45_attempt_pair<2, CAREFUL>(p, m0, odd, A, B, U, V, rA, rB, fA, fB, fU, t, tb, ha, h, tnew, rejected,
                                          new_step, need_init, st);
        else
            rk45_attempt_pair<3, CAREFUL>(p, m0, odd, A, B, U, V, rA, rB, fA, fB, fU, t, tb, ha, h, tnew, rejected,
                                          new_step, need_init, st);
    }
    tip[0] = dpp_qp<DPP_FROM_EVEN>(rA);
    tip[1] = dpp_qp<DPP_FROM_EVEN>(rB);
    tip[2] = dpp_qp<DPP_FROM_ODD>(rA);
    if (isnan(tip[0]) || isnan(tip[1]) || isnan(tip[2])) st.status |= CTR_STATUS_NAN;
}

// ------------------------------------------------------------------------------------------
// Env logic
// ------------------------------------------------------------------------------------------
// obs.py:166-183 in float32 with numpy-2 scalar rules (python float -> float32).
__device__ __forceinline__ void set_action_lane(const ctr_system_t &sy, bool constrain_alpha, float q[6],
                                                const float a[6])
{
#pragma clang fp contract(off)
    #pragma unroll
    for (int i = 0; i < 6; ++i) {
        float lo, hi;
        if (i < 3) { lo = (float)(-sy.L[i] + 1e-3); hi = 0.0f; }   // obs.py:75-76 Box(float32)
        else if (constrain_alpha) { lo = -3.14159274101257324f; hi = 3.14159274101257324f; }
        else { lo = -INFINITY; hi = INFINITY; }
        float v = q[i] + a[i];
        if (i < 3 || constrain_alpha) {   // the +-inf bounds clamp nothing (NaN included)
            v = v < lo ? lo : v;
            v = v > hi ? hi : v;
        }
        q[i] = v;
    }
    #pragma unroll
    for (int i = 1; i < 3; ++i) {
        const float x = q[i - 1], yv = q[i];
        const float m = (yv < x) ? yv : x;                       // min(b[i-1], b[i])
        const float d = (float)(sy.L[i] - sy.L[i - 1]);
        const float z = d + yv;
        q[i - 1] = (z > m) ? z : m;                              // max(., L_i - L_{i-1} + b[i])
    }
}

// The step's n_substeps set_action passes (ctr_reach_env.py:133-135).  The constrain_alpha test is
// taken once, outside the loop, so the unconstrained case runs without the angle clamps.
__device__ __forceinline__ void set_action_substeps(const ctr_system_t &sy, bool constrain_alpha, int n, float q[6],
                                                    const float a[6])
{
    if (constrain_alpha)
        for (int k = 0; k < n; ++k) set_action_lane(sy, true, q, a);
    else
        for (int k = 0; k < n; ++k) set_action_lane(sy, false, q, a);
}

// obs.py:136-164.  Writes obs_dim (13 or 14) values in float64, the reference's dtype; the env
// stores them as float32 (rounded once) or float64 (ctr_env_config_t.obs_f64).  Needs the
// workgroup's trig table (trig_table_fill, done by stage_systems).
__device__ __forceinline__ void obs_lane(const float q[6], const double dg[3], const double ag[3], double tol,
                                         int sys, bool multi, bool egocentric, double *out)
{
    double b[3], a[3], s[3], c[3];
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        b[i] = (double)q[i];
        a[i] = (double)q[3 + i];
        if (egocentric && i > 0) { b[i] -= (double)q[i - 1]; a[i] -= (double)q[3 + i - 1]; }
    }
    // the workgroup's LDS sincos table (<= 2 ulp, tests/test_math.py, like sincos_cw); angles
    // beyond its |x| < 2^20 range (never reached by bounded episodes) take the exact path
    ctr_math::sincos_tab2(a[0], a[1], s_trig_tab, s[0], c[0], s[1], c[1]);
    ctr_math::sincos_tab(a[2], s_trig_tab, s[2], c[2]);
    if (__builtin_expect(__ballot(ctr_math::sincos_needs_slow(a[0]) || ctr_math::sincos_needs_slow(a[1]) ||
                                  ctr_math::sincos_needs_slow(a[2])) != 0, 0)) {
        #pragma unroll
        for (int i = 0; i < 3; ++i)
            if (ctr_math::sincos_needs_slow(a[i])) {
                const ctr_math::SinCos r = ctr_math::sincos_slow(a[i]);
                s[i] = r.s;
                c[i] = r.c;
            }
    }
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        out[3 * i + 0] = c[i];
        out[3 * i + 1] = s[i];
        out[3 * i + 2] = b[i];
    }
    #pragma unroll
    for (int k = 0; k < 3; ++k) out[9 + k] = dg[k] - ag[k];
    out[12] = tol;
    out[13] = multi ? (double)sys : 0.0;
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 counter RNG and the sample_goal rejection sampler.
// counter = {draw, epoch, env_lo, env_hi ^ (stream << 24)}, key = seed.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1)
{
    // each 32 x 32 -> 64-bit product as one v_mad_u64_u32 (the lo and hi halves from one
    // instruction instead of a v_mul_lo_u32 / v_mul_hi_u32 pair: 20 % faster per Philox block on
    // gfx950, tools/ubench/philox_mul.hip; the same bits)
    #pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b)
{
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// obs.py:185-207 (sample_goal's rejection sampler) with the build's Philox stream.  A candidate is
// six uniforms from three Philox blocks 3c, 3c + 1, 3c + 2 (u0, u1 | u2, u3 | u4, u5); the
// extensions (u0..u2) decide acceptance, so the third block (the last two angles) is generated
// for the returned candidate only.  Returns the number of candidates drawn (> 1000: the
// reference's "stuck" case) and sets q.  The wave's lanes help each other (every lane of the wave
// calls it; `need` marks the lanes that sample).  Lane L's answer is the first accepted candidate of ITS
// sequence (candidates are keyed by L's env, reset number and stream), so any lane can evaluate
// any lane's candidate c.  Each round, every lane evaluates one candidate of one unresolved lane:
// the k unresolved lanes get 64 / k consecutive candidates each, and a lane is resolved by its
// lowest accepted candidate.  Identical results to sampling each lane alone (candidate 1000 is taken
// unconditionally, as the serial loop does after 1000 rejections), in ~(sum of tries) / 64 rounds
// instead of (max tries over the wave).
__device__ __forceinline__ int nth_set_bit(uint64_t m, int n)
{
    // position of the n-th (0-based) set bit of m, by halving the search window
    int pos = 0;
    #pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t lo = m & ((w == 64) ? ~0ull : ((1ull << w) - 1ull));
        const int c = __popcll(lo);
        if (n >= c) { n -= c; m >>= w; pos += w; }
        else m = lo;
    }
    return pos;
}

// Per-round constants of the wave sampler for k = 1..64 unresolved lanes (k is wave-uniform, so
// each is one scalar load): div16[k] = ceil(2^16 / k), which gives x / k = (x div16[k]) >> 16
// exactly for 0 <= x <= 128 (checked for every k and x), and stride[k] = the bits 0, k, 2k, ...
// below 64 (a lane's helpers are its rank + that, as a mask).
struct SampleTabs {
    uint32_t div16[65];
    uint64_t stride[65];
};
constexpr SampleTabs make_sample_tabs()
{
    SampleTabs t{};
    for (int k = 1; k <= 64; ++k) {
        t.div16[k] = (65536u + (uint32_t)k - 1u) / (uint32_t)k;
        uint64_t m = 0;
        for (int i = 0; i < 64; i += k) m |= 1ull << i;
        t.stride[k] = m;
    }
    return t;
}
static __constant__ SampleTabs c_sample_tabs = make_sample_tabs();   // internal linkage: the header may enter several translation units

__device__ __forceinline__ int sample_joints_wave(const ctr_system_t &sy, uint64_t seed, uint32_t epoch,
                                                  uint32_t stream, uint64_t env, bool need, float q[6])
{
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const uint32_t ctr2 = (uint32_t)env, ctr3 = (uint32_t)(env >> 32) ^ (stream << 24);
    uint32_t next = 0;               // first candidate of this lane's sequence not yet evaluated
    uint32_t answer = 0;
    bool unresolved = need;
    for (;;) {
        const uint64_t m = __ballot(unresolved);
        if (!m) break;
        const int cnt = __popcll(m);
        const uint32_t dv = c_sample_tabs.div16[cnt];
        const int lq = (int)(((uint32_t)lane * dv) >> 16);          // lane / cnt
        const int target = nth_set_bit(m, lane - lq * cnt);          // lane % cnt
        const uint32_t c = (uint32_t)__shfl((int)next, target) + (uint32_t)lq;
        const uint32_t t_ep = (uint32_t)__shfl((int)epoch, target);
        const uint32_t t2 = (uint32_t)__shfl((int)ctr2, target), t3 = (uint32_t)__shfl((int)ctr3, target);
        double tl[3];
        #pragma unroll
        for (int i = 0; i < 3; ++i) tl[i] = __shfl(sy.L[i], target);
        bool ok = false;
        if (c < 1000u) {
            uint32_t c0[4] = {3u * c, t_ep, t2, t3}, c1[4] = {3u * c + 1u, t_ep, t2, t3};
            philox(c0, k0, k1);
            philox(c1, k0, k1);
            const double u[3] = {u53(c0[0], c0[1]), u53(c0[2], c0[3]), u53(c1[0], c1[1])};
            float b[3];
            #pragma unroll
            for (int i = 0; i < 3; ++i) {
                const double lo = (double)(float)(-tl[i] + 1e-3);
                b[i] = (float)(lo + (0.0 - lo) * u[i]);
            }
            ok = true;
            #pragma unroll
            for (int i = 1; i < 3; ++i) {
                const float lhs = b[i - 1] + (float)tl[i - 1];
                const float rhs_ = (float)tl[i] + b[i];
                ok = ok && (b[i - 1] <= b[i]) && (lhs >= rhs_);
            }
        } else if (c == 1000u) {
            ok = true;                                    // tries > 1000: the serial loop stops here
        }
        const uint64_t acc = __ballot(ok);
        if (unresolved) {
            const int rank = __popcll(m & ((1ull << lane) - 1ull));
            const uint64_t mine = c_sample_tabs.stride[cnt] << rank;   // this lane's helpers: rank, rank + cnt, ...
            const uint64_t hit = acc & mine;
            if (hit) {
                answer = next + ((uint32_t)(__builtin_ctzll(hit) - rank) * dv >> 16);
                unresolved = false;
            } else {
                next += (uint32_t)(64 - rank + cnt - 1) * dv >> 16;
            }
        }
    }
    if (!need) return 0;
    // the chosen candidate in full: extensions and angles (blocks 3a, 3a + 1, 3a + 2)
    uint32_t c0[4] = {3u * answer, epoch, ctr2, ctr3}, c1[4] = {3u * answer + 1u, epoch, ctr2, ctr3},
             c2[4] = {3u * answer + 2u, epoch, ctr2, ctr3};
    philox(c0, k0, k1);
    philox(c1, k0, k1);
    philox(c2, k0, k1);
    const double u[6] = {u53(c0[0], c0[1]), u53(c0[2], c0[3]), u53(c1[0], c1[1]),
                         u53(c1[2], c1[3]), u53(c2[0], c2[1]), u53(c2[2], c2[3])};
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double lo = (double)(float)(-sy.L[i] + 1e-3);
        q[i] = (float)(lo + (0.0 - lo) * u[i]);
        const double alo = -3.1415927410125732, ahi = 3.1415927410125732;
        q[3 + i] = (float)(alo + (ahi - alo) * u[3 + i]);
    }
    return (int)answer + 1;
}

// Uniform system pick (np.random.randint(n_systems), ctr_reach_env.py:95) from the stream.
__device__ __forceinline__ int sample_system(uint64_t seed, uint32_t epoch, uint64_t env, int n_systems)
{
    if (n_systems <= 1) return 0;
    uint32_t c[4] = {0u, epoch, (uint32_t)env, (uint32_t)(env >> 32) ^ (2u << 24)};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    int s = (int)(u53(c[0], c[1]) * (double)n_systems);
    return s < n_systems ? s : n_systems - 1;
}

// Domain randomisation: the tube table of reset `epoch` of env `env` (Model.randomize_parameters,
// model.py:20-28; sample_parameters / randomize_value, model_utils.py:5-35; Tube.__init__,
// Tube.py:7-19).  Per tube j, five uniforms u[5j .. 5j+4] from Philox stream 3 re-sample
// (d_in, d_out, E, G, U_x) as numpy's uniform(low, high) = low + (high - low) * u with
// low = v - v*rand, high = v + v*rand; L, L_c and U_y keep their values (randomisation 0).
// d^4 is (d*d)*(d*d) (the reference uses math.pow; <= 1 ulp apart), I = pi d4 / 64,
// J = pi d4 / 32, EI = E*I, GJ = G*J.
__device__ __forceinline__ void domain_system(const ctr_system_t &base, const ctr_tube_raw_t &raw, double rnd,
                                              uint64_t seed, uint32_t epoch, uint64_t env, ctr_system_t &out,
                                              ctr_tube_raw_t *raw_out)
{
#pragma clang fp contract(off)
    double u[16];
    #pragma unroll
    for (int blk = 0; blk < 8; ++blk) {
        uint32_t c[4] = {(uint32_t)blk, epoch, (uint32_t)env, (uint32_t)(env >> 32) ^ (3u << 24)};
        philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
        u[2 * blk] = u53(c[0], c[1]);
        u[2 * blk + 1] = u53(c[2], c[3]);
    }
    #pragma unroll
    for (int j = 0; j < 3; ++j) {
        double v[5] = {raw.Din[j], raw.Dout[j], raw.E[j], raw.G[j], base.Ux[j]};
        #pragma unroll
        for (int k = 0; k < 5; ++k) {
            const double lo = v[k] - v[k] * rnd, hi = v[k] + v[k] * rnd;
            v[k] = lo + (hi - lo) * u[5 * j + k];
        }
        const double di2 = v[0] * v[0], do2 = v[1] * v[1];
        const double d4 = do2 * do2 - di2 * di2;
        const double J = (3.141592653589793 * d4) / 32.0;
        const double I = (3.141592653589793 * d4) / 64.0;
        out.L[j] = base.L[j];
        out.Lc[j] = base.Lc[j];
        out.EI[j] = v[2] * I;
        out.GJ[j] = v[3] * J;
        out.Ux[j] = v[4];
        out.Uy[j] = base.Uy[j];
        if (raw_out) {
            raw_out->Din[j] = v[0];
            raw_out->Dout[j] = v[1];
            raw_out->E[j] = v[2];
            raw_out->G[j] = v[3];
        }
    }
}

}  // namespace ctr
