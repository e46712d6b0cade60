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
//   sample_joints_lane envs/obs.py:185-207 (Philox4x32-10 stream instead of numpy MT19937)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ctr_reach_amd.h"

namespace ctr {

constexpr int NS = 18;  // [u_z(3), alpha(3), r(3), R row-major(9)]   (model.py:136)

// ------------------------------------------------------------------------------------------
// Segmentation (Segment.py:6-61).  Ten transition points [0, beta, d_c, d_tip] are sorted,
// the gaps floored to 10 um, and per-gap tube presence / curvature decided.  The result is
// kept "raw" (9 gaps in sorted order, many of which are dropped later) so that every array
// index is static; integration walks the gaps with a cursor.
// ------------------------------------------------------------------------------------------
struct Seg {
    double end[9];     // cumsum(len[0..k]) + min(beta): end arclength of raw gap k
    uint32_t kept;     // bit k: gap k has non-zero length and ends after s = 0 (kept in S)
    uint64_t mask;     // 6 bits per gap: bits 0-2 tube i present (EI != 0), 3-5 tube i curved
};

__device__ __forceinline__ void cswap(double &a, double &b, int &ia, int &ib)
{
    // Stable compare-exchange: swap only when strictly out of order.
    bool s = b < a;
    double ta = s ? b : a, tb = s ? a : b;
    int ja = s ? ib : ia, jb = s ? ia : ib;
    a = ta; b = tb; ia = ja; ib = jb;
}

__device__ __forceinline__ Seg seg_build(const ctr_system_t &sy, const double beta[3])
{
#pragma clang fp contract(off)
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
    #pragma unroll
    for (int k = 0; k < 9; ++k) len[k] = 1e-5 * floor(1e5 * (v[k + 1] - v[k]));   // :16

    uint64_t mask = 0;
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        int a = 0, b = 0, c = 0;
        #pragma unroll
        for (int k = 0; k < 10; ++k) {
            a = (id[k] == i + 1) ? k : a;
            b = (id[k] == i + 4) ? k : b;
            c = (id[k] == i + 7) ? k : c;
        }
        auto len_at = [&](int x) {
            double r = 1.0;              // index 9 is never zero-tested by the reference
            #pragma unroll
            for (int k = 0; k < 9; ++k) r = (x == k) ? len[k] : r;
            return r;
        };
        if (len_at(a) == 0) a += 1;       // :29-36
        if (len_at(b) == 0) b += 1;
        if (len_at(a) == 0) a += 1;
        if (c <= 8 && len_at(c) == 0) c += 1;
        #pragma unroll
        for (int k = 0; k < 9; ++k) {
            uint64_t pres = (k >= a && k < c) ? 1ull : 0ull;
            uint64_t curv = (k >= b && k < c) ? 1ull : 0ull;
            mask |= (pres << (6 * k + i)) | (curv << (6 * k + 3 + i));
        }
    }
    double bmin = fmin(fmin(beta[0], beta[1]), beta[2]);
    Seg sg;
    sg.kept = 0;
    sg.mask = mask;
    double cum = 0.0;
    #pragma unroll
    for (int k = 0; k < 9; ++k) {         // :46-55 (adding a zero gap is an exact no-op)
        cum += len[k];
        sg.end[k] = cum + bmin;
        sg.kept |= ((len[k] != 0.0) && (cum + bmin > 0.0)) ? (1u << k) : 0u;
    }
    return sg;
}

__device__ __forceinline__ double sel9(const double a[9], int k)
{
    double r = a[0];
    #pragma unroll
    for (int j = 1; j < 9; ++j) r = (k == j) ? a[j] : r;
    return r;
}

// Per-segment RHS constants.  w* = EI_j * U*_j exactly as the reference's left-to-right
// product ei[j] * ux_0[j] (model.py:85-90); kz = EI/GJ (model.py:97).
struct SegPar {
    double wx[3], wy[3], ux0[3], uy0[3], kz[3], inv;
    uint32_t present;  // bit j: tube j present (EI_j != 0)
};

__device__ __forceinline__ SegPar seg_par(const ctr_system_t &sy, uint32_t bits6)
{
    SegPar p;
    double esum = 0.0;
    double ei[3];
    #pragma unroll
    for (int j = 0; j < 3; ++j) {
        bool pres = (bits6 >> j) & 1u;
        bool curv = (bits6 >> (3 + j)) & 1u;
        ei[j] = pres ? sy.EI[j] : 0.0;
        double gj = pres ? sy.GJ[j] : 1.0;
        p.ux0[j] = curv ? sy.Ux[j] : 0.0;
        p.uy0[j] = curv ? sy.Uy[j] : 0.0;
        p.wx[j] = ei[j] * p.ux0[j];
        p.wy[j] = ei[j] * p.uy0[j];
        p.kz[j] = pres ? ei[j] / gj : 0.0;
    }
    esum = (ei[0] + ei[1]) + ei[2];
    p.inv = 1.0 / esum;
    p.present = (uint32_t)(bits6 & 7u);
    return p;
}

// ------------------------------------------------------------------------------------------
// RHS of the torsionally compliant model (model.py:72-117).  The three distinct relative
// angles alpha_i - alpha_j are evaluated once each (sin odd, cos even).
// ------------------------------------------------------------------------------------------
template <bool HAS_UY>
__device__ __forceinline__ void rhs(const SegPar &p, const double *y, double *dy)
{
    double s10, c10, s20, c20, s21, c21;
    sincos(y[4] - y[3], &s10, &c10);
    sincos(y[5] - y[3], &s20, &c20);
    sincos(y[5] - y[4], &s21, &c21);
    // c[i][j] = cos(a_i - a_j), s[i][j] = sin(a_i - a_j)
    const double c[3][3] = {{1.0, c10, c20}, {c10, 1.0, c21}, {c20, c21, 1.0}};
    const double s[3][3] = {{0.0, -s10, -s20}, {s10, 0.0, -s21}, {s20, s21, 0.0}};
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
        double tz = HAS_UY ? (ux[j] * p.uy0[j] - uy[j] * p.ux0[j]) : (-uy[j] * p.ux0[j]);
        dy[j] = p.kz[j] * tz;                                  // model.py:97 (0 if absent)
        dy[3 + j] = ((p.present >> j) & 1u) ? y[j] : 0.0;      // model.py:98
    }
    const double *R = y + 9;
    const double uz = y[0], a = ux[0], b = uy[0];
    dy[6] = R[2]; dy[7] = R[5]; dy[8] = R[8];                  // dr = R e3
    #pragma unroll
    for (int r = 0; r < 3; ++r) {                               // dR = R [u]x
        const double r0 = R[3 * r], r1 = R[3 * r + 1], r2 = R[3 * r + 2];
        dy[9 + 3 * r + 0] = r1 * uz - r2 * b;
        dy[9 + 3 * r + 1] = r2 * a - r0 * uz;
        dy[9 + 3 * r + 2] = r0 * b - r1 * a;
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
}  // namespace rk

struct FkStats {
    uint32_t nfev, nstep, nrej, nseg, status;
};

__device__ __forceinline__ double rms18(const double *x)
{
    double s = 0.0;
    #pragma unroll
    for (int i = 0; i < NS; ++i) s += x[i] * x[i];
    return sqrt(s) * 0.23570226039551584;   // 1/sqrt(18)
}

// Forward kinematics of one lane: joints (f32, promoted to f64 as model.py:51) -> tip (f64).
template <bool HAS_UY>
__device__ void fk_lane(const ctr_system_t &sy, const float q[6], double tip[3], FkStats &st)
{
    using namespace rk;
    const double beta[3] = {(double)q[0], (double)q[1], (double)q[2]};
    const Seg sg = seg_build(sy, beta);

    double y[NS];
    {
        const double a0 = (double)q[3];
        double s0, c0;
        sincos(a0, &s0, &c0);
        #pragma unroll
        for (int i = 0; i < NS; ++i) y[i] = 0.0;
        y[3] = (double)q[3]; y[4] = (double)q[4]; y[5] = (double)q[5];
        y[9] = c0; y[10] = -s0; y[12] = s0; y[13] = c0; y[17] = 1.0;   // R0 = Rz(alpha_0)
    }

    double f[NS];
    SegPar p;
    double t = 0.0, tb = 0.0, ha = 0.0, min_step = 0.0, prev_end = 0.0;
    uint32_t remaining = sg.kept;   // kept gaps not yet integrated, in arclength order
    bool need_init = true, new_step = true, rejected = false;

    for (;;) {
        if (need_init) {
            // advance to the next kept gap (Segment.S), or finish
            if (remaining == 0) break;
            const int k = __builtin_ctz(remaining);
            remaining &= remaining - 1u;
            p = seg_par(sy, (uint32_t)((sg.mask >> (6 * k)) & 63u));
            const double endk = sel9(sg.end, k);
            const double a = prev_end, b = endk - 1e-6;     // model.py:141 linspace endpoints
            const double t0 = fmin(a, b);
            tb = fmax(a, b);                                 // :145-151 sorted span
            prev_end = endk;
            rhs<HAS_UY>(p, y, f);                            // RungeKutta.__init__: f = fun(t0, y0)
            st.nfev++;
            st.nseg++;
            const double interval = tb - t0;
            if (interval == 0.0) continue;                   // OdeSolver.step: t == t_bound
            // select_initial_step (common.py:68-140), order 4, direction +1
            double sc[NS], tmp[NS];
            #pragma unroll
            for (int i = 0; i < NS; ++i) sc[i] = ATOL + fabs(y[i]) * RTOL;
            #pragma unroll
            for (int i = 0; i < NS; ++i) tmp[i] = y[i] / sc[i];
            const double d0 = rms18(tmp);
            #pragma unroll
            for (int i = 0; i < NS; ++i) tmp[i] = f[i] / sc[i];
            const double d1 = rms18(tmp);
            double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
            h0 = fmin(h0, interval);
            double y1[NS], f1[NS];
            #pragma unroll
            for (int i = 0; i < NS; ++i) y1[i] = y[i] + h0 * f[i];
            rhs<HAS_UY>(p, y1, f1);
            st.nfev++;
            #pragma unroll
            for (int i = 0; i < NS; ++i) tmp[i] = (f1[i] - f[i]) / sc[i];
            const double d2 = rms18(tmp) / h0;
            double h1;
            if (d1 <= 1e-15 && d2 <= 1e-15) h1 = fmax(1e-6, h0 * 1e-3);
            else h1 = pow(0.01 / fmax(d1, d2), 0.2);
            ha = fmin(fmin(100.0 * h0, h1), interval);
            t = t0;
            need_init = false;
            new_step = true;
        }

        // ---- one attempt of RungeKutta._step_impl (rk.py:111-175) ----
        if (new_step) {
            min_step = 10.0 * fabs(nextafter(t, INFINITY) - t);
            if (ha < min_step) ha = min_step;
            rejected = false;
            new_step = false;
        }
        if (ha < min_step) {                         // TOO_SMALL_STEP -> solver failed
            st.status |= CTR_STATUS_STEP_UNDERFLOW;
            break;
        }
        double tnew = t + ha;
        if (tnew - tb > 0.0) tnew = tb;
        const double h = tnew - t;
        ha = fabs(h);

        double K1[NS], K2[NS], K3[NS], K4[NS], K5[NS], K6[NS], yt[NS];
        #pragma unroll
        for (int i = 0; i < NS; ++i) yt[i] = y[i] + (f[i] * A10) * h;
        rhs<HAS_UY>(p, yt, K1);
        #pragma unroll
        for (int i = 0; i < NS; ++i) yt[i] = y[i] + (f[i] * A20 + K1[i] * A21) * h;
        rhs<HAS_UY>(p, yt, K2);
        #pragma unroll
        for (int i = 0; i < NS; ++i) yt[i] = y[i] + (f[i] * A30 + K1[i] * A31 + K2[i] * A32) * h;
        rhs<HAS_UY>(p, yt, K3);
        #pragma unroll
        for (int i = 0; i < NS; ++i)
            yt[i] = y[i] + (f[i] * A40 + K1[i] * A41 + K2[i] * A42 + K3[i] * A43) * h;
        rhs<HAS_UY>(p, yt, K4);
        #pragma unroll
        for (int i = 0; i < NS; ++i)
            yt[i] = y[i] + (f[i] * A50 + K1[i] * A51 + K2[i] * A52 + K3[i] * A53 + K4[i] * A54) * h;
        rhs<HAS_UY>(p, yt, K5);
        double ynew[NS];
        #pragma unroll
        for (int i = 0; i < NS; ++i)
            ynew[i] = y[i] + h * (f[i] * B0 + K2[i] * B2 + K3[i] * B3 + K4[i] * B4 + K5[i] * B5);
        rhs<HAS_UY>(p, ynew, K6);
        st.nfev += 6;
        double en2 = 0.0;
        #pragma unroll
        for (int i = 0; i < NS; ++i) {
            const double scale = ATOL + fmax(fabs(y[i]), fabs(ynew[i])) * RTOL;
            const double e = ((f[i] * E0 + K2[i] * E2 + K3[i] * E3 + K4[i] * E4 + K5[i] * E5 + K6[i] * E6) * h)
                             / scale;
            en2 += e * e;
        }
        const double en = sqrt(en2) * 0.23570226039551584;
        if (en < 1.0) {
            double factor = (en == 0.0) ? 10.0 : fmin(10.0, 0.9 * pow(en, -0.2));
            if (rejected) factor = fmin(1.0, factor);
            ha *= factor;
            #pragma unroll
            for (int i = 0; i < NS; ++i) { y[i] = ynew[i]; f[i] = K6[i]; }
            t = tnew;
            st.nstep++;
            new_step = true;
            if (t - tb >= 0.0) need_init = true;    // segment finished (status 'finished')
        } else {
            ha *= fmax(0.2, 0.9 * pow(en, -0.2));
            rejected = true;
            st.nrej++;
        }
    }
    tip[0] = y[6]; tip[1] = y[7]; tip[2] = y[8];
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
        v = v < lo ? lo : v;
        v = v > hi ? hi : v;
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

// obs.py:136-164.  Writes obs_dim (13 or 14) floats.
__device__ __forceinline__ void obs_lane(const float q[6], const double dg[3], const double ag[3], double tol,
                                         int sys, bool multi, bool egocentric, float *out)
{
    #pragma unroll
    for (int i = 0; i < 3; ++i) {
        double b = (double)q[i], a = (double)q[3 + i];
        if (egocentric && i > 0) { b -= (double)q[i - 1]; a -= (double)q[3 + i - 1]; }
        double s, c;
        sincos(a, &s, &c);
        out[3 * i + 0] = (float)c;
        out[3 * i + 1] = (float)s;
        out[3 * i + 2] = (float)b;
    }
    #pragma unroll
    for (int k = 0; k < 3; ++k) out[9 + k] = (float)(dg[k] - ag[k]);
    out[12] = (float)tol;
    if (multi) out[13] = (float)sys;
}

// ------------------------------------------------------------------------------------------
// Philox4x32-10 counter RNG and the sample_goal rejection sampler.
// counter = {draw, epoch, env_lo, env_hi ^ (stream << 24)}, key = seed.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1)
{
    #pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}

__device__ __forceinline__ double u53(uint32_t a, uint32_t b)
{
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// Returns the number of candidates drawn; sets q.  Restates obs.py:185-207.
__device__ __forceinline__ int sample_joints_lane(const ctr_system_t &sy, uint64_t seed, uint32_t epoch,
                                                  uint32_t stream, uint64_t env, float q[6])
{
#pragma clang fp contract(off)
    uint32_t draw = 0;
    int tries = 0;
    for (;;) {
        double u[6];
        #pragma unroll
        for (int blk = 0; blk < 3; ++blk) {
            uint32_t c[4] = {draw, epoch, (uint32_t)env, (uint32_t)(env >> 32) ^ (stream << 24)};
            philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
            ++draw;
            u[2 * blk] = u53(c[0], c[1]);
            u[2 * blk + 1] = u53(c[2], c[3]);
        }
        float b[3], al[3];
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double lo = (double)(float)(-sy.L[i] + 1e-3);
            b[i] = (float)(lo + (0.0 - lo) * u[i]);
            const double alo = -3.1415927410125732, ahi = 3.1415927410125732;
            al[i] = (float)(alo + (ahi - alo) * u[3 + i]);
        }
        ++tries;
        bool ok = true;
        #pragma unroll
        for (int i = 1; i < 3; ++i) {
            const float lhs = b[i - 1] + (float)sy.L[i - 1];
            const float rhs_ = (float)sy.L[i] + b[i];
            ok = ok && (b[i - 1] <= b[i]) && (lhs >= rhs_);
        }
        if (ok || tries > 1000) {
            #pragma unroll
            for (int i = 0; i < 3; ++i) { q[i] = b[i]; q[3 + i] = al[i]; }
            return tries;
        }
    }
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

}  // namespace ctr
