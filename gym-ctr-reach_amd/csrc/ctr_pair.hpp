// ctr_pair.hpp -- forward kinematics of 64 environments on a PAIR of waves (scipy RK45,
// torsionally compliant model): k_step / k_fk for the reference's configuration.
//
// Why a pair.  One env per lane needs ~380 registers per lane (the 18-vector state, six RK stages
// and the controller), so 65 536 envs are exactly one wave per SIMD: every fp64 latency is
// exposed and every non-fp64 instruction costs a full issue slot.  The ODE splits cleanly:
//   (u_z, alpha)  is autonomous: d(u_z)/ds and d(alpha)/ds depend on u_z and alpha only, through
//                 the three relative-angle sin/cos pairs (model.py:83-98);
//   (R, r)        is driven: dR/ds = R [u]x needs only the curvature triple u = (u_x0, u_y0,
//                 u_z0) of the stage (model.py:103-109), dr/ds = R e3.
// Wave A (threads 0-63) integrates (u_z, alpha), evaluates the trig and runs the step-size
// controller; wave B (threads 64-127) integrates (R, r).  Per RHS evaluation A hands B the
// triple through LDS; per segment start and per attempt B hands A its partial norms.  Each
// wave holds about half the state, so two pairs' waves share a SIMD and hide each other's
// latency: 65 536 envs become 2 048 waves, two per SIMD.
//
// Arithmetic is the single-lane fk_lane's (csrc/ctr_device.hpp) component for component; only
// the norms are summed as (A's part) + (B's part), which moves them by rounding.
//
// Synchronisation.  Both waves run the same loop and meet at the same barriers (workgroup =
// one pair, so a barrier joins exactly A and B).  One iteration:
//   A: decide (segment start? which lanes attempt?), segment start part 1   | B: -
//   -- S_a --  B learns the flags and applies the previous attempt's acceptance
//   [segment-start block, only if some lane starts a segment:]
//     B: f_R at y, partial d0 / d1                | A: -
//     -- S_b --  A: h0, probe stage, partial d2   | B: -
//     -- S_c --  B: probe R', partial d2          | A: -
//     -- S_d --  A: h1 -> h
//   A: stage 1 triple                              | B: -
//   -- S_1 -- B: stage 1 | A: stage 2 -- S_2 -- ... -- S_5 -- B: stage 5 | A: y_new, K6 triple
//   -- S_6 -- B: y_new, K6, partial error          | A: -
//   -- S_7 -- A: error norm, accept / reject, next h
// The loop ends when A has no active lane (a flag read by both after S_a).
#pragma once
#include "ctr_device.hpp"

namespace ctr {

constexpr int PAIR_LANES = 64;                    // envs per pair (one wave each for A and B)
constexpr int PAIR_BLOCK = 2 * PAIR_LANES;        // one pair per workgroup

// A -> B per-lane flags
constexpr uint32_t PF_INIT = 1u;      // this iteration runs the segment-start block for the lane
constexpr uint32_t PF_ACCEPT = 2u;    // the lane's previous attempt was accepted: y <- y_new
constexpr uint32_t PF_NAN = 4u;       // the FK ended with a NaN tip (tube gap / NaN step size)

struct PairLds {
    double u[8][3][PAIR_LANES];   // curvature triples (u_z0, u_x0, u_y0): 0 = f at a segment
                                  // start, 1 = select_initial_step probe, 2..7 = stages K1..K6
    double part[3][PAIR_LANES];   // B -> A partial sums: d0 / d1 at a segment start, then d2;
                                  // the attempt's error sum reuses part[0]
    double part1[PAIR_LANES];
    double h0[PAIR_LANES];        // A -> B: probe step of select_initial_step
    double h[PAIR_LANES];         // A -> B: the attempt's step (0: no attempt)
    double a0[PAIR_LANES];        // A -> B: alpha_0 of the joints (R0 = Rz(alpha_0))
    double tip[3][PAIR_LANES];    // B -> A: r at the end
    uint32_t flags[PAIR_LANES];
    int32_t any_init;             // A -> B: some lane runs the segment-start block
    int32_t cont;                 // A -> B: some lane is still integrating
};

// The A-side RHS: d(u_z)/ds and the curvature triple (u_z0, u_x0, u_y0) of the stage (rhs_core's
// arithmetic without the frame product).
template <bool HAS_UY>
__device__ __forceinline__ void rhs_A(const SegPar &p, const Trig &t, const double uz[3], double duz[3], double &ua,
                                      double &ub)
{
    if constexpr (!HAS_UY) {
        const double sy1 = fma(p.wx[2], t.s20, p.wx[1] * t.s10);
        const double sy2 = fma(p.wx[2], t.s21, -(p.wx[0] * t.s10));
        const double sy3 = fma(p.wx[1], t.s21, p.wx[0] * t.s20);
        duz[0] = -(p.g[0] * sy1);
        duz[1] = -(p.g[1] * sy2);
        duz[2] = p.g[2] * sy3;
        ua = p.inv * fma(p.wx[2], t.c20, fma(p.wx[1], t.c10, p.wx[0]));
        ub = p.inv * sy1;
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
            sx += p.wy[j] * s[i][j];
            sy += p.wy[j] * c[i][j];
        }
        ux[i] = p.inv * sx;
        uy[i] = p.inv * sy;
    }
    #pragma unroll
    for (int j = 0; j < 3; ++j) duz[j] = p.kz[j] * (ux[j] * p.uy0[j] - uy[j] * p.ux0[j]);
    ua = ux[0];
    ub = uy[0];
}

// The B-side RHS: dR = R [u]x for u = (a, b, u0) (model.py:103-110), rhs_core's expressions.
__device__ __forceinline__ void rhs_B(const double R[9], double u0, double a, double b, double dR[9])
{
    #pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double r0 = R[3 * r], r1 = R[3 * r + 1], r2 = R[3 * r + 2];
        dR[3 * r + 0] = r1 * u0 - r2 * b;
        dR[3 * r + 1] = r2 * a - r0 * u0;
        dR[3 * r + 2] = r0 * b - r1 * a;
    }
}

__device__ __forceinline__ void pair_put_u(PairLds &X, int slot, int lane, double u0, double a, double b)
{
    X.u[slot][0][lane] = u0;
    X.u[slot][1][lane] = a;
    X.u[slot][2][lane] = b;
}

// ------------------------------------------------------------------------------------------
// Wave A: (u_z, alpha), trig, step-size control.  `live` = the lane has an env.  Returns the tip
// (from B) in tip[].  Every lane of the wave calls it; so does every lane of wave B (fk_pair_B).
template <bool HAS_UY, bool CAREFUL>
__device__ __forceinline__ void fk_pair_A(const SysK &sy, const double q[6], bool live, double tip[3], FkStats &st, PairLds &X)
{
    using namespace rk;
    const int lane = threadIdx.x & (PAIR_LANES - 1);
    const double beta[3] = {q[0], q[1], q[2]};
    __shared__ double s_endp[9][PAIR_LANES];
    double *end_lds = &s_endp[0][lane];
    const Seg sg = seg_build<PAIR_LANES>(sy, beta, end_lds);

    double yu[3] = {0.0, 0.0, 0.0}, uzf[3] = {0.0, 0.0, 0.0};
    double ya[3] = {q[3], q[4], q[5]};
    X.a0[lane] = ya[0];
    Trig ty = trig_of<CAREFUL>(ya);
    double fu[3] = {0.0, 0.0, 0.0}, fa[3] = {0.0, 0.0, 0.0};   // FSAL derivative (u_z', alpha')
    SegPar p = seg_par(sy, 0u, false);
    double t = 0.0, tb = 0.0, ha = 0.0, min_step = 0.0, prev_end = 0.0;
    uint32_t remaining = sg.kept;
    bool need_init = true, new_step = true, rejected = false, active = live, nan_out = false;
    bool accepted = false;

    for (;;) {
        // ---- decide; segment start, part 1: f at y with the new segment's constants ----
        bool init_ok = false, skip = false;
        double t0 = 0.0, interval = 0.0;
        double isc_u[3], isc_a[3], yuref[3], d0A = 0.0, d1A = 0.0;
        if (active && need_init) {
            if (remaining == 0) {
                active = false;
            } else {
                const int k = __builtin_ctz(remaining);
                remaining &= remaining - 1u;
                p = seg_par(sy, seg_bits(sg, k), false);
                #pragma unroll
                for (int j = 1; j < 3; ++j) {
                    const bool absent = !((p.present >> j) & 1u);
                    uzf[j] = (absent && yu[j] != 0.0) ? yu[j] : uzf[j];
                    yu[j] = absent ? 0.0 : yu[j];
                }
                const double endk = end_lds[k * PAIR_LANES];
                const double a = prev_end, b = endk - 1e-6;       // model.py:141
                t0 = fmin(a, b);
                tb = fmax(a, b);                                  // :145-151
                prev_end = endk;
                double ua, ub;
                rhs_A<HAS_UY>(p, ty, yu, fu, ua, ub);             // RungeKutta.__init__: f = fun(t0, y0)
                #pragma unroll
                for (int j = 0; j < 3; ++j) fa[j] = (j > 0 || (p.present & 1u)) ? yu[j] : 0.0;
                st.nfev++;
                st.nseg++;
                interval = tb - t0;
                if (interval == 0.0) {
                    skip = true;                                  // t == t_bound: next segment
                } else if (p.present == 0u) {
                    nan_out = true;                               // tube gap (see fk_lane)
                    st.status |= CTR_STATUS_NAN;
                    active = false;
                } else {
                    init_ok = true;
                    pair_put_u(X, 0, lane, yu[0], ua, ub);
                    #pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        yuref[i] = (i == 0 || ((p.present >> i) & 1u)) ? yu[i] : uzf[i];
                        isc_u[i] = ctr_math::rcp_est(ATOL + fabs(yuref[i]) * RTOL);
                        isc_a[i] = ctr_math::rcp_est(ATOL + fabs(ya[i]) * RTOL);
                        d0A += (yuref[i] * isc_u[i]) * (yuref[i] * isc_u[i]) + (ya[i] * isc_a[i]) * (ya[i] * isc_a[i]);
                        d1A += (fu[i] * isc_u[i]) * (fu[i] * isc_u[i]) + (fa[i] * isc_a[i]) * (fa[i] * isc_a[i]);
                    }
                }
            }
        }
        X.flags[lane] = (init_ok ? PF_INIT : 0u) | (accepted ? PF_ACCEPT : 0u) | (nan_out ? PF_NAN : 0u);
        accepted = false;
        const bool any_init = __ballot(init_ok) != 0;
        const bool cont = __ballot(active) != 0;
        if (lane == 0) {
            X.any_init = any_init ? 1 : 0;
            X.cont = cont ? 1 : 0;
        }
        __syncthreads();                                                          // S_a
        if (!cont) break;

        if (any_init) {
            __syncthreads();                                                      // S_b
            double h0 = 0.0, d2A = 0.0;
            if (init_ok) {
                double f1u[3], f1a[3];
                // select_initial_step (common.py:68-140): d0, d1 -> h0, probe
                const double s0 = d0A + X.part[0][lane], s1 = d1A + X.part1[lane];
                const double d0sq = s0 * (1.0 / 18), d1sq = s1 * (1.0 / 18);
                const double h0n = 0.01 * ctr_math::sqrt_rsq(s0 * ctr_math::rcp1(s1));
                h0 = (d0sq < 1e-10 || d1sq < 1e-10) ? 1e-6 : h0n;
                h0 = fmin(h0, interval);
                double u1[3], a1[3];
                #pragma unroll
                for (int i = 0; i < 3; ++i) { u1[i] = yu[i] + h0 * fu[i]; a1[i] = ya[i] + h0 * fa[i]; }
                const Trig t1 = trig_of<CAREFUL>(a1);
                double ua, ub;
                rhs_A<HAS_UY>(p, t1, u1, f1u, ua, ub);
                #pragma unroll
                for (int j = 0; j < 3; ++j) f1a[j] = (j > 0 || (p.present & 1u)) ? u1[j] : 0.0;
                pair_put_u(X, 1, lane, u1[0], ua, ub);
                X.h0[lane] = h0;
                st.nfev++;
                #pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const double du = (f1u[i] - fu[i]) * isc_u[i], da = (f1a[i] - fa[i]) * isc_a[i];
                    d2A += du * du + da * da;
                }
            }
            __syncthreads();                                                      // S_c
            __syncthreads();                                                      // S_d
            if (init_ok) {
                const double s1 = d1A + X.part1[lane];
                const double d1sq = s1 * (1.0 / 18);
                const double s2 = d2A + X.part[2][lane];
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
        }

        // ---- one attempt of RungeKutta._step_impl (rk.py:111-175) ----
        bool att = false;
        double h = 0.0, tnew = 0.0;
        if (active && !need_init && !skip) {
            const double ms = 10.0 * fabs(nextafter(t, INFINITY) - t);
            min_step = new_step ? ms : min_step;
            ha = (new_step && ha < ms) ? ms : ha;
            rejected = new_step ? false : rejected;
            new_step = false;
            if (!(ha >= min_step)) {
                if (ha < min_step) {
                    st.status |= CTR_STATUS_STEP_UNDERFLOW;
                } else {
                    nan_out = true;
                    st.status |= CTR_STATUS_NAN;
                }
                active = false;
            } else {
                tnew = t + ha;
                if (tnew - tb > 0.0) tnew = tb;
                h = tnew - t;
                ha = fabs(h);
                att = true;
            }
        }
        X.h[lane] = att ? h : 0.0;
        const double a10 = A10 * h;
        const double a20 = A20 * h, a21 = A21 * h;
        const double a30 = A30 * h, a31 = A31 * h, a32 = A32 * h;
        const double a40 = A40 * h, a41 = A41 * h, a42 = A42 * h, a43 = A43 * h;
        const double a50 = A50 * h, a51 = A51 * h, a52 = A52 * h, a53 = A53 * h, a54 = A54 * h;
        double K1u[3], K1a[3], K2u[3], K2a[3], K3u[3], K3a[3], K4u[3], K4a[3], K5u[3], K5a[3];
        double ui[3], ai[3];
#define CTR_PAIR_STAGE_A(KU, KA, SLOT, EXPR_U, EXPR_A)                                         \
        {                                                                                      \
            _Pragma("unroll") for (int i = 0; i < 3; ++i) { ui[i] = EXPR_U; ai[i] = EXPR_A; }  \
            const Trig tt = trig_of<CAREFUL>(ai);                                              \
            double ua, ub;                                                                     \
            rhs_A<HAS_UY>(p, tt, ui, KU, ua, ub);                                              \
            _Pragma("unroll") for (int j = 0; j < 3; ++j)                                      \
                KA[j] = (j > 0 || (p.present & 1u)) ? ui[j] : 0.0;                             \
            pair_put_u(X, SLOT, lane, ui[0], ua, ub);                                          \
        }
        CTR_PAIR_STAGE_A(K1u, K1a, 2, fma(fu[i], a10, yu[i]), fma(fa[i], a10, ya[i]))
        __syncthreads();                                                          // S_1
        CTR_PAIR_STAGE_A(K2u, K2a, 3, fma(K1u[i], a21, fma(fu[i], a20, yu[i])),
                         fma(K1a[i], a21, fma(fa[i], a20, ya[i])))
        __syncthreads();                                                          // S_2
        CTR_PAIR_STAGE_A(K3u, K3a, 4, fma(K2u[i], a32, fma(K1u[i], a31, fma(fu[i], a30, yu[i]))),
                         fma(K2a[i], a32, fma(K1a[i], a31, fma(fa[i], a30, ya[i]))))
        __syncthreads();                                                          // S_3
        CTR_PAIR_STAGE_A(K4u, K4a, 5,
                         fma(K3u[i], a43, fma(K2u[i], a42, fma(K1u[i], a41, fma(fu[i], a40, yu[i])))),
                         fma(K3a[i], a43, fma(K2a[i], a42, fma(K1a[i], a41, fma(fa[i], a40, ya[i])))))
        __syncthreads();                                                          // S_4
        CTR_PAIR_STAGE_A(K5u, K5a, 6,
                         fma(K4u[i], a54, fma(K3u[i], a53, fma(K2u[i], a52, fma(K1u[i], a51, fma(fu[i], a50, yu[i]))))),
                         fma(K4a[i], a54, fma(K3a[i], a53, fma(K2a[i], a52, fma(K1a[i], a51, fma(fa[i], a50, ya[i]))))))
#undef CTR_PAIR_STAGE_A
        __syncthreads();                                                          // S_5
        // y_new, the error combination and K6 for (u_z, alpha)
        const double b0 = B0 * h, b2 = B2 * h, b3 = B3 * h, b4 = B4 * h, b5 = B5 * h;
        double nu[3], na[3], K6u[3], K6a[3];
        double errA = 0.0;
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            nu[i] = fma(K5u[i], b5, fma(K4u[i], b4, fma(K3u[i], b3, fma(K2u[i], b2, fma(fu[i], b0, yu[i])))));
            na[i] = fma(K5a[i], b5, fma(K4a[i], b4, fma(K3a[i], b3, fma(K2a[i], b2, fma(fa[i], b0, ya[i])))));
        }
        const Trig tn = trig_of<CAREFUL>(na);
        {
            double ua, ub;
            rhs_A<HAS_UY>(p, tn, nu, K6u, ua, ub);
            #pragma unroll
            for (int j = 0; j < 3; ++j) K6a[j] = (j > 0 || (p.present & 1u)) ? nu[j] : 0.0;
            pair_put_u(X, 7, lane, nu[0], ua, ub);
        }
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double eu = fu[i] * E0 + K2u[i] * E2 + K3u[i] * E3 + K4u[i] * E4 + K5u[i] * E5;
            const double ea = fa[i] * E0 + K2a[i] * E2 + K3a[i] * E3 + K4a[i] * E4 + K5a[i] * E5;
            const double xu = fma(K6u[i], E6, eu) * ctr_math::rcp_est(fma(ctr_math::absmax(yu[i], nu[i]), RTOL, ATOL));
            const double xa = fma(K6a[i], E6, ea) * ctr_math::rcp_est(fma(ctr_math::absmax(ya[i], na[i]), RTOL, ATOL));
            errA = fma(xu, xu, errA);
            errA = fma(xa, xa, errA);
        }
        __syncthreads();                                                          // S_6
        __syncthreads();                                                          // S_7
        if (att) {
            st.nfev += 6;
            double en2 = errA + X.part[0][lane];
            en2 *= h * h;
            const double en2n = en2 * (1.0 / 18);
            const double fpow = (en2n < 1e300) ? 0.9 * ctr_math::inv_root10(en2n) : 0.0;
            if (en2n < 1.0) {
                double factor = (en2n == 0.0) ? 10.0 : fmin(10.0, fpow);
                if (rejected) factor = fmin(1.0, factor);
                ha *= factor;
                #pragma unroll
                for (int i = 0; i < 3; ++i) { yu[i] = nu[i]; ya[i] = na[i]; fu[i] = K6u[i]; fa[i] = K6a[i]; }
                ty = tn;
                t = tnew;
                st.nstep++;
                new_step = true;
                accepted = true;
                if (t - tb >= 0.0) {                              // segment finished
                    need_init = true;
                    if (remaining == 0) active = false;
                }
            } else {
                ha *= fmax(0.2, fpow);
                rejected = true;
                st.nrej++;
            }
        }
    }
    __syncthreads();                                                              // S_end: B wrote r
    tip[0] = X.tip[0][lane];
    tip[1] = X.tip[1][lane];
    tip[2] = X.tip[2][lane];
    if (isnan(tip[0]) || isnan(tip[1]) || isnan(tip[2])) st.status |= CTR_STATUS_NAN;
}

// ------------------------------------------------------------------------------------------
// Wave B: (R, r) driven by A's curvature triples.
__device__ __forceinline__ void fk_pair_B(PairLds &X)
{
    using namespace rk;
    const int lane = threadIdx.x & (PAIR_LANES - 1);
    double yr[3] = {0.0, 0.0, 0.0}, yR[9];
    #pragma unroll
    for (int i = 0; i < 9; ++i) yR[i] = 0.0;
    bool first = true;
    double fR[9];                                        // FSAL dR at y (set at the first segment start)
    #pragma unroll
    for (int i = 0; i < 9; ++i) fR[i] = 0.0;
    double nR[9], nr[3], K6R[9];
    #pragma unroll
    for (int i = 0; i < 9; ++i) { nR[i] = 0.0; K6R[i] = 0.0; }
    nr[0] = nr[1] = nr[2] = 0.0;
    bool nan_out = false;

    for (;;) {
        __syncthreads();                                                          // S_a
        if (first) {                                     // A wrote alpha_0 before its first S_a
            double s0, c0;
            ctr_math::sincos_cw(X.a0[lane], &s0, &c0);   // R0 = Rz(alpha_0)  model.py:57-60
            yR[0] = c0; yR[1] = -s0; yR[2] = 0.0;
            yR[3] = s0; yR[4] = c0;  yR[5] = 0.0;
            yR[6] = 0.0; yR[7] = 0.0; yR[8] = 1.0;
            first = false;
        }
        const uint32_t fl = X.flags[lane];
        if (fl & PF_ACCEPT) {
            #pragma unroll
            for (int i = 0; i < 9; ++i) { yR[i] = nR[i]; fR[i] = K6R[i]; }
            #pragma unroll
            for (int i = 0; i < 3; ++i) yr[i] = nr[i];
        }
        nan_out = (fl & PF_NAN) != 0;
        if (!X.cont) break;

        if (X.any_init) {
            const bool init = (fl & PF_INIT) != 0;
            double isc_r[3], isc_R[9];
            if (init) {
                rhs_B(yR, X.u[0][0][lane], X.u[0][1][lane], X.u[0][2][lane], fR);
                double d0B = 0.0, d1B = 0.0;
                #pragma unroll
                for (int i = 0; i < 3; ++i) {
                    isc_r[i] = ctr_math::rcp_est(ATOL + fabs(yr[i]) * RTOL);
                    const double fr = yR[3 * i + 2];
                    d0B += (yr[i] * isc_r[i]) * (yr[i] * isc_r[i]);
                    d1B += (fr * isc_r[i]) * (fr * isc_r[i]);
                }
                #pragma unroll
                for (int i = 0; i < 9; ++i) {
                    isc_R[i] = ctr_math::rcp_est(ATOL + fabs(yR[i]) * RTOL);
                    d0B += (yR[i] * isc_R[i]) * (yR[i] * isc_R[i]);
                    d1B += (fR[i] * isc_R[i]) * (fR[i] * isc_R[i]);
                }
                X.part[0][lane] = d0B;
                X.part1[lane] = d1B;
            }
            __syncthreads();                                                      // S_b
            __syncthreads();                                                      // S_c
            if (init) {
                const double h0 = X.h0[lane];
                double R1[9], f1R[9];
                #pragma unroll
                for (int i = 0; i < 9; ++i) R1[i] = yR[i] + h0 * fR[i];
                rhs_B(R1, X.u[1][0][lane], X.u[1][1][lane], X.u[1][2][lane], f1R);
                double d2B = 0.0;
                #pragma unroll
                for (int i = 0; i < 3; ++i) {
                    const double dr = (R1[3 * i + 2] - yR[3 * i + 2]) * isc_r[i];
                    d2B += dr * dr;
                }
                #pragma unroll
                for (int i = 0; i < 9; ++i) {
                    const double dR = (f1R[i] - fR[i]) * isc_R[i];
                    d2B += dR * dR;
                }
                X.part[2][lane] = d2B;
            }
            __syncthreads();                                                      // S_d
        }

        // ---- the attempt: stages 1..5 one barrier behind A, then y_new / K6 / error ----
        __syncthreads();                                                          // S_1
        const double h = X.h[lane];
        const double a10 = A10 * h;
        const double a20 = A20 * h, a21 = A21 * h;
        const double a30 = A30 * h, a31 = A31 * h, a32 = A32 * h;
        const double a40 = A40 * h, a41 = A41 * h, a42 = A42 * h, a43 = A43 * h;
        const double a50 = A50 * h, a51 = A51 * h, a52 = A52 * h, a53 = A53 * h, a54 = A54 * h;
        double br[3], er[3];
        #pragma unroll
        for (int i = 0; i < 3; ++i) { br[i] = yR[3 * i + 2] * B0; er[i] = yR[3 * i + 2] * E0; }
        double K1R[9], K2R[9], K3R[9], K4R[9], K5R[9], Ri[9];
#define CTR_PAIR_STAGE_B(KR, SLOT, EXPR_R, BCOEF, ECOEF)                                       \
        {                                                                                      \
            _Pragma("unroll") for (int i = 0; i < 9; ++i) Ri[i] = EXPR_R;                      \
            rhs_B(Ri, X.u[SLOT][0][lane], X.u[SLOT][1][lane], X.u[SLOT][2][lane], KR);         \
            _Pragma("unroll") for (int i = 0; i < 3; ++i) {                                    \
                br[i] += Ri[3 * i + 2] * (BCOEF);                                              \
                er[i] += Ri[3 * i + 2] * (ECOEF);                                              \
            }                                                                                  \
        }
        CTR_PAIR_STAGE_B(K1R, 2, fma(fR[i], a10, yR[i]), 0.0, 0.0)
        __syncthreads();                                                          // S_2
        CTR_PAIR_STAGE_B(K2R, 3, fma(K1R[i], a21, fma(fR[i], a20, yR[i])), B2, E2)
        __syncthreads();                                                          // S_3
        CTR_PAIR_STAGE_B(K3R, 4, fma(K2R[i], a32, fma(K1R[i], a31, fma(fR[i], a30, yR[i]))), B3, E3)
        __syncthreads();                                                          // S_4
        CTR_PAIR_STAGE_B(K4R, 5, fma(K3R[i], a43, fma(K2R[i], a42, fma(K1R[i], a41, fma(fR[i], a40, yR[i])))),
                         B4, E4)
        __syncthreads();                                                          // S_5
        CTR_PAIR_STAGE_B(K5R, 6,
                         fma(K4R[i], a54, fma(K3R[i], a53, fma(K2R[i], a52, fma(K1R[i], a51, fma(fR[i], a50, yR[i]))))),
                         B5, E5)
#undef CTR_PAIR_STAGE_B
        __syncthreads();                                                          // S_6
        const double b0 = B0 * h, b2 = B2 * h, b3 = B3 * h, b4 = B4 * h, b5 = B5 * h;
        #pragma unroll
        for (int i = 0; i < 9; ++i)
            nR[i] = fma(K5R[i], b5, fma(K4R[i], b4, fma(K3R[i], b3, fma(K2R[i], b2, fma(fR[i], b0, yR[i])))));
        #pragma unroll
        for (int i = 0; i < 3; ++i) nr[i] = yr[i] + h * br[i];
        rhs_B(nR, X.u[7][0][lane], X.u[7][1][lane], X.u[7][2][lane], K6R);
        double errB = 0.0;
        #pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double xr = fma(nR[3 * i + 2], E6, er[i]) *
                              ctr_math::rcp_est(fma(ctr_math::absmax(yr[i], nr[i]), RTOL, ATOL));
            errB = fma(xr, xr, errB);
        }
        #pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double eR = fR[i] * E0 + K2R[i] * E2 + K3R[i] * E3 + K4R[i] * E4 + K5R[i] * E5;
            const double xR = fma(K6R[i], E6, eR) * ctr_math::rcp_est(fma(ctr_math::absmax(yR[i], nR[i]), RTOL, ATOL));
            errB = fma(xR, xR, errB);
        }
        X.part[0][lane] = errB;
        __syncthreads();                                                          // S_7
    }
    X.tip[0][lane] = nan_out ? NAN : yr[0];
    X.tip[1][lane] = nan_out ? NAN : yr[1];
    X.tip[2][lane] = nan_out ? NAN : yr[2];
    __syncthreads();                                                              // S_end
}

}  // namespace ctr
