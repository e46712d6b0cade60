/* sanitize_main.c -- TEST INFRASTRUCTURE ONLY: drives the CPU oracle (ctr_oracle.c) built with
 * -fsanitize=address,undefined over sampled joints, edge joints (ties, limits, a tube gap that
 * must stop with a NaN tip) and a few env steps, so memory and UB errors in the host restatement
 * surface (sanitizers on host code).  Exit 0 = clean run. */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../ctr_oracle.h"

static void system0(oracle_system_t *s)
{
    /* registration system ctr_0 (ctr_reach_envs/__init__.py), I and J as Tube.__init__ */
    const double L[3] = {0.431, 0.332, 0.174}, Lc[3] = {0.103, 0.113, 0.134};
    const double di[3] = {0.0007, 0.0014, 0.002}, dout[3] = {0.0011, 0.0018, 0.0024};
    const double E[3] = {102500000000.0, 686000000000.0, 169600000000.0};
    const double G[3] = {187900000000.0, 115300000000.0, 142500000000.0};
    const double Ux[3] = {21.3, 13.1, 3.5};
    memset(s, 0, sizeof *s);
    for (int i = 0; i < 3; ++i) {
        s->L[i] = L[i]; s->Lc[i] = Lc[i]; s->E[i] = E[i]; s->G[i] = G[i]; s->Ux[i] = Ux[i];
        s->I[i] = M_PI * (pow(dout[i], 4) - pow(di[i], 4)) / 64.0;
        s->J[i] = 2.0 * s->I[i];
    }
}

int main(void)
{
    oracle_system_t sy;
    system0(&sy);
    enum { N = 64 };
    float q[N * 6];
    int32_t tries[N];
    oracle_sample_joints(N, &sy, NULL, 7, NULL, 0, 0, q, tries);
    /* edge rows: all retracted to the limit, equal betas, huge angles, a tube gap */
    const float edge[4][6] = {{-0.43f, -0.331f, -0.173f, 0.f, 0.f, 0.f},
                              {-0.1f, -0.1f, -0.1f, 1e6f, -1e6f, 3.f},
                              {0.f, 0.f, 0.f, 0.5f, 0.5f, 0.5f},
                              {-0.43f, 0.01f, 0.02f, 0.f, 0.f, 0.f}};   /* tubes 1, 2 start past tube 0 tip */
    memcpy(q, edge, sizeof edge);
    double tip[N * 3];
    int32_t nfev[N], nstep[N], nseg[N], status[N];
    oracle_fk(q, NULL, N, &sy, tip, nfev, nstep, nseg, status);
    double shape_r[N * 270 * 3], shape_s[N * 270], shape_tip[N * 3];
    int32_t npts[N], st2[N];
    oracle_fk_shape(q, NULL, N, &sy, 270, shape_tip, shape_r, shape_s, npts, st2);
    double jq[8 * 6], jtip[8 * 3], jac[8 * 18];
    for (int i = 0; i < 8 * 6; ++i) jq[i] = q[6 * 8 + i];
    oracle_jacobian(jq, NULL, 8, &sy, 0, 0, 0, 1e-4, jtip, jac);
    /* a few env steps */
    float a[N * 6];
    for (int i = 0; i < N * 6; ++i) a[i] = (i % 6 < 3) ? 1e-3f * ((i % 5) - 2) / 2.f : 0.05f * ((i % 7) - 3);
    double dg[N * 3], ach[N * 3], obs[N * 14], rew[N], err[N], tol[N];
    uint8_t done[N], succ[N];
    int32_t t[N];
    memset(t, 0, sizeof t);
    for (int i = 0; i < N * 3; ++i) dg[i] = isfinite(tip[i]) ? tip[i] : 0.0;
    for (int i = 0; i < N; ++i) tol[i] = 0.02;
    for (int k = 0; k < 3; ++k)
        oracle_step(N, &sy, NULL, q, a, dg, t, tol, 10, 150, 0, 0, 1, ach, obs, rew, done, succ, err, nfev);
    int gap_nan = isnan(tip[3 * 3]);
    printf("sanitized oracle run: tube-gap row NaN=%d, step t[4]=%d\n", gap_nan, t[4]);
    return gap_nan && t[4] == 3 ? 0 : 1;
}
