/* Diagnostic (not product code): how far the RK45 stage inputs' angle differences move from the
 * step's start, |(a1 - a0)(stage) - (a1 - a0)(y)| and the same for (a2 - a0), over every stage of
 * every attempt of the CPU oracle's FK -- the size of the rotation a stage's sin/cos could be
 * reached by from the trig of y.  Builds the oracle with a stage hook:
 *   gcc -O2 -fPIC -shared -fopenmp -ffp-contract=off -std=c11 -D_GNU_SOURCE tools/dalpha_probe.c -o tools/libdalpha_probe.so -lm
 * and is driven by tools/dalpha_probe.py. */
#include <math.h>
#include <stdint.h>
#define DALPHA_BINS 40
static long long g_hist[2][DALPHA_BINS];      /* bin b: 2^-(b) > |delta| >= 2^-(b+1); bin 0: >= 0.5 */
static void dalpha_stage(const double *y, const double *ys)
{
    const double d[2] = {fabs((ys[4] - ys[3]) - (y[4] - y[3])), fabs((ys[5] - ys[3]) - (y[5] - y[3]))};
    for (int k = 0; k < 2; ++k) {
        int b = 0;
        double lim = 0.5;
        while (b < DALPHA_BINS - 1 && d[k] < lim) { lim *= 0.5; ++b; }
#pragma omp atomic
        g_hist[k][b]++;
    }
}
#define ORACLE_STAGE_HOOK(y, ys) dalpha_stage(y, ys)
#include "../oracle/ctr_oracle.c"

void dalpha_reset(void)
{
    for (int k = 0; k < 2; ++k)
        for (int b = 0; b < DALPHA_BINS; ++b) g_hist[k][b] = 0;
}

void dalpha_hist(long long *out)
{
    for (int k = 0; k < 2; ++k)
        for (int b = 0; b < DALPHA_BINS; ++b) out[k * DALPHA_BINS + b] = g_hist[k][b];
}
