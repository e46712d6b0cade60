// Accuracy of v_rcp_f64 / v_rsq_f64 (no refinement) against IEEE division, in ulp.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
__global__ void k(const double *x, double *r, double *q, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { r[i] = __builtin_amdgcn_rcp(x[i]); q[i] = 1.0 / x[i]; }
}
int main()
{
    const int n = 1 << 20;
    double *hx = (double *)malloc(n * 8), *hr = (double *)malloc(n * 8), *hq = (double *)malloc(n * 8);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        hx[i] = ldexp(1.0 + (s >> 11) * (1.0 / 9007199254740992.0), (int)(s % 40) - 20);
    }
    double *dx, *dr, *dq;
    hipMalloc(&dx, n * 8); hipMalloc(&dr, n * 8); hipMalloc(&dq, n * 8);
    hipMemcpy(dx, hx, n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dr, dq, n);
    hipMemcpy(hr, dr, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hq, dq, n * 8, hipMemcpyDeviceToHost);
    double mx = 0; long bad = 0;
    for (int i = 0; i < n; ++i) {
        double u = fabs(hr[i] - hq[i]) / (nextafter(fabs(hq[i]), INFINITY) - fabs(hq[i]));
        if (u > mx) mx = u;
        if (u > 0) ++bad;
    }
    printf("v_rcp_f64 vs IEEE 1/x: max %.3g ulp, %ld of %d differ\n", mx, bad, n);
    return 0;
}
