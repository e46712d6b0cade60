// f64 FMA issue vs latency for one wave per SIMD: C independent chains, N dependent FMAs each.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define N 512
template <int C>
__global__ __launch_bounds__(256) void kern(double *out, unsigned long long *cyc, double seed)
{
    double v[C];
    #pragma unroll
    for (int c = 0; c < C; ++c) v[c] = seed + threadIdx.x * 1e-3 + c;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        #pragma unroll
        for (int c = 0; c < C; ++c) v[c] = fma(v[c], 1.0000001, 1e-9);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    #pragma unroll
    for (int c = 0; c < C; ++c) s += v[c];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int C>
void run(double *out, unsigned long long *cyc)
{
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(kern<C>, dim3(256), dim3(256), 0, 0, out, cyc, 1.5);
    (void)hipDeviceSynchronize();
    unsigned long long h[256];
    (void)hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += h[i];
    m /= 256;
    printf("chains %2d: %6.2f cycles per FMA (per wave), %6.2f cycles per chain step\n", C, m / (C * N), m / N);
}
int main()
{
    double *out; unsigned long long *cyc;
    (void)hipMalloc(&out, 256 * 256 * 8); (void)hipMalloc(&cyc, 256 * 8);
    run<1>(out, cyc); run<2>(out, cyc); run<4>(out, cyc); run<8>(out, cyc); run<16>(out, cyc);
    return 0;
}
