// Micro-benchmark: per-instruction issue cost of fp64 operations for ONE wave per SIMD
// (the k_step regime).  Each lane runs 4 independent chains of an op, N iterations; cycles via
// s_memtime.  Prints cycles per op per wave (throughput with 4-way ILP).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../gym-ctr-reach_amd/csrc/ctr_math.hpp"

#define N 256
template <int OP>
__global__ __launch_bounds__(256) void kern(double *out, unsigned long long *cyc, double seed)
{
    double a = seed + threadIdx.x * 1e-3, b = a + 0.1, c = a + 0.2, d = a + 0.3;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    #pragma unroll 4
    for (int i = 0; i < N; ++i) {
        if (OP == 0) { a = fma(a, 1.0000001, 1e-9); b = fma(b, 1.0000001, 1e-9); c = fma(c, 1.0000001, 1e-9); d = fma(d, 1.0000001, 1e-9); }
        if (OP == 1) { a = __builtin_amdgcn_rcp(a) + 0.5; b = __builtin_amdgcn_rcp(b) + 0.5; c = __builtin_amdgcn_rcp(c) + 0.5; d = __builtin_amdgcn_rcp(d) + 0.5; }
        if (OP == 2) { a = sqrt(a) + 0.5; b = sqrt(b) + 0.5; c = sqrt(c) + 0.5; d = sqrt(d) + 0.5; }
        if (OP == 3) { a = 1.0 / a + 0.5; b = 1.0 / b + 0.5; c = 1.0 / c + 0.5; d = 1.0 / d + 0.5; }
        if (OP == 4) { a = exp2(-a) + 0.5; b = exp2(-b) + 0.5; c = exp2(-c) + 0.5; d = exp2(-d) + 0.5; }
        if (OP == 5) { a = log2(a) + 1.5; b = log2(b) + 1.5; c = log2(c) + 1.5; d = log2(d) + 1.5; }
        if (OP == 6) { a = pow(a, -0.2) + 0.5; b = pow(b, -0.2) + 0.5; c = pow(c, -0.2) + 0.5; d = pow(d, -0.2) + 0.5; }
        if (OP == 7) { double s, co; ctr_math::sincos_fast(a, s, co); a = s + co; ctr_math::sincos_fast(b, s, co); b = s + co;
                       ctr_math::sincos_fast(c, s, co); c = s + co; ctr_math::sincos_fast(d, s, co); d = s + co; }
        if (OP == 8) { a = ctr_math::rcp1(a) + 0.5; b = ctr_math::rcp1(b) + 0.5; c = ctr_math::rcp1(c) + 0.5; d = ctr_math::rcp1(d) + 0.5; }
        if (OP == 9) { a = ctr_math::powpos(a, -0.2) + 0.5; b = ctr_math::powpos(b, -0.2) + 0.5; c = ctr_math::powpos(c, -0.2) + 0.5; d = ctr_math::powpos(d, -0.2) + 0.5; }
        if (OP == 10) { a = __builtin_amdgcn_rsq(a) + 0.5; b = __builtin_amdgcn_rsq(b) + 0.5; c = __builtin_amdgcn_rsq(c) + 0.5; d = __builtin_amdgcn_rsq(d) + 0.5; }
        if (OP == 12) { a = rint(a) + 0.37; b = rint(b) + 0.37; c = rint(c) + 0.37; d = rint(d) + 0.37; }
        if (OP == 13) { a = (double)(int)a + 0.37; b = (double)(int)b + 0.37; c = (double)(int)c + 0.37; d = (double)(int)d + 0.37; }
        if (OP == 14) { a = (double)(float)a + 0.37; b = (double)(float)b + 0.37; c = (double)(float)c + 0.37; d = (double)(float)d + 0.37; }
        if (OP == 15) { a = fmax(a, 0.3) + 0.37; b = fmax(b, 0.3) + 0.37; c = fmax(c, 0.3) + 0.37; d = fmax(d, 0.3) + 0.37; }
        if (OP == 16) { a = (a + 6755399441055744.0) - 6755399441055744.0 + 0.37; b = (b + 6755399441055744.0) - 6755399441055744.0 + 0.37;
                        c = (c + 6755399441055744.0) - 6755399441055744.0 + 0.37; d = (d + 6755399441055744.0) - 6755399441055744.0 + 0.37; }
        if (OP == 11) { a = (double)__builtin_amdgcn_rcpf((float)a) + 0.5; b = (double)__builtin_amdgcn_rcpf((float)b) + 0.5; c = (double)__builtin_amdgcn_rcpf((float)c) + 0.5; d = (double)__builtin_amdgcn_rcpf((float)d) + 0.5; }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 256 + threadIdx.x] = a + b + c + d;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char *name, double *out, unsigned long long *cyc)
{
    hipLaunchKernelGGL(kern<OP>, dim3(256), dim3(256), 0, 0, out, cyc, 1.5);
    hipLaunchKernelGGL(kern<OP>, dim3(256), dim3(256), 0, 0, out, cyc, 1.5);
    hipDeviceSynchronize();
    unsigned long long h[256];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += h[i];
    m /= 256;
    printf("%-28s %7.1f cycles per op per wave (4 independent chains)\n", name, m / (4.0 * N));
}

int main()
{
    double *out;
    unsigned long long *cyc;
    hipMalloc(&out, 256 * 256 * sizeof(double));
    hipMalloc(&cyc, 256 * sizeof(unsigned long long));
    run<0>("v_fma_f64", out, cyc);
    run<12>("v_rndne_f64 (+add)", out, cyc);
    run<13>("cvt f64->i32->f64 (+add)", out, cyc);
    run<14>("cvt f64->f32->f64 (+add)", out, cyc);
    run<15>("v_max_f64 (+add)", out, cyc);
    run<16>("2 adds (magic round) (+add)", out, cyc);
    run<1>("v_rcp_f64 (+add)", out, cyc);
    run<8>("rcp1 (rcp+2fma)(+add)", out, cyc);
    run<11>("f32 rcp via cvt (+add)", out, cyc);
    run<10>("v_rsq_f64 (+add)", out, cyc);
    run<2>("sqrt f64 (+add)", out, cyc);
    run<3>("IEEE div f64 (+add)", out, cyc);
    run<4>("exp2 f64 ocml (+add)", out, cyc);
    run<5>("log2 f64 ocml (+add)", out, cyc);
    run<6>("pow f64 ocml (+add)", out, cyc);
    run<9>("exp2(y*log2 x) (+add)", out, cyc);
    run<7>("sincos_fast (+add)", out, cyc);
    return 0;
}
