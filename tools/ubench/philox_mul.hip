// Philox4x32-10 multiply forms on gfx950: 32-bit lo/hi multiplies vs one 32x32->64 product (v_mad_u64_u32)
// Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/philox_mul.hip -o tools/ubench/philox_mul
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
__device__ __forceinline__ void philox_a(uint32_t c[4], uint32_t k0, uint32_t k1) {
    #pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
        const uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
__device__ __forceinline__ void philox_b(uint32_t c[4], uint32_t k0, uint32_t k1) {
    #pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b) {
    uint64_t r;
    asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ void philox_c(uint32_t c[4], uint32_t k0, uint32_t k1) {
    #pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = mad64(0xD2511F53u, c[0]), p1 = mad64(0xCD9E8D57u, c[2]);
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
}
template <int V>
__global__ void kp(uint32_t *out, int iters, uint32_t k0, uint32_t k1) {
    uint32_t c[4] = {threadIdx.x, blockIdx.x, 7u, 9u};
    uint32_t d[4] = {threadIdx.x + 1, blockIdx.x, 7u, 9u};
    for (int i = 0; i < iters; ++i) {
        if (V == 0) { philox_a(c, k0, k1); philox_a(d, k0, k1); }
        else if (V == 1) { philox_b(c, k0, k1); philox_b(d, k0, k1); }
        else { philox_c(c, k0, k1); philox_c(d, k0, k1); }
        c[0] ^= d[1];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c[0] ^ c[1] ^ c[2] ^ c[3] ^ d[0] ^ d[3];
}
int main() {
    uint32_t *o; hipMalloc(&o, 1024 * 256 * 4);
    uint32_t *h = (uint32_t*)malloc(1024*256*4), *h0 = (uint32_t*)malloc(1024*256*4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int v = 0; v < 3; ++v) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(a);
            if (v == 0) kp<0><<<1024, 64>>>(o, 200, 1u, 2u);
            else if (v == 1) kp<1><<<1024, 64>>>(o, 200, 1u, 2u);
            else kp<2><<<1024, 64>>>(o, 200, 1u, 2u);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep == 2) printf("variant %d: %.1f us (%.1f ns per philox pair-round)\n", v, ms * 1e3, ms * 1e6 / (200 * 10));
        }
        hipMemcpy(v == 0 ? h0 : h, o, 1024*256*4 > 1024*64*4 ? 1024*64*4 : 0, hipMemcpyDeviceToHost);
        if (v > 0) printf("  equal to variant 0: %d\n", memcmp(h, h0, 1024*64*4) == 0);
    }
    return 0;
}
