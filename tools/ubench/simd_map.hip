// Which SIMD each wave of a 512-lane workgroup lands on (HW_ID register), with 160 KB of LDS per
// workgroup (one workgroup per CU, as k_step_split).  Prints, for wave w of the workgroup, the
// SIMD ids seen over all workgroups.  Diagnostic for the configs[4] split.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(512) void k_map(unsigned *out)
{
    __shared__ double pad[20000];                   // 160 000 B: one workgroup per CU
    pad[threadIdx.x] = (double)threadIdx.x;
    __syncthreads();
    const unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = hw + (pad[threadIdx.x + 1] > 1e30 ? 1u : 0u);
}

int main()
{
    const int wg = 1024;
    unsigned *d, h[wg * 8];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    hipLaunchKernelGGL(k_map, dim3(wg), dim3(512), 0, 0, d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int same_as_w4[4] = {0, 0, 0, 0}, same_as_w1[4] = {0, 0, 0, 0};
    int hist[8][4] = {};
    for (int b = 0; b < wg; ++b) {
        unsigned simd[8];
        for (int w = 0; w < 8; ++w) { simd[w] = (h[b * 8 + w] >> 4) & 3u; hist[w][simd[w]]++; }
        for (int w = 0; w < 4; ++w) {
            same_as_w4[w] += simd[w] == simd[w + 4];
            same_as_w1[w] += simd[2 * (w / 2) + (w & 1)] == simd[2 * (w / 2) + 1 - (w & 1)];
        }
    }
    printf("{\"workgroups\": %d, \"pairs_w_w+4_same_simd\": [%d, %d, %d, %d], \"pairs_2k_2k+1_same_simd\": [%d, %d, %d, %d], \"simd_hist_per_wave\": [",
           wg, same_as_w4[0], same_as_w4[1], same_as_w4[2], same_as_w4[3], same_as_w1[0], same_as_w1[1], same_as_w1[2], same_as_w1[3]);
    for (int w = 0; w < 8; ++w) printf("%s[%d, %d, %d, %d]", w ? ", " : "", hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    printf("]}\n");
    hipFree(d);
    return 0;
}
