// Stand-in for RCCL's all-gather kernel on one GPU (tools/gather_interference.py): workgroups
// with the device kernel's footprint (ncclDevKernel_Generic_* in librccl 7.2, gfx950: 256 VGPRs,
// 37.7 KB LDS, 256 lanes) that stay resident for a fixed number of shader-clock cycles, so the
// dispatch interplay with k_step (one 368-register wave per SIMD) can be timed without 8 GPUs.
// Build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/fake_gather.hip -o tools/libfake_gather.so
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void k_fake_gather(uint64_t cycles, int *sink)
{
    __shared__ int lds[37664 / 4];
    // pin the register footprint at 256 VGPRs, as the RCCL kernel's
    asm volatile("v_mov_b32 v255, 0" ::: "v255");
    lds[threadIdx.x] = (int)threadIdx.x;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    int acc = 0;
    while (__builtin_amdgcn_s_memtime() - t0 < cycles) acc += lds[(threadIdx.x + acc) & 255];
    if (acc == 0x7fffffff) sink[0] = acc;      // keeps the loop; never true in practice
}

extern "C" int fake_gather_launch(int blocks, uint64_t cycles, int *sink, void *stream)
{
    hipLaunchKernelGGL(k_fake_gather, dim3(blocks), dim3(256), 0, (hipStream_t)stream, cycles, sink);
    return (int)hipGetLastError();
}
