// Host cost of one kernel launch vs the size of its by-value argument block (k_step passes
// KCfg + ctr_batch_t + ctr_step_out_t by value: ~2.4 KB).  Empty kernels, 4000 launches each on
// one stream, host time per hipLaunchKernelGGL call, then the device drain.
// Build: hipcc -O2 --offload-arch=gfx950 tools/ubench/launch_cost.hip -o tools/ubench/launch_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

template <int N>
struct Blob {
    unsigned char b[N];
};

template <int N>
__global__ void k_empty(Blob<N> arg, int *sink)
{
    if (arg.b[threadIdx.x % N] == 0xAB && threadIdx.x == 1000000) sink[0] = 1;
}

template <int N>
void run(hipStream_t s, int *sink)
{
    Blob<N> blob = {};
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k_empty<N>, dim3(256), dim3(256), 0, s, blob, sink);
    hipStreamSynchronize(s);
    const int K = 4000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < K; ++i) hipLaunchKernelGGL(k_empty<N>, dim3(256), dim3(256), 0, s, blob, sink);
    auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(s);
    auto t2 = std::chrono::steady_clock::now();
    printf("kernarg %5d B: host %.2f us/launch, host+drain %.2f us/launch\n", N + 8,
           std::chrono::duration<double, std::micro>(t1 - t0).count() / K,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / K);
}

int main()
{
    hipStream_t s;
    hipStreamCreate(&s);
    int *sink;
    hipMalloc(&sink, 4);
    run<8>(s, sink);
    run<24>(s, sink);
    run<56>(s, sink);
    run<120>(s, sink);
    run<184>(s, sink);
    run<248>(s, sink);
    run<256>(s, sink);
    run<512>(s, sink);
    run<1024>(s, sink);
    run<2048>(s, sink);
    run<2400>(s, sink);
    run<3072>(s, sink);
    run<4000>(s, sink);
    return 0;
}
