// traffic_probe.hip -- calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// shapes k_step issues (bench.py roofline.traffic; MI355X_MICROARCH.md HBM section: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Every kernel below moves a KNOWN number of bytes; run under rocprofv3 --pmc FETCH_SIZE (and a
// separate WRITE_SIZE pass) and divide:
//   k_rows_cold    k_step's input rows at 65 536 envs, loaded with k_step's per-lane code shape
//                  (system i32, joints 6 x f32, actions 6 x f32, t i32, desired goal 3 x f64,
//                  epoch i32: 84 B/env), after a 1 GiB sweep evicted L2 and the Infinity Cache;
//                  writes one i32 per env
//   k_rows_warm    the same loads right after k_rows_write rewrote the state rows (joints, t,
//                  goal), as the previous step's k_step does: the rows sit dirty in each XCD's L2
//   k_stream_cold  the same byte count as 16-B/lane streaming loads (the guide's x2 case)
//   k_rows_write   k_step's output rows at 65 536 envs with its store shape (joints 6 x f32,
//                  achieved goal 3 x f64, t i32, obs 13 x f32, reward f32, done u8, success u8,
//                  error f32, status u32: 118 B/env) plus the state rows the next step reads
//                  (joints, t, desired goal: 52 B/env), 170 B/env: the WRITE_SIZE reference
// Build: hipcc -O3 --offload-arch=gfx950 tools/traffic_probe.hip -o tools/traffic_probe
// Run:   rocprofv3 --pmc FETCH_SIZE -- ./tools/traffic_probe   (then WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

constexpr int BLOCK = 256;
constexpr int64_t N = 65536;

struct Rows {
    int32_t *system, *t, *epoch;
    float *joints, *actions;
    double *dg;
};

__device__ __forceinline__ int32_t load_rows(const Rows &r, int64_t e)
{
    // k_step (csrc/ctr_kernels.hip step_body / step_finish): one lane per env, scalar loads
    float q[6], a[6];
    const int s = r.system[e];
    #pragma unroll
    for (int i = 0; i < 6; ++i) { q[i] = r.joints[6 * e + i]; a[i] = r.actions[6 * e + i]; }
    const int32_t t = r.t[e];
    double dg[3];
    #pragma unroll
    for (int i = 0; i < 3; ++i) dg[i] = r.dg[3 * e + i];
    const uint32_t ep = (uint32_t)r.epoch[e];
    float acc = 0.f;
    #pragma unroll
    for (int i = 0; i < 6; ++i) acc += q[i] * a[i];
    return (int32_t)(acc * 7.0f) ^ s ^ t ^ (int32_t)ep ^ (int32_t)(dg[0] + dg[1] + dg[2]);
}

__global__ __launch_bounds__(BLOCK) void k_rows_cold(Rows r, int32_t *sink)
{
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e < N) sink[e] = load_rows(r, e);
}

__global__ __launch_bounds__(BLOCK) void k_rows_warm(Rows r, int32_t *sink)
{
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e < N) sink[e] = load_rows(r, e);
}

// the same 84 B/env as whole 16-B loads (5 x 16 B + 4 B per env, laid out flat)
__global__ __launch_bounds__(BLOCK) void k_stream_cold(const int4 *src, int64_t n16, int32_t *sink)
{
    int32_t acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n16; i += (int64_t)gridDim.x * BLOCK) {
        const int4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink[(int64_t)blockIdx.x * BLOCK + threadIdx.x] = acc;
}

struct Outs {
    float *joints, *obs, *reward, *error;
    double *ag;
    int32_t *t;
    uint8_t *done, *success;
    uint32_t *status;
};

__global__ __launch_bounds__(BLOCK) void k_rows_write(Outs o, Rows r, float v)
{
    const int64_t e = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (e >= N) return;
    #pragma unroll
    for (int i = 0; i < 6; ++i) o.joints[6 * e + i] = v + i;
    #pragma unroll
    for (int i = 0; i < 3; ++i) o.ag[3 * e + i] = (double)v * i;
    o.t[e] = (int32_t)e;
    #pragma unroll
    for (int k = 0; k < 13; ++k) o.obs[13 * e + k] = v * k;
    o.reward[e] = -1.f;
    o.done[e] = 0;
    o.success[e] = 1;
    o.error[e] = v;
    o.status[e] = 0;
    // the state rows the next "step" reads (the previous k_step writes them)
    #pragma unroll
    for (int i = 0; i < 6; ++i) r.joints[6 * e + i] = v - i;
    r.t[e] = (int32_t)e + 1;
    #pragma unroll
    for (int i = 0; i < 3; ++i) r.dg[3 * e + i] = (double)v + i;
}

__global__ __launch_bounds__(BLOCK) void k_flush(int4 *buf, int64_t n16, int32_t salt)
{
    for (int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x; i < n16; i += (int64_t)gridDim.x * BLOCK)
        buf[i] = make_int4(salt, (int)i, salt, (int)i);
}

int main()
{
    Rows r;
    Outs o;
    int32_t *sink;
    int4 *flat, *flush;
    const int64_t flush16 = (int64_t)1 << 26;            // 1 GiB of 16-B lines
    const int64_t flat16 = N * 84 / 16;                   // 84 B/env as 16-B loads
    CHECK(hipMalloc(&r.system, N * 4));
    CHECK(hipMalloc(&r.t, N * 4));
    CHECK(hipMalloc(&r.epoch, N * 4));
    CHECK(hipMalloc(&r.joints, N * 24));
    CHECK(hipMalloc(&r.actions, N * 24));
    CHECK(hipMalloc(&r.dg, N * 24));
    CHECK(hipMalloc(&o.joints, N * 24));
    CHECK(hipMalloc(&o.obs, N * 52));
    CHECK(hipMalloc(&o.reward, N * 4));
    CHECK(hipMalloc(&o.error, N * 4));
    CHECK(hipMalloc(&o.ag, N * 24));
    CHECK(hipMalloc(&o.t, N * 4));
    CHECK(hipMalloc(&o.done, N));
    CHECK(hipMalloc(&o.success, N));
    CHECK(hipMalloc(&o.status, N * 4));
    CHECK(hipMalloc(&sink, N * 4 * 4));
    CHECK(hipMalloc(&flat, flat16 * 16));
    CHECK(hipMalloc(&flush, flush16 * 16));
    CHECK(hipMemset(r.system, 0, N * 4));
    CHECK(hipMemset(r.epoch, 0, N * 4));
    CHECK(hipMemset(r.actions, 0, N * 24));
    CHECK(hipMemset(flat, 1, flat16 * 16));
    const dim3 grid((unsigned)(N / BLOCK));
    for (int it = 0; it < 5; ++it) {
        hipLaunchKernelGGL(k_flush, dim3(4096), dim3(BLOCK), 0, 0, flush, flush16, it);
        hipLaunchKernelGGL(k_rows_cold, grid, dim3(BLOCK), 0, 0, r, sink);
        hipLaunchKernelGGL(k_flush, dim3(4096), dim3(BLOCK), 0, 0, flush, flush16, it + 100);
        hipLaunchKernelGGL(k_stream_cold, grid, dim3(BLOCK), 0, 0, flat, flat16, sink);
        hipLaunchKernelGGL(k_flush, dim3(4096), dim3(BLOCK), 0, 0, flush, flush16, it + 200);
        hipLaunchKernelGGL(k_rows_write, grid, dim3(BLOCK), 0, 0, o, r, (float)it);
        hipLaunchKernelGGL(k_rows_warm, grid, dim3(BLOCK), 0, 0, r, sink);
    }
    CHECK(hipDeviceSynchronize());
    printf("{\"envs\": %lld, \"read_bytes_known\": %lld, \"stream_bytes_known\": %lld, \"write_bytes_known\": %lld, "
           "\"sink_bytes\": %lld}\n",
           (long long)N, (long long)(N * 84), (long long)(flat16 * 16), (long long)(N * 170), (long long)(N * 4));
    return 0;
}
