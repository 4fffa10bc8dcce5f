// Micro-benchmark: dependent-chain latency of fp64 ops on gfx950 (one wave per
// SIMD, one chain), to size the sequential envelope recursion of the compressor.
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench_latency.hip -o /tmp/ml && /tmp/ml
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain_fma(double *out, int iters, double a, double b) {
    double v = threadIdx.x * 1e-3;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) v = fma(v, a, b);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

__global__ void chain_add(double *out, int iters, double a, double b) {
    double v = threadIdx.x * 1e-3;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) v = v + a;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

// the compressor envelope step (pydub compress_dynamic_range), fed from registers
__global__ void chain_env(double *out, int iters, double m0, double inc0, double dec0) {
    double att = 0.0;
    double m = m0 + threadIdx.x * 1e-9, inc = inc0, dec = dec0;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const bool over = (k & 3) != 3;
            if (over && att <= m) {
                att = att + inc;
                att = (m < att) ? m : att;
            } else {
                att = att - dec;
                att = (0.0 > att) ? 0.0 : att;
            }
            m = m * 1.0000001;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = att;
}

__global__ void chain_int64(long long *out, int iters, long long a) {
    long long v = threadIdx.x;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) v = v * 3 + a;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

template <class F>
float timeit(F f) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipEventRecord(a);
    for (int r = 0; r < 5; r++) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    double *out;
    (void)hipMalloc(&out, sizeof(double) * 1024 * 256);
    const int iters = 4096;
    const double steps = (double)iters * 16;
    int clk_khz = 0;
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const double ghz = clk_khz / 1e6;
    auto rep = [&](const char *name, float ms) {
        const double ns = ms * 1e6 / steps;
        printf("%-16s %.3f ms  %.2f ns/step  ~%.1f cycles/step at %.2f GHz\n", name, ms, ns,
               ns * ghz, ghz);
    };
    // one wave per SIMD: 256 blocks x 256 threads = 4 waves per CU
    rep("fma chain", timeit([&] { hipLaunchKernelGGL(chain_fma, dim3(256), dim3(256), 0, 0, out, iters, 0.999, 1e-3); }));
    rep("add chain", timeit([&] { hipLaunchKernelGGL(chain_add, dim3(256), dim3(256), 0, 0, out, iters, 1e-3, 0.0); }));
    rep("env step chain", timeit([&] { hipLaunchKernelGGL(chain_env, dim3(256), dim3(256), 0, 0, out, iters, 10.0, 0.05, 0.005); }));
    rep("int64 mad chain", timeit([&] { hipLaunchKernelGGL(chain_int64, dim3(256), dim3(256), 0, 0, (long long *)out, iters, 7LL); }));
    (void)hipFree(out);
    return 0;
}
