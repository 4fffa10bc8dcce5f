// Micro-benchmark: fp64 FMA issue rate and dependent latency on gfx950, and the
// cost of a DF-II-T biquad chain, to calibrate the IIR kernels' roofline.
//   hipcc --offload-arch=gfx950 -O3 scripts/microbench_fp64.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CHAINS>
__global__ void fma_chains(double *out, int iters, double a, double b) {
    double v[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; c++) v[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) v[c] = fma(v[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) s += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// one biquad (5 FMA) per frame per thread, dependent across frames
__global__ void biquad(double *out, int iters, double b0, double b1, double b2, double a1,
                       double a2) {
    double z0 = 0, z1 = 0, x = threadIdx.x * 1e-3;
    double acc = 0;
    for (int i = 0; i < iters; i++) {
        double y = fma(b0, x, z0);
        z0 = fma(-a1, y, fma(b1, x, z1));
        z1 = fma(-a2, y, b2 * x);
        acc += y;
        x = x * 0.999 + 1e-6;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <class F>
float timeit(F f) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / 5;
}

int main() {
    double *out;
    const int blocks = 256 * 8, threads = 256;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    const int iters = 4096;
    auto rep = [&](const char *name, int chains, int wpb, float ms) {
        double fmas = (double)256 * wpb * threads * iters * chains;
        printf("%-28s blocks/CU=%d  %.3f ms  %.2f TFMA/s (%.1f TFLOP/s)\n", name, wpb, ms,
               fmas / ms / 1e9, 2 * fmas / ms / 1e9);
    };
    for (int bpc : {1, 2, 4, 8}) {
        int nb = 256 * bpc;
        float ms;
        ms = timeit([&] { hipLaunchKernelGGL(fma_chains<1>, dim3(nb), dim3(threads), 0, 0, out, iters, 0.999, 1e-3); });
        rep("1 chain", 1, bpc, ms);
        ms = timeit([&] { hipLaunchKernelGGL(fma_chains<4>, dim3(nb), dim3(threads), 0, 0, out, iters, 0.999, 1e-3); });
        rep("4 chains", 4, bpc, ms);
        ms = timeit([&] { hipLaunchKernelGGL(fma_chains<16>, dim3(nb), dim3(threads), 0, 0, out, iters, 0.999, 1e-3); });
        rep("16 chains", 16, bpc, ms);
        ms = timeit([&] { hipLaunchKernelGGL(biquad, dim3(nb), dim3(threads), 0, 0, out, iters, 0.1, 0.2, 0.1, -1.5, 0.6); });
        rep("biquad (5 FMA+2 op/frame)", 7, bpc, ms);
    }
    hipFree(out);
    return 0;
}
