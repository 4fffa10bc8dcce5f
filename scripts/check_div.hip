// Checks that device double division m / A reproduces the host quotients bit for bit
// for the compressor tables (amx_dyn.hip derives inc = m/A, dec = m/R on the device).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
__global__ void kdiv(const double *m, int n, double A, double R, double *q1, double *q2) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { q1[i] = m[i] / A; q2[i] = m[i] / R; }
}
int main() {
    const int n = 32769;
    std::vector<double> m(n), h1(n), h2(n), d1(n), d2(n);
    int bad = 0;
    for (int fs : {44100, 48000, 96000}) {
        const double A = 5.0 * (fs / 1000.0), R = 50.0 * (fs / 1000.0);
        for (double thr_db : {-25.0, -20.0, -15.0}) {
            for (double ratio : {6.0, 3.0, 4.0}) {
                double thr = 32768.0 * std::pow(10.0, thr_db / 20.0), k = 1.0 - 1.0 / ratio;
                for (int r = 0; r < n; r++) {
                    double over = 0.0;
                    if (r) { double db = 20 * (std::log((double)r / thr) / std::log(10.0)); over = 0 > db ? 0.0 : db; }
                    m[r] = k * over; h1[r] = m[r] / A; h2[r] = m[r] / R;
                }
                double *dm, *a, *b;
                hipMalloc(&dm, n * 8); hipMalloc(&a, n * 8); hipMalloc(&b, n * 8);
                hipMemcpy(dm, m.data(), n * 8, hipMemcpyHostToDevice);
                hipLaunchKernelGGL(kdiv, dim3((n + 255) / 256), dim3(256), 0, 0, dm, n, A, R, a, b);
                hipMemcpy(d1.data(), a, n * 8, hipMemcpyDeviceToHost);
                hipMemcpy(d2.data(), b, n * 8, hipMemcpyDeviceToHost);
                for (int r = 0; r < n; r++) bad += (memcmp(&d1[r], &h1[r], 8) != 0) + (memcmp(&d2[r], &h2[r], 8) != 0);
                hipFree(dm); hipFree(a); hipFree(b);
            }
        }
    }
    printf("division mismatches: %d\n", bad);
    return bad != 0;
}
