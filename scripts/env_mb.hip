// Micro-benchmark of k_env0's per-frame instruction mix (csrc/amx_dyn.hip env0_tile):
// which instruction class stops a CU from stepping more envelope frames when it holds
// more waves.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/env_mb.hip -o /tmp/env_mb && /tmp/env_mb
//
// One workgroup per CU (dynamic LDS pins it), WG = 1 / 2 / 4 / 8 waves, every lane one
// segment stepping NT 16-frame tiles; each wave stamps s_memtime around its loop.
// MODE bits select what a tile does:
//   G  the m gathers from the 3 x 32769 table (else m = r * 1e-3: one cvt + mul)
//   L  k_env0's cooperative staging (4 lanes per row load r, gather, ds_write, each lane
//      ds_reads its own row); else each lane loads its own row's 32 B and gathers its 16 m
//   C  the two Markstein quotients + the exact step per frame (else att += m)
//   S  the checkpoint store per tile
//   Q  the any-over-threshold OR per tile
// Reported: cycles per wave-frame (median over waves) and CU frame-steps per kcycle.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define TAB 32769
#define MP 18
#define PF 8
enum { G = 1, L = 2, C = 4, S = 8, Q = 16 };

typedef double d2v __attribute__((ext_vector_type(2)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double min_raw(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double qdiv(double m, double a, double ra) {
    const double q = m * ra;
    return fma(fma(-q, a, m), ra, q);
}

template <int MODE>
__device__ __forceinline__ void mval(const double *__restrict__ mt, uint32_t r, double &m) {
    if constexpr (MODE & G) m = mt[r];
    else m = (double)r * 1e-3;
}

template <int MODE>
__global__ void mb(const uint16_t *__restrict__ rr, const double *__restrict__ mt, double *__restrict__ ck,
                   double *__restrict__ out, long long *__restrict__ cyc, int ntile, int rowlen,
                   double A, double rA, double R, double rR) {
    extern __shared__ __attribute__((aligned(16))) double dyn[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int nw = blockDim.x >> 6;
    double *sm = dyn + wv * 64 * MP;
    const int j = (blockIdx.x * nw + wv) * 64 + lane;
    const uint16_t *row = rr + (size_t)j * rowlen;
    double *ckr = ck + (size_t)j * (rowlen / 16);
    const uint16_t *irow[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int rw = 16 * i + (lane >> 2);
        irow[i] = rr + (size_t)((blockIdx.x * nw + wv) * 64 + rw) * rowlen + 4 * (lane & 3);
    }
    double att = 0.0;
    bool any = false;
    const long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (MODE & L) {
        u2v I[PF][4];
#pragma unroll
        for (int u = 0; u < PF; u++)
#pragma unroll
            for (int i = 0; i < 4; i++) I[u][i] = *reinterpret_cast<const u2v *>(irow[i] + u * 16);
        double Gm[2][16];
        auto gather = [&](const u2v (&Ii)[4], double (&Gd)[16]) {
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int e = 0; e < 4; e++) mval<MODE>(mt, (Ii[i][e >> 1] >> (16 * (e & 1))) & 0xffffu, Gd[4 * i + e]);
        };
        gather(I[0], Gm[0]);
        gather(I[1], Gm[1]);
        for (int q0 = 0; q0 < ntile; q0 += PF) {
#pragma unroll
            for (int u = 0; u < PF; u++) {
                const int q = q0 + u;
                double (&Gc)[16] = Gm[u & 1];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    double *d = sm + ((lane >> 2) + 16 * i) * MP + 4 * (lane & 3);
                    *reinterpret_cast<d2v *>(d) = d2v{Gc[4 * i], Gc[4 * i + 1]};
                    *reinterpret_cast<d2v *>(d + 2) = d2v{Gc[4 * i + 2], Gc[4 * i + 3]};
                }
                __builtin_amdgcn_wave_barrier();
                const int qn = (q + PF < ntile ? q + PF : q) * 16;
#pragma unroll
                for (int i = 0; i < 4; i++) I[u][i] = *reinterpret_cast<const u2v *>(irow[i] + qn);
                gather(I[(u + 2) % PF], Gc);
                double mv[16];
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const d2v v = *reinterpret_cast<const d2v *>(sm + lane * MP + 2 * i);
                    mv[2 * i] = v.x;
                    mv[2 * i + 1] = v.y;
                }
                __builtin_amdgcn_wave_barrier();
                if constexpr (MODE & S) ckr[q] = att;
                if constexpr (MODE & Q) {
                    uint32_t h = 0, l = 0;
#pragma unroll
                    for (int f = 0; f < 16; f++) {
                        const unsigned long long x = (unsigned long long)__double_as_longlong(mv[f]);
                        h |= (uint32_t)(x >> 32);
                        l |= (uint32_t)x;
                    }
                    any |= ((h & 0x7fffffffu) | l) != 0u;
                }
                if constexpr (MODE & C) {
                    double iv[16], dv[16];
#pragma unroll
                    for (int f = 0; f < 16; f++) { iv[f] = qdiv(mv[f], A, rA); dv[f] = qdiv(mv[f], R, rR); }
#pragma unroll
                    for (int f = 0; f < 16; f++) {
                        const double up = min_raw(att + iv[f], mv[f]);
                        const double dn = fmax(att - dv[f], 0.0);
                        att = att <= mv[f] ? up : dn;
                    }
                } else {
#pragma unroll
                    for (int f = 0; f < 16; f++) att += mv[f];
                }
            }
        }
    } else {
        // own row: 2 x 16-B loads of r per tile, PF tiles ahead; 16 gathers a tile ahead
        u4v I[PF][2];
#pragma unroll
        for (int u = 0; u < PF; u++) {
            I[u][0] = *reinterpret_cast<const u4v *>(row + u * 16);
            I[u][1] = *reinterpret_cast<const u4v *>(row + u * 16 + 8);
        }
        double Gm[2][16];
        auto gather = [&](const u4v (&Ii)[2], double (&Gd)[16]) {
#pragma unroll
            for (int f = 0; f < 16; f++) mval<MODE>(mt, (Ii[f >> 3][(f >> 1) & 3] >> (16 * (f & 1))) & 0xffffu, Gd[f]);
        };
        gather(I[0], Gm[0]);
        for (int q0 = 0; q0 < ntile; q0 += PF) {
#pragma unroll
            for (int u = 0; u < PF; u++) {
                const int q = q0 + u;
                double mv[16];
#pragma unroll
                for (int f = 0; f < 16; f++) mv[f] = Gm[u & 1][f];
                gather(I[(u + 1) % PF], Gm[(u + 1) & 1]);
                const int qn = (q + PF < ntile ? q + PF : q) * 16;
                I[u][0] = *reinterpret_cast<const u4v *>(row + qn);
                I[u][1] = *reinterpret_cast<const u4v *>(row + qn + 8);
                if constexpr (MODE & S) ckr[q] = att;
                if constexpr (MODE & Q) {
                    uint32_t h = 0, l = 0;
#pragma unroll
                    for (int f = 0; f < 16; f++) {
                        const unsigned long long x = (unsigned long long)__double_as_longlong(mv[f]);
                        h |= (uint32_t)(x >> 32);
                        l |= (uint32_t)x;
                    }
                    any |= ((h & 0x7fffffffu) | l) != 0u;
                }
                if constexpr (MODE & C) {
                    double iv[16], dv[16];
#pragma unroll
                    for (int f = 0; f < 16; f++) { iv[f] = qdiv(mv[f], A, rA); dv[f] = qdiv(mv[f], R, rR); }
#pragma unroll
                    for (int f = 0; f < 16; f++) {
                        const double up = min_raw(att + iv[f], mv[f]);
                        const double dn = fmax(att - dv[f], 0.0);
                        att = att <= mv[f] ? up : dn;
                    }
                } else {
#pragma unroll
                    for (int f = 0; f < 16; f++) att += mv[f];
                }
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[j] = att + (any ? 1.0 : 0.0);
    if (lane == 0) cyc[blockIdx.x * nw + wv] = t1 - t0;
}

// compute only, no memory at all: m from an in-register walk (the step's own cost)
template <int CH>
__global__ void mb_comp(double *__restrict__ out, long long *__restrict__ cyc, int ntile, double A, double rA,
                        double R, double rR) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int j = (blockIdx.x * nw + wv) * 64 + lane;
    double att[CH], mm = 3.0 + lane * 1e-3;
    for (int c = 0; c < CH; c++) att[c] = c * 0.1;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int q = 0; q < ntile; q++) {
        double mv[16];
#pragma unroll
        for (int f = 0; f < 16; f++) { mv[f] = mm; mm = mm * 0.9999 + 1e-4; }
        double iv[16], dv[16];
#pragma unroll
        for (int f = 0; f < 16; f++) { iv[f] = qdiv(mv[f], A, rA); dv[f] = qdiv(mv[f], R, rR); }
#pragma unroll
        for (int f = 0; f < 16; f++) {
#pragma unroll
            for (int c = 0; c < CH; c++) {
                const double up = min_raw(att[c] + iv[f], mv[f]);
                const double dn = fmax(att[c] - dv[f], 0.0);
                att[c] = att[c] <= mv[f] ? up : dn;
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int c = 0; c < CH; c++) s += att[c];
    out[j] = s;
    if (lane == 0) cyc[blockIdx.x * nw + wv] = t1 - t0;
}

static double median(std::vector<long long> v) {
    std::sort(v.begin(), v.end());
    return (double)v[v.size() / 2];
}

int main() {
    const int NCU = 256, NT = 128, ROWLEN = NT * 16 + PF * 16 + 16;
    const int MAXW = 8;
    const size_t nseg = (size_t)NCU * MAXW * 64;
    std::vector<uint16_t> hr(nseg * ROWLEN);
    // slowly varying r (a 100 ms period) with +-16 noise, a different phase per row
    std::vector<double> wave(4800);
    for (int f = 0; f < 4800; f++) wave[f] = 14000.0 + 9000.0 * sin(f * 6.2831853 / 4800.0);
    uint32_t s = 12345;
    for (size_t j = 0; j < nseg; j++) {
        const int ph = (int)((j * 2371) % 4800);
        for (int f = 0; f < ROWLEN; f++) {
            s = s * 1664525u + 1013904223u;
            hr[j * ROWLEN + f] = (uint16_t)(wave[(f + ph) % 4800] + (double)(s >> 27));
        }
    }
    std::vector<double> ht(3 * TAB);
    for (int r = 0; r < TAB; r++) ht[r] = r < 6000 ? 0.0 : 0.75 * 20.0 * log10((double)r / 6000.0);
    uint16_t *dr;
    double *dt, *dck, *dout;
    long long *dc;
    hipMalloc(&dr, hr.size() * 2);
    hipMalloc(&dt, ht.size() * 8);
    hipMalloc(&dck, nseg * (ROWLEN / 16) * 8);
    hipMalloc(&dout, nseg * 8);
    hipMalloc(&dc, NCU * MAXW * 8);
    hipMemcpy(dr, hr.data(), hr.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dt, ht.data(), ht.size() * 8, hipMemcpyHostToDevice);
    const double A = 240.0, R = 2400.0;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const size_t lds = 100 * 1024;   // one workgroup per CU
    auto run = [&](const char *name, auto kern, int comp) {
        for (int wg : {1, 2, 4, 8}) {
            float best = 1e30f;
            std::vector<long long> hc(NCU * wg);
            for (int rep = 0; rep < 3; rep++) {
                hipEventRecord(e0);
                if (comp == 1) hipLaunchKernelGGL(mb_comp<1>, dim3(NCU), dim3(64 * wg), lds, 0, dout, dc, NT, A, 1.0 / A, R, 1.0 / R);
                else if (comp == 2) hipLaunchKernelGGL(mb_comp<2>, dim3(NCU), dim3(64 * wg), lds, 0, dout, dc, NT, A, 1.0 / A, R, 1.0 / R);
                else if (comp == 4) hipLaunchKernelGGL(mb_comp<4>, dim3(NCU), dim3(64 * wg), lds, 0, dout, dc, NT, A, 1.0 / A, R, 1.0 / R);
                else hipLaunchKernelGGL(kern, dim3(NCU), dim3(64 * wg), lds, 0, dr, dt, dck, dout, dc, NT, ROWLEN, A,
                                        1.0 / A, R, 1.0 / R);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                best = std::min(best, ms);
            }
            hipMemcpy(hc.data(), dc, hc.size() * 8, hipMemcpyDeviceToHost);
            const double cpf = median(hc) / (NT * 16.0);
            printf("%-22s WG=%d  %8.1f us  cyc/wave-frame %7.1f  CU cyc per wave-frame %6.1f\n", name, wg,
                   best * 1e3, cpf, cpf / wg);
        }
    };
    if (hipGetLastError() != hipSuccess) return 1;
    run("FULL  (G L C S Q)", mb<G | L | C | S | Q>, 0);
    run("no gathers", mb<L | C | S | Q>, 0);
    run("no compute", mb<G | L | S | Q>, 0);
    run("no store", mb<G | L | C | Q>, 0);
    run("no any-OR", mb<G | L | C | S>, 0);
    run("gathers+staging only", mb<G | L>, 0);
    run("staging only (no G)", mb<L>, 0);
    run("own-row FULL", mb<G | C | S | Q>, 0);
    run("own-row no gathers", mb<C | S | Q>, 0);
    run("own-row gathers only", mb<G>, 0);
    run("compute only (regs)", mb<0>, 1);
    run("compute only, 2 chains", mb<0>, 2);
    run("compute only, 4 chains", mb<0>, 4);
    hipError_t e = hipDeviceSynchronize();
    printf("status %s\n", hipGetErrorString(e));
    return e == hipSuccess ? 0 : 1;
}
