// amx_scan.hip -- exact segment start states of a linear recurrence
//     s_{j+1} = M s_j + e_j        (M = A^L, e_j = zero-state end state of segment j)
// over the segments of each stream (a chunk for the EQ / crossover, a track span
// for the K filter), with s_first = carry (or rest).
//
// Two levels:
//   up    : per block of S consecutive segments, E_b = sum_q M^{n-1-q} e_q (Horner);
//   top   : Kogge-Stone over blocks with powers of Mb = A^{L*S}: block start states;
//   down  : per block, s_{q+1} = M s_q + e_q from the block start state.
// up/down run one lane group of GP >= D lanes per (block, channel): lane i owns row
// i of M in VGPRs and the D-vector is exchanged through LDS each step, so a step is
// D FMAs + D/2 broadcast LDS reads per lane.  Cost per segment: 2 D^2 FMAs per
// channel, independent of the scan depth (the single-level Kogge-Stone paid
// levels x D^2 and needed levels ~ log2(decay / L)).
#include "amx_dev.hpp"

namespace amx {

// ------------------------------------------------ up / down sweeps in a block
template <int D, int GP, bool DOWN>
__global__ void __launch_bounds__(AMX_BLOCK) k_scan_blk(const ScanBlk *__restrict__ blks,
                                                        int n_blk, const double *__restrict__ e,
                                                        double *__restrict__ s,
                                                        const double *__restrict__ M,
                                                        const double *__restrict__ bst,
                                                        double *__restrict__ eb) {
    static_assert(GP >= D && GP <= 64 && (64 % GP) == 0, "group must tile a wave");
    constexpr int GPB = AMX_BLOCK / GP;
    __shared__ double lds[AMX_BLOCK];
    const int t = threadIdx.x;
    const int gi = t / GP, i = t % GP;
    const int64_t g = (int64_t)blockIdx.x * GPB + gi;     // (block, channel) = 2 b + ch
    const bool gvalid = g < 2LL * n_blk;
    const int b = gvalid ? (int)(g >> 1) : 0;
    const int ch = (int)(g & 1);
    const ScanBlk bk = blks[b];
    const bool row = i < D;
    double mrow[D];
#pragma unroll
    for (int k = 0; k < D; k++) mrow[k] = row ? M[i * D + k] : 0.0;
    double v = 0.0;
    if (DOWN && gvalid && row) v = bst[((int64_t)b * 2 + ch) * D + i];
    const int n = gvalid && (DOWN || !bk.last) ? bk.nseg : 0;
    double *my = lds + gi * GP;
    for (int q = 0; q < n; q++) {
        const int64_t jj = (int64_t)bk.seg0 + q;
        if (DOWN) {
            if (row) s[(jj * 2 + ch) * D + i] = v;
            if (q == n - 1) break;                         // next block starts from `top`
        }
        const double ev = row ? e[(jj * 2 + ch) * D + i] : 0.0;
        my[i] = v;
        __builtin_amdgcn_wave_barrier();
        double acc = ev;
#pragma unroll
        for (int k = 0; k < D; k++) acc = fma(mrow[k], my[k], acc);
        __builtin_amdgcn_wave_barrier();
        v = acc;
    }
    if (!DOWN && n > 0 && row) eb[((int64_t)b * 2 + ch) * D + i] = v;
}

// ---------------------------------------------- Kogge-Stone over the blocks
// x_b = carry (b == first) or E_{b-1};   B_b = sum_{k<K} Mb^k x_{b-k}  (same stream).
// One workgroup = 256 consecutive blocks of one channel; the first K-1 are halo.
template <int D>
__global__ void __launch_bounds__(AMX_BLOCK) k_scan_top(const ScanBlk *__restrict__ blks,
                                                        int n_blk, const double *__restrict__ eb,
                                                        double *__restrict__ bst,
                                                        const double *__restrict__ Mp,
                                                        int levels,
                                                        const double *__restrict__ carry) {
    __shared__ double lds[AMX_BLOCK * D];
    const int K = 1 << levels;
    const int HALO = K - 1;
    const int OUT = blockDim.x - HALO;
    const int ch = blockIdx.y;
    const int t = threadIdx.x;
    const int64_t b = (int64_t)blockIdx.x * OUT - HALO + t;
    double v[D], nb[D];
    const bool in = b >= 0 && b < n_blk;
    int first = 0x7fffffff;
    ScanBlk bk{};
    if (in) {
        bk = blks[b];
        first = bk.first;
    }
#pragma unroll
    for (int d = 0; d < D; d++) {
        double x = 0.0;
        if (in) {
            if (b == first) x = carry ? carry[((int64_t)bk.stream * 2 + ch) * D + d] : 0.0;
            else x = eb[((b - 1) * 2 + ch) * D + d];
        }
        v[d] = x;
    }
    for (int l = 0; l < levels; l++) {
        const int off = 1 << l;
#pragma unroll
        for (int d = 0; d < D; d++) lds[t * D + d] = v[d];
        __syncthreads();
        const bool use = (t - off >= 0) && (b - off >= first) && in;
        if (use) {
#pragma unroll
            for (int d = 0; d < D; d++) nb[d] = lds[(t - off) * D + d];
        }
        __syncthreads();
        if (use) {
            const double *Ml = Mp + (int64_t)l * D * D;
#pragma unroll
            for (int r = 0; r < D; r++) {
                double acc = v[r];
#pragma unroll
                for (int k = 0; k < D; k++) acc = fma(Ml[r * D + k], nb[k], acc);
                v[r] = acc;
            }
        }
    }
    if (t >= HALO && in)
#pragma unroll
        for (int d = 0; d < D; d++) bst[(b * 2 + ch) * D + d] = v[d];
}

// ================================================================ launchers
template <int D, int GP>
static hipError_t scan_t(const ScanPlan &p, const double *e, double *s, const double *carry,
                         double *eb, double *bst, hipStream_t st) {
    constexpr int GPB = AMX_BLOCK / GP;
    const dim3 gb((unsigned)((2 * (int64_t)p.n_blk + GPB - 1) / GPB));
    hipLaunchKernelGGL((k_scan_blk<D, GP, false>), gb, dim3(AMX_BLOCK), 0, st, p.blks, p.n_blk, e,
                       s, p.M, bst, eb);
    const int K = 1 << p.levels;
    const int OUT = AMX_BLOCK - (K - 1);
    if (OUT <= 0) return hipErrorInvalidValue;
    dim3 gt((unsigned)((p.n_blk + OUT - 1) / OUT), 2);
    hipLaunchKernelGGL(k_scan_top<D>, gt, dim3(AMX_BLOCK), 0, st, p.blks, p.n_blk, eb, bst, p.Mbp,
                       p.levels, carry);
    hipLaunchKernelGGL((k_scan_blk<D, GP, true>), gb, dim3(AMX_BLOCK), 0, st, p.blks, p.n_blk, e,
                       s, p.M, bst, eb);
    return hipGetLastError();
}

hipError_t launch_scan(const ScanPlan &p, const double *e, double *s, const double *carry,
                       double *eb, double *bst, hipStream_t st) {
    if (p.n_blk <= 0 || p.D <= 0) return hipSuccess;
    switch (p.D) {
    case 2: return scan_t<2, 2>(p, e, s, carry, eb, bst, st);
    case 4: return scan_t<4, 4>(p, e, s, carry, eb, bst, st);
    case 8: return scan_t<8, 8>(p, e, s, carry, eb, bst, st);
    case 10: return scan_t<10, 16>(p, e, s, carry, eb, bst, st);
    case 12: return scan_t<12, 16>(p, e, s, carry, eb, bst, st);
    case 16: return scan_t<16, 16>(p, e, s, carry, eb, bst, st);
    case 18: return scan_t<18, 32>(p, e, s, carry, eb, bst, st);
    case 20: return scan_t<20, 32>(p, e, s, carry, eb, bst, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace amx
