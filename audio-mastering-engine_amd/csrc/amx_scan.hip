// amx_scan.hip -- exact segment start states of a linear recurrence
//     s_{j+1} = M s_j + e_j        (M = A^L, e_j = zero-state end state of segment j)
// over the segments of each stream (a chunk for the EQ / crossover, a track span
// for the K filter), with s_first = carry (or rest).
//
// Two levels:
//   up    : per block of S consecutive segments, E_b = sum_q M^{n-1-q} e_q (Horner);
//   down  : block start state B_b = sum_{k<K} Mb^k x_{b-k} (x_b = E_{b-1}, or the
//           carry at the stream's first block; Mb = A^{L*S}, K = the first power
//           with ||Mb^K|| <= 1e-22, so the window is exact to rounding), then
//           s_{q+1} = M s_q + e_q through the block.
// up/down run one lane group of GP >= D lanes per (block, channel): lane i owns row
// i of M in VGPRs and the D-vector is exchanged through LDS each step, so a step is
// D FMAs + D/2 broadcast LDS reads per lane.  Cost per segment: 2 D^2 FMAs per
// channel, independent of the scan depth (the single-level Kogge-Stone paid
// levels x D^2 and needed levels ~ log2(decay / L)).
#include "amx_dev.hpp"

namespace amx {

typedef double d2s __attribute__((ext_vector_type(2)));

// ------------------------------------------------ up / down sweeps in a block
template <int D, int GP, bool DOWN>
__global__ void __launch_bounds__(AMX_BLOCK) k_scan_blk(const ScanBlk *__restrict__ blks,
                                                        int n_blk, const double *__restrict__ e,
                                                        double *__restrict__ s,
                                                        const double *__restrict__ M,
                                                        const double *__restrict__ Mbk, int K,
                                                        const double *__restrict__ carry,
                                                        double *__restrict__ eb,
                                                        const double *__restrict__ tailP,
                                                        double *__restrict__ tail) {
    // GW groups of GP lanes in each wave (a group never straddles waves, so wave
    // barriers order its LDS exchange); lanes past GW GP are idle.  GP = D packs the
    // groups: D = 20 -> 3 groups per wave (60 lanes) instead of 2 of 32.
    static_assert(GP >= D && GP <= 64, "group fits a wave");
    constexpr int GW = 64 / GP;
    constexpr int GPB = GW * (AMX_BLOCK / 64);
    __shared__ __attribute__((aligned(16))) double lds[AMX_BLOCK];
    // the window's block powers Mb^k (k = 1 .. K - 1, (K - 1) D^2 doubles), staged in LDS
    // once per workgroup: read from memory inside the window loop they put a load's
    // latency on each of its K - 1 dependent steps (C5: K = 6)
    __shared__ __attribute__((aligned(16))) double s_pow[DOWN ? AMX_SCAN_PW * D * D : 1];
    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    if constexpr (DOWN) {
        const int np = (K - 1 < AMX_SCAN_PW ? K - 1 : AMX_SCAN_PW) * D * D;
        for (int k = t; k < np; k += AMX_BLOCK) s_pow[k] = Mbk[k];
        __syncthreads();
    }
    const int gl = l / GP, i = l % GP;
    const bool lane_ok = gl < GW;
    const int64_t g = (int64_t)blockIdx.x * GPB + w * GW + (lane_ok ? gl : 0);   // (block, channel) = 2 b + ch
    const bool gvalid = lane_ok && g < 2LL * n_blk;
    const int b = gvalid ? (int)(g >> 1) : 0;
    const int ch = (int)(g & 1);
    const ScanBlk bk = blks[b];
    const bool row = lane_ok && i < D;
    const int ri = row ? i : 0;
    double mrow[D];
#pragma unroll
    for (int k = 0; k < D; k++) mrow[k] = row ? M[i * D + k] : 0.0;
    const int n = gvalid && (DOWN || !bk.last) ? bk.nseg : 0;
    // all of the block's e rows are loaded up front (clamped, unconditional): a load
    // per step would put one HBM round trip on every step of the sequential chain
    double ev[AMX_SCAN_S];
#pragma unroll
    for (int q = 0; q < AMX_SCAN_S; q++) {
        const int qq = q < n ? q : 0;
        const int64_t jj = (int64_t)bk.seg0 + qq;
        ev[q] = e[(jj * 2 + ch) * D + ri];
    }
    // an idle lane reads group 0's vector (discarded) and writes nothing
    double *my = lds + w * 64 + (lane_ok ? gl * GP : 0);
    double v = 0.0;
    if constexpr (DOWN) {
        // block start state: windowed sum over the previous K blocks of the stream
        auto xin = [&](int bb) -> double {      // x_bb, component ri
            if (bb == bk.first)
                return carry ? carry[((int64_t)bk.stream * 2 + ch) * D + ri] : 0.0;
            return eb[((int64_t)(bb - 1) * 2 + ch) * D + ri];
        };
        v = (gvalid && row) ? xin(b) : 0.0;
        // the window's inputs, loaded before its chain
        double xs[AMX_SCAN_PW + 1];
#pragma unroll
        for (int k = 1; k <= AMX_SCAN_PW; k++) {
            const int bb = b - k;
            xs[k] = (k < K && gvalid && bb >= bk.first && row) ? xin(bb) : 0.0;
        }
        for (int k = 1; k < K; k++) {
            const int bb = b - k;
            const bool ok = gvalid && bb >= bk.first;
            double xk = 0.0;
#pragma unroll
            for (int q = 1; q <= AMX_SCAN_PW; q++) xk = q == k ? xs[q] : xk;
            if (lane_ok) my[i] = k <= AMX_SCAN_PW ? xk : ((ok && row) ? xin(bb) : 0.0);
            __builtin_amdgcn_wave_barrier();
            const double *P = (k <= AMX_SCAN_PW ? s_pow : Mbk) + ((int64_t)(k - 1) * D + ri) * D;
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int m = 0; m < D; m += 2) {
                a0 = fma(P[m], my[m], a0);
                if (m + 1 < D) a1 = fma(P[m + 1], my[m + 1], a1);
            }
            __builtin_amdgcn_wave_barrier();
            if (ok && row) v += a0 + a1;
        }
    }
#pragma unroll
    for (int q = 0; q < AMX_SCAN_S; q++) {
        if (q >= n) break;
        if (DOWN) {
            const int64_t jj = (int64_t)bk.seg0 + q;
            if (row) s[(jj * 2 + ch) * D + i] = v;
            if (q == n - 1) {                              // the next block has its own B
                if constexpr (D == AMX_KW_DIM) {
                    // the stream's end state from these start states (k_kw_tail's
                    // product, same order): P_t s_last + e_last, by the last block
                    if (tail && bk.last) {
                        if (lane_ok) my[i] = v;
                        __builtin_amdgcn_wave_barrier();
                        double acc = 0.0;
#pragma unroll
                        for (int qq = 0; qq < AMX_SCAN_S; qq++) acc = qq == q ? ev[qq] : acc;
                        const double *Pt = tailP + (int64_t)bk.stream * 16;
#pragma unroll
                        for (int k = 0; k < D; k++) acc = fma(Pt[ri * 4 + k], my[k], acc);
                        if (row) tail[((int64_t)bk.stream * 2 + ch) * D + i] = acc;
                        __builtin_amdgcn_wave_barrier();
                    }
                }
                break;
            }
        }
        if (lane_ok) my[i] = v;
        __builtin_amdgcn_wave_barrier();
        // four partial sums: the dependent fp64 FMA latency (~30 cycles) would
        // otherwise serialise D FMAs per step
        // the vector is read as 16-B pairs (D even): half the LDS instructions
        double a0 = row ? ev[q] : 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
        double mv[D];
#pragma unroll
        for (int k = 0; k < D; k += 2) {
            if (k + 1 < D) {
                const d2s pr = *reinterpret_cast<const d2s *>(my + k);
                mv[k] = pr.x;
                mv[k + 1] = pr.y;
            } else {
                mv[k] = my[k];
            }
        }
#pragma unroll
        for (int k = 0; k < D; k += 4) {
            a0 = fma(mrow[k], mv[k], a0);
            if (k + 1 < D) a1 = fma(mrow[k + 1], mv[k + 1], a1);
            if (k + 2 < D) a2 = fma(mrow[k + 2], mv[k + 2], a2);
            if (k + 3 < D) a3 = fma(mrow[k + 3], mv[k + 3], a3);
        }
        __builtin_amdgcn_wave_barrier();
        v = (a0 + a1) + (a2 + a3);
    }
    if (!DOWN && n > 0 && row) eb[((int64_t)b * 2 + ch) * D + i] = v;
}

// ================================================================ launchers
template <int D, int GP>
static hipError_t scan_t(const ScanPlan &p, const double *e, double *s, const double *carry,
                         double *eb, bool up, const double *tailP, double *tail, hipStream_t st) {
    constexpr int GPB = (64 / GP) * (AMX_BLOCK / 64);
    const dim3 gb((unsigned)((2 * (int64_t)p.n_blk + GPB - 1) / GPB));
    if (up)
        hipLaunchKernelGGL((k_scan_blk<D, GP, false>), gb, dim3(AMX_BLOCK), 0, st, p.blks, p.n_blk, e,
                           s, p.M, p.Mbk, p.K, carry, eb, nullptr, nullptr);
    hipLaunchKernelGGL((k_scan_blk<D, GP, true>), gb, dim3(AMX_BLOCK), 0, st, p.blks, p.n_blk, e,
                       s, p.M, p.Mbk, p.K, carry, eb, tailP, tail);
    return hipGetLastError();
}

// up false: eb already holds the up sweep of these e (the block sums do not depend on
// the carry), only the down sweep runs
hipError_t launch_scan(const ScanPlan &p, const double *e, double *s, const double *carry,
                       double *eb, hipStream_t st, bool up, const double *tailP, double *tail) {
    if (p.n_blk <= 0 || p.D <= 0) return hipSuccess;
    if (tail && p.D != AMX_KW_DIM) return hipErrorInvalidValue;
    switch (p.D) {
    case 2: return scan_t<2, 2>(p, e, s, carry, eb, up, tailP, tail, st);
    case 4: return scan_t<4, 4>(p, e, s, carry, eb, up, tailP, tail, st);
    case 8: return scan_t<8, 8>(p, e, s, carry, eb, up, tailP, tail, st);
    case 10: return scan_t<10, 10>(p, e, s, carry, eb, up, tailP, tail, st);
    case 12: return scan_t<12, 12>(p, e, s, carry, eb, up, tailP, tail, st);
    case 16: return scan_t<16, 16>(p, e, s, carry, eb, up, tailP, tail, st);
    case 18: return scan_t<18, 18>(p, e, s, carry, eb, up, tailP, tail, st);
    case 20: return scan_t<20, 20>(p, e, s, carry, eb, up, tailP, tail, st);
    }
    return hipErrorInvalidValue;
}

}  // namespace amx
