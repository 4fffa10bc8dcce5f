// amx_loud.hip -- loudnorm pass-1 measurement (ffmpeg af_loudnorm / libebur128,
// audio_mastering_engine.py:229): K-weighting, 100 ms hop energies, 400 ms gating
// blocks and 3 s short-term blocks -> histograms, sample peak.
// The K filter is continuous over the concatenated track (chunks do NOT reset it),
// so it uses the same GEMV + scan + re-run scheme over the track span, with the
// span's incoming state (carry) from the previous rank when chunk-sharded.
#include "amx_dev.hpp"

namespace amx {

// K-weighting pass 1: zero-state end state GEMV + per-(segment, channel) peak
// (reduced per track by k_peak_reduce)
__global__ void __launch_bounds__(AMX_BLOCK) k_kw1(const KwSegDev *__restrict__ ks, int n_kseg,
                                                   int L, const uint32_t *__restrict__ x,
                                                   const double *__restrict__ G,
                                                   double *__restrict__ e,
                                                   uint32_t *__restrict__ pk,
                                                   const int32_t *__restrict__ gate) {
    if (AMX_LN_GATED(gate)) return;
    __shared__ uint32_t s_in[Tile<1>::WORDS];
    __shared__ int64_t rb[AMX_BLOCK];
    __shared__ int rlo[AMX_BLOCK], rhi[AMX_BLOCK];
    const int t = threadIdx.x;
    const int j = blockIdx.x * AMX_BLOCK + t;
    const bool valid = j < n_kseg;
    const KwSegDev sg = ks[valid ? j : n_kseg - 1];
    // a partial (span-final) segment is read right-aligned in its L-frame row: its
    // len frames occupy rows [L-len, L) after zeros (the filter at rest sees zeros),
    // so every lane uses the same G row n (wave-uniform -> scalar loads)
    const int shift = valid ? L - sg.len : 0;
    rb[t] = valid ? sg.out_pos - shift : 0;
    rlo[t] = valid ? shift : 0;
    rhi[t] = valid ? L : 0;
    double e0[AMX_KW_DIM], e1[AMX_KW_DIM];
#pragma unroll
    for (int d = 0; d < AMX_KW_DIM; d++) { e0[d] = 0.0; e1[d] = 0.0; }
    int m0 = 0, m1 = 0;
    __syncthreads();
    for (int k = 0; k < L; k += AMX_TF) {
        tile_load<1>(s_in, x, rb, rlo, rhi, k);
        __syncthreads();
        const uint32_t *row = s_in + t * Tile<1>::PITCH;
#pragma unroll 4
        for (int f = 0; f < AMX_TF; f++) {
            const uint32_t p = row[f];
            const int a = lo16(p), b = hi16(p);
            m0 = max(m0, abs(a));
            m1 = max(m1, abs(b));
            const double xa = (double)a * (1.0 / 32768.0), xb = (double)b * (1.0 / 32768.0);
            const double *g = G + (int64_t)(k + f) * AMX_KW_DIM;
#pragma unroll
            for (int d = 0; d < AMX_KW_DIM; d++) {
                e0[d] = fma(g[d], xa, e0[d]);
                e1[d] = fma(g[d], xb, e1[d]);
            }
        }
        __syncthreads();
    }
    if (valid) {
        double *o = e + (int64_t)j * 2 * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) { o[d] = e0[d]; o[AMX_KW_DIM + d] = e1[d]; }
    }
    if (valid) {
        pk[(int64_t)j * 2] = (uint32_t)m0;
        pk[(int64_t)j * 2 + 1] = (uint32_t)m1;
    }
}

#define AMX_KW2_TILES 8   // segments of up to 128 frames (the plan's Lkw <= 128)
#define AMX_KW2_PITCH (AMX_TF + 1)
// K-weighting pass 2: filter from the true state (two DF-II-T biquads, see
// amx_plan.cpp), y^2 summed per 100 ms hop piece.  One thread per (segment,
// channel), lanes 2i / 2i+1 = L / R of row i.  parts[j][piece][ch], part_hop[j] =
// whole-track hop index of piece 0 (a segment spans <= 2 hops).
//
// Loads: thread t of wave w moves column t % 16 of rows 32 w + (t % 64) / 16 + 4 m
// (m < 8) of every 16-frame tile -- the wave's own rows, so tiles need no
// workgroup barrier; the row pointers are formed once, so a tile costs 8 loads with
// immediate offsets, all 8 tiles are issued up front (the recursion per tile is
// too short to hide an HBM round trip), and only a workgroup holding a partial
// (span-final) segment clamps addresses and masks frames (PART).
// ALIGNED (the hop is a multiple of 16 frames and every segment starts on a
// 16-frame boundary of the track): a segment's hop split falls on a tile
// boundary, so the accumulator is picked once per tile instead of per frame;
// each piece is still one sequential FMA chain in frame order.
// The 1/32768 sample scaling is folded into the first biquad's numerator
// (a power of two: the products, and so every rounding, are unchanged).
template <bool ALIGNED, bool PART>
__device__ __forceinline__ void kw2_run(const uint32_t *__restrict__ const *bp, const int *lm,
                                        int c, int rg, uint32_t *s_in, int row, int chn, int L,
                                        int len, int split, const double *c1, const double *c2,
                                        double *v, double &acc0, double &acc1) {
    uint32_t R[AMX_KW2_TILES][8];
#pragma unroll
    for (int q = 0; q < AMX_KW2_TILES; q++) {
        if (q * AMX_TF >= L) break;
#pragma unroll
        for (int m = 0; m < 8; m++) {
            if constexpr (PART) {
                const bool ok = q * AMX_TF + c < lm[m];
                R[q][m] = bp[m][ok ? q * AMX_TF : -c];     // frame 0 of the row: in range
                R[q][m] = ok ? R[q][m] : 0u;
            } else {
                R[q][m] = bp[m][q * AMX_TF];
            }
        }
    }
    const uint32_t *rp = s_in + row * AMX_KW2_PITCH;
    const int sh = chn ? 16 : 0;
#pragma unroll
    for (int q = 0; q < AMX_KW2_TILES; q++) {
        const int k = q * AMX_TF;
        if (k >= L) break;
#pragma unroll
        for (int m = 0; m < 8; m++) s_in[(rg + 4 * m) * AMX_KW2_PITCH + c] = R[q][m];
        amx_wave_sync();
        if constexpr (ALIGNED && !PART) {
            const bool lo = k < split;
            double a = lo ? acc0 : acc1;
#pragma unroll
            for (int f = 0; f < AMX_TF; f++) {
                const double xs = (double)(int)(int16_t)(rp[f] >> sh);
                const double u = bq_step(c1, v[0], v[1], xs);
                const double y = bq_step(c2, v[2], v[3], u);
                a = fma(y, y, a);
            }
            if (lo) acc0 = a;
            else acc1 = a;
        } else {
#pragma unroll 4
            for (int f = 0; f < AMX_TF; f++) {
                const int n = k + f;
                const double xs = (double)(int)(int16_t)(rp[f] >> sh);
                const double u = bq_step(c1, v[0], v[1], xs);
                double y = bq_step(c2, v[2], v[3], u);
                if constexpr (PART) y = n < len ? y : 0.0;
                if (n >= split) acc1 = fma(y, y, acc1);
                else acc0 = fma(y, y, acc0);
            }
        }
        amx_wave_sync();
    }
}

template <bool ALIGNED>
__global__ void __launch_bounds__(AMX_BLOCK) k_kw2(const ChainDev *__restrict__ cdp,
                                                   const KwSegDev *__restrict__ ks, int n_kseg,
                                                   int L, int hop,
                                                   const uint32_t *__restrict__ x,
                                                   const double *__restrict__ s,
                                                   double *__restrict__ parts,
                                                   int64_t *__restrict__ part_hop,
                                                   const int32_t *__restrict__ gate) {
    if (AMX_LN_GATED(gate)) return;
    constexpr int ROWS = AMX_BLOCK / 2;
    __shared__ uint32_t s_in[ROWS * AMX_KW2_PITCH];
    __shared__ int64_t rb[ROWS];
    __shared__ int rl[ROWS];
    const int t = threadIdx.x, row = t >> 1, chn = t & 1;
    const int j = blockIdx.x * ROWS + row;
    const bool valid = j < n_kseg;
    const KwSegDev sg = ks[valid ? j : n_kseg - 1];
    const int len = valid ? sg.len : 0;
    if (chn == 0) {
        rb[row] = valid ? sg.out_pos : 0;
        rl[row] = len;
    }
    double c1[5], c2[5];
#pragma unroll
    for (int i = 0; i < 3; i++) { c1[i] = cdp->kw1[i] * (1.0 / 32768.0); c2[i] = cdp->kw2[i]; }
    c1[3] = cdp->kw1[4]; c1[4] = cdp->kw1[5];
    c2[3] = cdp->kw2[4]; c2[4] = cdp->kw2[5];
    double v[4];
    const double *st = s + ((int64_t)(valid ? j : 0) * 2 + chn) * AMX_KW_DIM;
#pragma unroll
    for (int d = 0; d < 4; d++) v[d] = valid ? st[d] : 0.0;
    const int64_t h0 = sg.tframe / hop;
    const int split = (int)((h0 + 1) * hop - sg.tframe);   // first frame of piece 1
    const int part = __syncthreads_or(len < L);
    // wave-local rows: wave w moves (and computes on) rows 32 w .. 32 w + 31 only
    const int c = t & 15, rg = 32 * (t >> 6) + ((t & 63) >> 4);
    const uint32_t *bp[8];
    int lm[8];
#pragma unroll
    for (int m = 0; m < 8; m++) {
        bp[m] = x + rb[rg + 4 * m] + c;
        lm[m] = rl[rg + 4 * m];
    }
    double acc0 = 0.0, acc1 = 0.0;
    if (part)
        kw2_run<ALIGNED, true>(bp, lm, c, rg, s_in, row, chn, L, len, split, c1, c2, v, acc0, acc1);
    else
        kw2_run<ALIGNED, false>(bp, lm, c, rg, s_in, row, chn, L, len, split, c1, c2, v, acc0, acc1);
    if (valid) {
        double *o = parts + (int64_t)j * 4;
        o[chn] = acc0;
        o[2 + chn] = acc1;
        if (chn == 0) part_hop[j] = h0;
    }
}

// per-hop sum of the segment pieces: one wave per hop, lanes over the hop's
// segments, then a fixed butterfly (deterministic for a given segment grid)
__global__ void __launch_bounds__(AMX_BLOCK) k_hops(const SpanDev *__restrict__ spans,
                                                    const KwSegDev *__restrict__ ks, int L,
                                                    int hop, const double *__restrict__ parts,
                                                    const int64_t *__restrict__ part_hop,
                                                    double *__restrict__ hops, int64_t max_hops) {
    const int t = blockIdx.y;
    const SpanDev sp = spans[t];
    const int lane = threadIdx.x & 63;
    const int64_t hfirst = sp.m_tframe0 / hop;
    const int64_t hlast = sp.nkseg ? (sp.m_tframe0 + sp.m_n - 1) / hop : hfirst - 1;
    const int64_t h = (int64_t)blockIdx.x * (AMX_BLOCK / 64) + (threadIdx.x >> 6);
    if (h >= max_hops) return;                       // wave-uniform
    if (h < hfirst || h > hlast) {                   // hops of other ranks' spans: 0
        if (lane == 0) {
            hops[((int64_t)t * max_hops + h) * 2] = 0.0;
            hops[((int64_t)t * max_hops + h) * 2 + 1] = 0.0;
        }
        return;
    }
    // span-local frame range of hop h (measurement stream)
    int64_t a = h * hop - sp.m_tframe0, bnd = (h + 1) * hop - sp.m_tframe0;
    if (a < 0) a = 0;
    if (bnd > sp.m_n) bnd = sp.m_n;
    const int64_t j0 = a / L, j1 = (bnd - 1) / L;
    double s0 = 0.0, s1 = 0.0;
    for (int64_t jj = j0 + lane; jj <= j1; jj += 64) {
        const int64_t j = sp.kseg0 + jj;
        const int pc = part_hop[j] == h ? 0 : 1;
        s0 += parts[j * 4 + 2 * pc];
        s1 += parts[j * 4 + 2 * pc + 1];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s0 += __shfl_xor(s0, o);
        s1 += __shfl_xor(s1, o);
    }
    if (lane == 0) {
        hops[((int64_t)t * max_hops + h) * 2] = s0;
        hops[((int64_t)t * max_hops + h) * 2 + 1] = s1;
    }
}

__device__ __forceinline__ int find_bin(const double *bounds, double energy) {
    int lo = 0, hi = 1000;
    do {
        int mid = (lo + hi) / 2;
        if (energy >= bounds[mid]) lo = mid; else hi = mid;
    } while (hi - lo != 1);
    return lo;
}

// gating blocks (400 ms every 100 ms) and short-term blocks (3 s every 1 s): one
// workgroup per track, histograms in LDS, written whole (no zeroing pass needed)
#define AMX_HIST_THREADS 1024
__global__ void __launch_bounds__(AMX_HIST_THREADS) k_hist(const SpanDev *__restrict__ spans,
                                                           int hop,
                                                           const double *__restrict__ hops,
                                                           int64_t max_hops,
                                                           const double *__restrict__ bounds,
                                                           unsigned long long *__restrict__ hist,
                                                           unsigned long long *__restrict__ st_hist) {
    __shared__ unsigned int h[AMX_HIST_BINS], sh[AMX_HIST_BINS];
    __shared__ double bd[AMX_HIST_BINS + 1];
    const int t = blockIdx.x;
    const SpanDev sp = spans[t];
    for (int i = threadIdx.x; i < AMX_HIST_BINS; i += AMX_HIST_THREADS) { h[i] = 0u; sh[i] = 0u; }
    for (int i = threadIdx.x; i <= AMX_HIST_BINS; i += AMX_HIST_THREADS) bd[i] = bounds[i];
    __syncthreads();
    int64_t nh = sp.m_total / hop;
    if (nh > max_hops) nh = max_hops;
    const double *H = hops + (int64_t)t * max_hops * 2;
    for (int64_t k = threadIdx.x; k + 4 <= nh; k += AMX_HIST_THREADS) {
        double c0 = ((H[2 * k] + H[2 * (k + 1)]) + H[2 * (k + 2)]) + H[2 * (k + 3)];
        double c1 = ((H[2 * k + 1] + H[2 * (k + 1) + 1]) + H[2 * (k + 2) + 1]) + H[2 * (k + 3) + 1];
        double en = (c0 + c1) / (double)(4 * (int64_t)hop);
        if (en >= bd[0]) atomicAdd(&h[find_bin(bd, en)], 1u);
    }
    // short-term block m ends at hop 30 + 10 m
    for (int64_t m = threadIdx.x; 30 + 10 * m <= nh; m += AMX_HIST_THREADS) {
        const int64_t end = 30 + 10 * m;
        double c0 = 0.0, c1 = 0.0;
        for (int64_t q = end - 30; q < end; q++) { c0 += H[2 * q]; c1 += H[2 * q + 1]; }
        double en = (c0 + c1) / (double)(30 * (int64_t)hop);
        if (en >= bd[0]) atomicAdd(&sh[find_bin(bd, en)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < AMX_HIST_BINS; i += AMX_HIST_THREADS) {
        hist[(int64_t)t * AMX_HIST_BINS + i] = h[i];
        st_hist[(int64_t)t * AMX_HIST_BINS + i] = sh[i];
    }
}

// ================================================================ launchers
hipError_t launch_kw1(const ChainDev *cd, const KwSegDev *ks, int n_kseg, int L,
                      const int16_t *x, const double *G, double *e, uint32_t *pk,
                      const int32_t *gate, hipStream_t st) {
    (void)cd;
    if (n_kseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_kw1, grid1(n_kseg), dim3(AMX_BLOCK), 0, st, ks, n_kseg, L,
                       reinterpret_cast<const uint32_t *>(x), G, e, pk, gate);
    return hipGetLastError();
}

hipError_t launch_kw2(const ChainDev *cd, const KwSegDev *ks, int n_kseg, int L, int hop,
                      const int16_t *x, const double *s, double *parts, int64_t *part_hop,
                      int aligned, const int32_t *gate, hipStream_t st) {
    if (n_kseg <= 0) return hipSuccess;
    if (L > AMX_KW2_TILES * AMX_TF || L % AMX_TF) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((n_kseg + AMX_BLOCK / 2 - 1) / (AMX_BLOCK / 2)));
    if (aligned)
        hipLaunchKernelGGL(k_kw2<true>, grid, dim3(AMX_BLOCK), 0, st, cd, ks, n_kseg, L, hop,
                           reinterpret_cast<const uint32_t *>(x), s, parts, part_hop, gate);
    else
        hipLaunchKernelGGL(k_kw2<false>, grid, dim3(AMX_BLOCK), 0, st, cd, ks, n_kseg, L, hop,
                           reinterpret_cast<const uint32_t *>(x), s, parts, part_hop, gate);
    return hipGetLastError();
}

hipError_t launch_hops(const SpanDev *spans, int n_tracks, const KwSegDev *ks, int L, int hop,
                       const double *parts, const int64_t *part_hop, double *hops,
                       int64_t max_hops, hipStream_t st) {
    const int wpb = AMX_BLOCK / 64;   // hops per workgroup (one wave each)
    dim3 g((unsigned)((max_hops + wpb - 1) / wpb), (unsigned)n_tracks);
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_hops, g, dim3(AMX_BLOCK), 0, st, spans, ks, L, hop, parts, part_hop,
                       hops, max_hops);
    return hipGetLastError();
}

hipError_t launch_hist(const SpanDev *spans, int n_tracks, int hop, const double *hops,
                       int64_t max_hops, const double *bounds, unsigned long long *hist,
                       unsigned long long *st_hist, hipStream_t st) {
    if (n_tracks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_hist, dim3(n_tracks), dim3(AMX_HIST_THREADS), 0, st, spans, hop, hops,
                       max_hops, bounds, hist, st_hist);
    return hipGetLastError();
}


// Sample peak per track from the per-(segment, channel) maxima k_front2 wrote
// when it ran the loudness pass-1 work fused (pk[j][ch] = max |x|).  grid.y =
// track, each workgroup reduces a contiguous run of that track's segments in LDS
// and issues one atomicMax per channel (the peak buffer is zeroed by
// amx_loudness_pass1 first): same-address atomics serialise, so there are few.
#define AMX_PEAK_THREADS 1024
#define AMX_PEAK_PER_THREAD 8
// kw_fix: k_front2 accumulated the K-filter GEMV with the row of a full L-frame
// segment (wave-uniform); a span's last segment shorter than L needs its rows
// right-aligned (G[n + L - len], as k_kw1 does), so wave 0 of the span's first
// workgroup redoes that one segment here (lanes split the frames, butterfly sum).
__global__ void __launch_bounds__(AMX_PEAK_THREADS) k_peak_reduce(const SpanDev *__restrict__ spans,
                                                                  const uint32_t *__restrict__ pk,
                                                                  double *__restrict__ peak,
                                                                  unsigned int *__restrict__ cnt,
                                                                  int *__restrict__ part,
                                                                  const KwSegDev *__restrict__ ks,
                                                                  int L, const uint32_t *__restrict__ x,
                                                                  const double *__restrict__ G,
                                                                  double *__restrict__ e, int kw_fix,
                                                                  int resamp) {
    __shared__ int red[4][AMX_PEAK_THREADS / 64];
    const int t = blockIdx.y;
    const SpanDev sp = spans[t];
    const int64_t q0 = (int64_t)blockIdx.x * AMX_PEAK_THREADS * AMX_PEAK_PER_THREAD;
    if (q0 >= sp.nkseg) return;                      // block-uniform
    if (kw_fix && blockIdx.x == 0 && threadIdx.x < 64) {
        const int64_t j = (int64_t)sp.kseg0 + sp.nkseg - 1;
        const KwSegDev sg = ks[j];
        if (sg.len < L) {                            // wave-uniform
            double a[2 * AMX_KW_DIM];
#pragma unroll
            for (int d = 0; d < 2 * AMX_KW_DIM; d++) a[d] = 0.0;
            const int sh = L - sg.len;
            for (int n = threadIdx.x; n < sg.len; n += 64) {
                const uint32_t p = x[sg.out_pos + n];
                const double xa = (double)lo16(p) * (1.0 / 32768.0), xb = (double)hi16(p) * (1.0 / 32768.0);
                const double *g = G + (int64_t)(n + sh) * AMX_KW_DIM;
#pragma unroll
                for (int d = 0; d < AMX_KW_DIM; d++) {
                    a[d] = fma(g[d], xa, a[d]);
                    a[AMX_KW_DIM + d] = fma(g[d], xb, a[AMX_KW_DIM + d]);
                }
            }
#pragma unroll
            for (int d = 0; d < 2 * AMX_KW_DIM; d++)
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) a[d] += __shfl_xor(a[d], o);
            if (threadIdx.x < 2 * AMX_KW_DIM) {
                double v = a[0];
#pragma unroll
                for (int d = 1; d < 2 * AMX_KW_DIM; d++) v = threadIdx.x == d ? a[d] : v;
                e[j * 2 * AMX_KW_DIM + threadIdx.x] = v;
            }
        }
    }
    // per segment: resamp -> [4] = 192 kHz |u| max L, R as float bits (non-negative
    // floats order like their bits), native |x| L, R as int16 magnitudes; else [2] = |x|
    const int stride = resamp ? 4 : 2;
    int m[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < AMX_PEAK_PER_THREAD; i++) {
        const int64_t q = q0 + threadIdx.x + (int64_t)i * AMX_PEAK_THREADS;
        const bool ok = q < sp.nkseg;
        const int64_t j = (int64_t)sp.kseg0 + (ok ? q : 0);
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t v = c < stride ? pk[j * stride + c] : 0u;
            m[c] = max(m[c], ok ? (int)v : 0);
        }
    }
#pragma unroll
    for (int c = 0; c < 4; c++)
        for (int o = 32; o > 0; o >>= 1) m[c] = max(m[c], __shfl_xor(m[c], o));
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int c = 0; c < 4; c++) red[c][threadIdx.x >> 6] = m[c];
    }
    __syncthreads();
    // the block's maxima go to its slot of `part`; the last block of the track to
    // finish (counter) reduces the slots and writes the peak, then re-arms the
    // counter -- no zeroing pass before, no atomics on the result
    __shared__ bool last;
    const int nb = (int)((sp.nkseg + (int64_t)AMX_PEAK_THREADS * AMX_PEAK_PER_THREAD - 1) /
                         ((int64_t)AMX_PEAK_THREADS * AMX_PEAK_PER_THREAD));
    if (threadIdx.x == 0) {
        int mm[4] = {0, 0, 0, 0};
        for (int w = 0; w < AMX_PEAK_THREADS / 64; w++)
            for (int c = 0; c < 4; c++) mm[c] = max(mm[c], red[c][w]);
        int *pt = part + ((int64_t)t * gridDim.x + blockIdx.x) * 4;
        // the hand-off of DESIGN.md §3.7: write-through (agent-scope atomic) stores of the
        // slot, drained, then one relaxed agent-scope count; the last block acquires once.
        // (__threadfence() in every block wrote back the XCD's whole L2)
        for (int c = 0; c < 4; c++) __hip_atomic_store(pt + c, mm[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(cnt + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nb - 1);
    }
    __syncthreads();
    if (last) {
        // the slots in parallel (a thread per slot and channel word, then the block's max),
        // not one thread's chain of dependent volatile loads
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int v = 0;
        for (int k = threadIdx.x; k < 4 * nb; k += AMX_PEAK_THREADS) {
            const volatile int *q = part + (int64_t)t * gridDim.x * 4 + k;
            v = max(v, *q);
        }
        // threads with the same k % 4 hold the same channel word: fold over the block
        for (int o = 4; o < 64; o <<= 1) v = max(v, __shfl_xor(v, o));
        __syncthreads();                                 // red[] of the first pass was read
        if ((threadIdx.x & 63) < 4) red[threadIdx.x & 3][threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            int ma[4] = {0, 0, 0, 0};
            for (int w = 0; w < AMX_PEAK_THREADS / 64; w++)
                for (int c = 0; c < 4; c++) ma[c] = max(ma[c], red[c][w]);
            // peak[t][4]: the measured stream's sample peak (loudnorm's input_tp) per
            // channel, then the chain output's own sample peak (the limiter's input bound)
            double *pp = peak + 4 * t;
            if (resamp) {
                pp[0] = (double)__int_as_float(ma[0]);
                pp[1] = (double)__int_as_float(ma[1]);
                pp[2] = (double)ma[2] * (1.0 / 32768.0);
                pp[3] = (double)ma[3] * (1.0 / 32768.0);
            } else {
                pp[0] = pp[2] = (double)ma[0] * (1.0 / 32768.0);
                pp[1] = pp[3] = (double)ma[1] * (1.0 / 32768.0);
            }
            cnt[t] = 0u;
        }
    }
}

int peak_reduce_blocks(int64_t max_nkseg) {
    const int64_t per = (int64_t)AMX_PEAK_THREADS * AMX_PEAK_PER_THREAD;
    return (int)((max_nkseg + per - 1) / per);
}

hipError_t launch_peak_reduce(const SpanDev *spans, int n_tracks, int64_t max_nkseg,
                              const uint32_t *pk, double *peak, unsigned int *cnt, int *part,
                              const KwSegDev *ks, int L, const int16_t *x, const double *G,
                              double *e, int kw_fix, int resamp, hipStream_t st) {
    dim3 g((unsigned)peak_reduce_blocks(max_nkseg), (unsigned)n_tracks);
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_peak_reduce, g, dim3(AMX_PEAK_THREADS), 0, st, spans, pk, peak, cnt, part,
                       ks, L, reinterpret_cast<const uint32_t *>(x), G, e, kw_fix, resamp);
    return hipGetLastError();
}

// K-filter state at each span end from rest: P_t * s_last + e_last (per lane)
__global__ void k_kw_tail(const SpanDev *__restrict__ spans, int n_tracks,
                          const double *__restrict__ s, const double *__restrict__ e,
                          const double *__restrict__ P, double *__restrict__ tail) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tracks) return;
    const SpanDev sp = spans[t];
    for (int c = 0; c < 2; c++) {
        double *o = tail + ((int64_t)t * 2 + c) * AMX_KW_DIM;
        if (sp.nkseg == 0) { for (int d = 0; d < AMX_KW_DIM; d++) o[d] = 0.0; continue; }
        const int64_t j = sp.kseg0 + sp.nkseg - 1;
        const double *sj = s + (j * 2 + c) * AMX_KW_DIM, *ej = e + (j * 2 + c) * AMX_KW_DIM;
        const double *Pt = P + (int64_t)t * 16;
        for (int i = 0; i < AMX_KW_DIM; i++) {
            double acc = ej[i];
            for (int k = 0; k < AMX_KW_DIM; k++) acc = fma(Pt[i * 4 + k], sj[k], acc);
            o[i] = acc;
        }
    }
}

hipError_t launch_kw_tail(const SpanDev *spans, int n_tracks, const double *s, const double *e,
                          const double *P, double *tail, hipStream_t st) {
    hipLaunchKernelGGL(k_kw_tail, dim3((n_tracks + 63) / 64), dim3(64), 0, st, spans, n_tracks, s,
                       e, P, tail);
    return hipGetLastError();
}

// ------------------------------------------------------------------ decision
// loudnorm pass-1 statistics and the pass-2 linear-mode decision (af_loudnorm
// init, audio_mastering_engine.py:229-242), the gain, and whether the final
// alimiter can engage -- on the device, so a step needs no host round trip.
// The arithmetic is amx/loudness.py's (libebur128 loop orders): one wave per track;
// non-empty histogram bins are compacted in ascending order (adding an empty bin's
// 0.0 is exact) and lane 0 runs the sequential double sums over them.

// round2 ("%.2f" then float()): amx_dev.hpp

__device__ __forceinline__ double lufs_of(double e) { return 10 * log10(e) - 0.691; }

// Wave-parallel histogram arithmetic: lane l owns bins [16 l, 16 l + 16).  Counts
// are integers (exact in double), so count sums and prefix walks are exact in any
// order; the energy sums keep libebur128's sequential order (wave_seq_sum).
#define AMX_BPL 16
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// sum over the bins j >= lo, ascending, of count_j * energy_j in libebur128's
// sequential order (ebur128_gated_loudness / ebur128_loudness_range loops): the
// owning lanes form the products, the non-empty ones are compacted in bin order into
// this wave's LDS buffer (adding an empty bin's 0.0 leaves the sum unchanged) and
// lane 0 adds them one by one; the sum is broadcast.  Bit-identical to the C loop.
__device__ double wave_seq_sum(const double (&cc)[AMX_BPL], const double (&en)[AMX_BPL], int lo,
                               double *sbuf) {
    const int lane = threadIdx.x & 63;
    int mine = 0;
#pragma unroll
    for (int q = 0; q < AMX_BPL; q++) mine += (lane * AMX_BPL + q >= lo && cc[q] != 0.0) ? 1 : 0;
    int incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int up = __shfl_up(incl, o);
        if (lane >= o) incl += up;
    }
    int off = incl - mine;
    const int tot = __shfl(incl, 63);
#pragma unroll
    for (int q = 0; q < AMX_BPL; q++)
        if (lane * AMX_BPL + q >= lo && cc[q] != 0.0) sbuf[off++] = cc[q] * en[q];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    double acc = 0.0;
    if (lane == 0)
        for (int k = 0; k < tot; k++) acc += sbuf[k];
    __builtin_amdgcn_wave_barrier();
    return __shfl(acc, 0);
}

// bin search without a table walk: the largest b < 1000 with bounds[b] <= v (what
// find_bin's bisection returns for v >= bounds[0]) is the number of the 1000 lower
// bounds <= v, minus one; each lane counts its 16, the wave sums
__device__ __forceinline__ int wave_find_bin(const double (&bd)[AMX_BPL], double v) {
    int c = 0;
#pragma unroll
    for (int q = 0; q < AMX_BPL; q++) c += bd[q] <= v ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    return c - 1;
}

// the energy of bin j from the lane that owns it
__device__ __forceinline__ double wave_bin_value(const double (&en)[AMX_BPL], int j) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < AMX_BPL; q++) v = (j % AMX_BPL) == q ? en[q] : v;
    return __shfl(v, j / AMX_BPL);
}

// two waves: wave 0 the integrated loudness (gating histogram), wave 1 the loudness
// range (short-term histogram) -- independent chains of dependent reductions, run
// side by side; wave 0's lane 0 then forms the statistics and the decision
__global__ void __launch_bounds__(128) k_decide(DecideArgs a) {
    const int t = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __shared__ double s_lra;
    __shared__ double s_sum[2][AMX_HIST_BINS];
    double I = -INFINITY, thr = -70.0, lra = 0.0;
    if (a.lufs_on) {
        // lane l owns bins [16 l, 16 l + 16): this wave's counts, the bin energies and
        // lower bounds in registers, every load in flight before the first use (bins
        // past 999 hold count 0 and bound +inf)
        const unsigned long long *C = (wv == 0 ? a.hist : a.st_hist) + (int64_t)t * AMX_HIST_BINS;
        double cc[AMX_BPL], en[AMX_BPL], bd[AMX_BPL];
#pragma unroll
        for (int q = 0; q < AMX_BPL; q++) {
            const int j = lane * AMX_BPL + q;
            const int jj = j < AMX_HIST_BINS ? j : AMX_HIST_BINS - 1;
            const bool ok = j < AMX_HIST_BINS;
            const unsigned long long h = C[jj];
            const double e = a.energies[jj], b = a.bounds[jj];
            cc[q] = ok ? (double)h : 0.0;
            en[q] = e;
            bd[q] = ok ? b : INFINITY;
        }
        const double b0 = __shfl(bd[0], 0);
        if (wv == 0) {
            // integrated loudness with the relative gate (ebur128_gated_loudness)
            double cnt = 0.0;
#pragma unroll
            for (int q = 0; q < AMX_BPL; q++) cnt += cc[q];
            double rel = wave_seq_sum(cc, en, 0, s_sum[0]);
            cnt = wave_sum(cnt);                           // integers: exact in any order
            if (cnt != 0.0) {
                rel /= cnt;
                rel *= 0.1;                                // pow(10, -10/10)
                thr = lufs_of(rel);
                int start;
                if (rel < b0) start = 0;
                else {
                    start = wave_find_bin(bd, rel);
                    if (rel > wave_bin_value(en, start)) ++start;
                }
                double above = 0.0;
#pragma unroll
                for (int q = 0; q < AMX_BPL; q++) above += lane * AMX_BPL + q >= start ? cc[q] : 0.0;
                const double g = wave_seq_sum(cc, en, start, s_sum[0]);
                above = wave_sum(above);
                if (above != 0.0) I = lufs_of(g / above);
            }
        } else {
            // loudness range (ebur128_loudness_range) on the short-term histogram
            double size = 0.0;
#pragma unroll
            for (int q = 0; q < AMX_BPL; q++) size += cc[q];
            size = wave_sum(size);
            double power = wave_seq_sum(cc, en, 0, s_sum[1]);
            if (size != 0.0) {
                power /= size;
                const double integ = 0.01 * power;         // pow(10, -20/10)
                int index;
                if (integ < b0) index = 0;
                else {
                    index = wave_find_bin(bd, integ);
                    if (integ > wave_bin_value(en, index)) ++index;
                }
                double mine = 0.0;                         // this lane's counts at bins >= index
                double cum[AMX_BPL];
#pragma unroll
                for (int q = 0; q < AMX_BPL; q++) {
                    mine += lane * AMX_BPL + q >= index ? cc[q] : 0.0;
                    cum[q] = mine;
                }
                // exclusive prefix of the lane totals (exact integer arithmetic)
                double incl = mine;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const double up = __shfl_up(incl, o);
                    if (lane >= o) incl += up;
                }
                const double before = incl - mine;
                const double tot = __shfl(incl, 63);
                if (tot != 0.0) {
                    const double plo = (double)(int64_t)((tot - 1) * 0.1 + 0.5);
                    const double phi = (double)(int64_t)((tot - 1) * 0.95 + 0.5);
                    // the walk stops at the first bin whose cumulative count exceeds p
                    int jl = 0x7fffffff, jh = 0x7fffffff;
#pragma unroll
                    for (int q = AMX_BPL - 1; q >= 0; q--) {
                        const int j = lane * AMX_BPL + q;
                        const double c = before + cum[q];
                        const bool nz = j >= index && cc[q] != 0.0;
                        if (nz && c > plo) jl = j;
                        if (nz && c > phi) jh = j;
                    }
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) {
                        jl = min(jl, __shfl_xor(jl, o));
                        jh = min(jh, __shfl_xor(jh, o));
                    }
                    lra = lufs_of(wave_bin_value(en, jh)) - lufs_of(wave_bin_value(en, jl));
                }
            }
            if (lane == 0) s_lra = lra;
        }
    }
    __syncthreads();
    if (a.lufs_on) lra = s_lra;
    if (threadIdx.x != 0) return;
    // input_tp: the measured (192 kHz) stream's sample peak; the limiter bound below
    // uses the chain output's own peak (the samples the gain and alimiter see)
    const double pk = fmax(a.peak[4 * t], a.peak[4 * t + 1]);
    const double pk_out = fmax(a.peak[4 * t + 2], a.peak[4 * t + 3]);
    const double tp = pk > 0.0 ? 20.0 * log10(pk) : -INFINITY;
    const double si = round2(I), stp = round2(tp), slra = round2(lra), sthr = round2(thr);
    int mode = 0;                                   // 0 off, 1 skip, 2 linear, 3 dynamic
    double gain = -1.0;
    if (a.lufs_on) {
        if (si == -INFINITY) mode = 1;
        else {
            const double offset = a.target_i - si;
            const double offset_tp = stp + offset;
            if (stp != 99 && sthr != -70 && slra != 0 && si != 0 && offset_tp <= a.target_tp &&
                slra <= a.target_lra) {
                mode = 2;
                gain = pow(10.0, offset / 20.0);
            } else {
                mode = 3;
            }
        }
    }
    // max |sample| after the gain stage (llrint(x*g) clipped), the limiter's input
    const double m16 = rint(pk_out * 32768.0);
    double amax = m16 / 32768.0;
    if (gain > 0.0) amax = fmin(rint(((m16 * (1.0 / 32768.0)) * gain) * 32768.0), 32768.0) / 32768.0;
    const bool fast = amax * a.level_in <= a.limit;
    double *o = a.stats + (int64_t)t * AMX_STATS;
    o[0] = I; o[1] = lra; o[2] = thr; o[3] = tp;
    o[4] = si; o[5] = stp; o[6] = slra; o[7] = sthr;
    o[8] = (double)mode; o[9] = gain; o[10] = fast ? 1.0 : 0.0; o[11] = pk; o[12] = pk_out;
    a.gains[t] = gain;
    const int32_t w = (fast ? AMX_CTL_FAST : 0) | (mode << 4);
    a.ctl[t] = w;
    // (amx_plan_set_publish) the word straight into the caller's pinned host memory, a
    // system-scope store: the host polls it while the limiter runs, no node of its own
    if (a.host_ctl) __hip_atomic_store(a.host_ctl + t, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_decide(const DecideArgs &a, hipStream_t st) {
    if (a.n_tracks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_decide, dim3(a.n_tracks), dim3(128), 0, st, a);
    return hipGetLastError();
}

// the decision words stored straight into the caller's pinned host memory (system-scope
// stores from one small kernel): no copy node, whose completion signalling stalled the
// stream ~25 us in a captured step
__global__ void k_publish(const int32_t *__restrict__ ctl, int32_t *host, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x)
        __hip_atomic_store(host + i, ctl[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_publish(const int32_t *ctl, int32_t *host, int n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, st, ctl, host, n);
    return hipGetLastError();
}

// K-filter state entering this rank's span from the other ranks' zero-start tails:
// carry = sum_q P_q tail_q (P_q = A^{frames between span q's end and this span},
// host-computed), per channel; one thread per (channel, row).
__global__ void k_kw_carry(const double *__restrict__ tails, const double *__restrict__ P,
                           int n_prev, double *__restrict__ carry) {
    const int c = threadIdx.x / AMX_KW_DIM, i = threadIdx.x % AMX_KW_DIM;
    if (c >= 2) return;
    double acc = 0.0;
    for (int q = 0; q < n_prev; q++) {
        const double *Pq = P + (int64_t)q * AMX_KW_DIM * AMX_KW_DIM;
        const double *tq = tails + ((int64_t)q * 2 + c) * AMX_KW_DIM;
#pragma unroll
        for (int k = 0; k < AMX_KW_DIM; k++) acc = fma(Pq[i * AMX_KW_DIM + k], tq[k], acc);
    }
    carry[c * AMX_KW_DIM + i] = acc;
}

hipError_t launch_kw_carry(const double *tails, const double *P, int n_prev, double *carry,
                           hipStream_t st) {
    hipLaunchKernelGGL(k_kw_carry, dim3(1), dim3(64), 0, st, tails, P, n_prev, carry);
    return hipGetLastError();
}

// the gathered exchange rows (row q: tail [2][4] at 0, peaks [4] at 8, stride ld):
// threads 0-7 the carry from the rows q < n_prev, threads 8-11 the peak max over all rows
__global__ void k_kw_carry_rows(const double *__restrict__ rows, int world, int ld,
                                const double *__restrict__ P, int n_prev, double *__restrict__ carry,
                                double *__restrict__ peak) {
    const int t = threadIdx.x;
    if (t < 2 * AMX_KW_DIM) {
        const int c = t / AMX_KW_DIM, i = t % AMX_KW_DIM;
        double acc = 0.0;
        for (int q = 0; q < n_prev; q++) {
            const double *Pq = P + (int64_t)q * AMX_KW_DIM * AMX_KW_DIM;
            const double *tq = rows + (int64_t)q * ld + c * AMX_KW_DIM;
#pragma unroll
            for (int k = 0; k < AMX_KW_DIM; k++) acc = fma(Pq[i * AMX_KW_DIM + k], tq[k], acc);
        }
        carry[t] = acc;
    } else if (t < 2 * AMX_KW_DIM + 4) {
        const int c = t - 2 * AMX_KW_DIM;
        double m = rows[2 * AMX_KW_DIM + c];
        for (int q = 1; q < world; q++) m = fmax(m, rows[(int64_t)q * ld + 2 * AMX_KW_DIM + c]);
        peak[c] = m;
    }
}

hipError_t launch_kw_carry_rows(const double *rows, int world, int ld, const double *P, int n_prev,
                                double *carry, double *peak, hipStream_t st) {
    hipLaunchKernelGGL(k_kw_carry_rows, dim3(1), dim3(64), 0, st, rows, world, ld, P, n_prev, carry, peak);
    return hipGetLastError();
}

}  // namespace amx
