// amx_loud.hip -- loudnorm pass-1 measurement (ffmpeg af_loudnorm / libebur128,
// audio_mastering_engine.py:229): K-weighting, 100 ms hop energies, 400 ms gating
// blocks and 3 s short-term blocks -> histograms, sample peak.
// The K filter is continuous over the concatenated track (chunks do NOT reset it),
// so it uses the same GEMV + scan + re-run scheme over the track span, with the
// span's incoming state (carry) from the previous rank when chunk-sharded.
#include "amx_dev.hpp"

namespace amx {

// K-weighting pass 1: zero-state end state GEMV + sample peak
__global__ void __launch_bounds__(AMX_BLOCK) k_kw1(const KwSegDev *__restrict__ ks, int n_kseg,
                                                   int L, const uint32_t *__restrict__ x,
                                                   const double *__restrict__ G,
                                                   double *__restrict__ e,
                                                   unsigned long long *__restrict__ peak) {
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
    // sample peak: wave max first, one atomic per wave when the wave is one track
    const int t0 = __shfl(sg.track, 0);
    const bool same = __ballot(sg.track != t0) == 0ull;
    if (same) {
        for (int o = 32; o > 0; o >>= 1) {
            m0 = max(m0, __shfl_xor(m0, o));
            m1 = max(m1, __shfl_xor(m1, o));
        }
    }
    if (valid && (!same || (threadIdx.x & 63) == 0)) {
        const double p0 = (double)m0 * (1.0 / 32768.0), p1 = (double)m1 * (1.0 / 32768.0);
        atomicMax(peak + 2 * sg.track, (unsigned long long)__double_as_longlong(p0));
        atomicMax(peak + 2 * sg.track + 1, (unsigned long long)__double_as_longlong(p1));
    }
}

// K-weighting pass 2: filter from the true state (two DF-II-T biquads, see
// amx_plan.cpp), y^2 summed per 100 ms hop piece.  One thread per (segment,
// channel), lanes 2i / 2i+1 = L / R of row i.  parts[j][piece][ch], part_hop[j] =
// whole-track hop index of piece 0 (a segment spans <= 2 hops).
__global__ void __launch_bounds__(AMX_BLOCK) k_kw2(const ChainDev *__restrict__ cdp,
                                                   const KwSegDev *__restrict__ ks, int n_kseg,
                                                   int L, int hop,
                                                   const uint32_t *__restrict__ x,
                                                   const double *__restrict__ s,
                                                   double *__restrict__ parts,
                                                   int64_t *__restrict__ part_hop) {
    constexpr int ROWS = AMX_BLOCK / 2;
    using T = Tile<1, ROWS>;
    __shared__ uint32_t s_in[T::WORDS];
    __shared__ int64_t rb[ROWS];
    __shared__ int rl[ROWS];
    __shared__ double s_c[12];
    const ChainDev &cd = *cdp;
    const int t = threadIdx.x, row = t >> 1, chn = t & 1;
    const int j = blockIdx.x * ROWS + row;
    const bool valid = j < n_kseg;
    const KwSegDev sg = ks[valid ? j : n_kseg - 1];
    if (chn == 0) {
        rb[row] = valid ? sg.out_pos : 0;
        rl[row] = valid ? sg.len : 0;
    }
    if (t < 6) s_c[t] = cd.kw1[t];
    else if (t < 12) s_c[t] = cd.kw2[t - 6];
    double v[4];
    const double *st = s + ((int64_t)(valid ? j : 0) * 2 + chn) * AMX_KW_DIM;
#pragma unroll
    for (int d = 0; d < 4; d++) v[d] = valid ? st[d] : 0.0;
    const int len = valid ? sg.len : 0;
    const int64_t h0 = sg.tframe / hop;
    const int64_t split = (h0 + 1) * hop - sg.tframe;   // first frame of piece 1
    double acc0 = 0.0, acc1 = 0.0;
    __syncthreads();
    double c1[5], c2[5];
#pragma unroll
    for (int i = 0; i < 3; i++) { c1[i] = s_c[i]; c2[i] = s_c[6 + i]; }
    c1[3] = s_c[4]; c1[4] = s_c[5];
    c2[3] = s_c[10]; c2[4] = s_c[11];
    for (int k = 0; k < L; k += AMX_TF) {
        tile_load<1, ROWS>(s_in, x, rb, nullptr, rl, k);
        __syncthreads();
        const uint32_t *rp = s_in + row * T::PITCH;
#pragma unroll 4
        for (int f = 0; f < AMX_TF; f++) {
            const uint32_t p = rp[f];
            const int n = k + f;
            const double xs = (double)(chn ? hi16(p) : lo16(p)) * (1.0 / 32768.0);
            const double u = bq_step(c1, v[0], v[1], xs);
            const double y = n < len ? bq_step(c2, v[2], v[3], u) : 0.0;
            if (n >= split) acc1 = fma(y, y, acc1);
            else acc0 = fma(y, y, acc0);
        }
        __syncthreads();
    }
    if (valid) {
        double *o = parts + (int64_t)j * 4;
        o[chn] = acc0;
        o[2 + chn] = acc1;
        if (chn == 0) part_hop[j] = h0;
    }
}

// per-hop deterministic sum of the segment pieces (segment order)
__global__ void __launch_bounds__(AMX_BLOCK) k_hops(const SpanDev *__restrict__ spans,
                                                    const KwSegDev *__restrict__ ks, int L,
                                                    int hop, const double *__restrict__ parts,
                                                    const int64_t *__restrict__ part_hop,
                                                    double *__restrict__ hops, int64_t max_hops) {
    const int t = blockIdx.y;
    const SpanDev sp = spans[t];
    if (sp.nkseg == 0) return;
    const int64_t hfirst = sp.tframe0 / hop;
    const int64_t hlast = (sp.tframe0 + sp.out_n - 1) / hop;
    const int64_t h = hfirst + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h > hlast || h >= max_hops) return;
    // span-local frame range of hop h
    int64_t a = h * hop - sp.tframe0, bnd = (h + 1) * hop - sp.tframe0;
    if (a < 0) a = 0;
    if (bnd > sp.out_n) bnd = sp.out_n;
    const int64_t j0 = a / L, j1 = (bnd - 1) / L;
    double s0 = 0.0, s1 = 0.0;
    for (int64_t jj = j0; jj <= j1; jj++) {
        const int64_t j = sp.kseg0 + jj;
        const int pc = part_hop[j] == h ? 0 : 1;
        s0 += parts[j * 4 + 2 * pc];
        s1 += parts[j * 4 + 2 * pc + 1];
    }
    hops[((int64_t)t * max_hops + h) * 2] = s0;
    hops[((int64_t)t * max_hops + h) * 2 + 1] = s1;
}

__device__ __forceinline__ int find_bin(const double *bounds, double energy) {
    int lo = 0, hi = 1000;
    do {
        int mid = (lo + hi) / 2;
        if (energy >= bounds[mid]) lo = mid; else hi = mid;
    } while (hi - lo != 1);
    return lo;
}

// gating blocks (400 ms every 100 ms) and short-term blocks (3 s every 1 s)
__global__ void __launch_bounds__(AMX_BLOCK) k_hist(const SpanDev *__restrict__ spans, int hop,
                                                    const double *__restrict__ hops,
                                                    int64_t max_hops,
                                                    const double *__restrict__ bounds,
                                                    unsigned long long *__restrict__ hist,
                                                    unsigned long long *__restrict__ st_hist) {
    const int t = blockIdx.y;
    const SpanDev sp = spans[t];
    int64_t nh = sp.ttotal / hop;
    if (nh > max_hops) nh = max_hops;
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double *H = hops + (int64_t)t * max_hops * 2;
    if (k + 4 <= nh) {
        double c0 = ((H[2 * k] + H[2 * (k + 1)]) + H[2 * (k + 2)]) + H[2 * (k + 3)];
        double c1 = ((H[2 * k + 1] + H[2 * (k + 1) + 1]) + H[2 * (k + 2) + 1]) + H[2 * (k + 3) + 1];
        double en = (c0 + c1) / (double)(4 * (int64_t)hop);
        if (en >= bounds[0]) atomicAdd(hist + (int64_t)t * AMX_HIST_BINS + find_bin(bounds, en), 1ull);
    }
    // short-term block m ends at hop 30 + 10 m
    const int64_t end = 30 + 10 * k;
    if (end <= nh) {
        double c0 = 0.0, c1 = 0.0;
        for (int64_t h = end - 30; h < end; h++) { c0 += H[2 * h]; c1 += H[2 * h + 1]; }
        double en = (c0 + c1) / (double)(30 * (int64_t)hop);
        if (en >= bounds[0])
            atomicAdd(st_hist + (int64_t)t * AMX_HIST_BINS + find_bin(bounds, en), 1ull);
    }
}

// ================================================================ launchers
hipError_t launch_kw1(const ChainDev *cd, const KwSegDev *ks, int n_kseg, int L,
                      const int16_t *x, const double *G, double *e, unsigned long long *peak,
                      hipStream_t st) {
    (void)cd;
    if (n_kseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_kw1, grid1(n_kseg), dim3(AMX_BLOCK), 0, st, ks, n_kseg, L,
                       reinterpret_cast<const uint32_t *>(x), G, e, peak);
    return hipGetLastError();
}

hipError_t launch_kw2(const ChainDev *cd, const KwSegDev *ks, int n_kseg, int L, int hop,
                      const int16_t *x, const double *s, double *parts, int64_t *part_hop,
                      hipStream_t st) {
    if (n_kseg <= 0) return hipSuccess;
    const dim3 grid((unsigned)((n_kseg + AMX_BLOCK / 2 - 1) / (AMX_BLOCK / 2)));
    hipLaunchKernelGGL(k_kw2, grid, dim3(AMX_BLOCK), 0, st, cd, ks, n_kseg, L, hop,
                       reinterpret_cast<const uint32_t *>(x), s, parts, part_hop);
    return hipGetLastError();
}

hipError_t launch_hops(const SpanDev *spans, int n_tracks, const KwSegDev *ks, int L, int hop,
                       const double *parts, const int64_t *part_hop, double *hops,
                       int64_t max_hops, hipStream_t st) {
    dim3 g = grid1(max_hops);
    g.y = (unsigned)n_tracks;
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_hops, g, dim3(AMX_BLOCK), 0, st, spans, ks, L, hop, parts, part_hop,
                       hops, max_hops);
    return hipGetLastError();
}

hipError_t launch_hist(const SpanDev *spans, int n_tracks, int hop, const double *hops,
                       int64_t max_hops, const double *bounds, unsigned long long *hist,
                       unsigned long long *st_hist, hipStream_t st) {
    dim3 g = grid1(max_hops);
    g.y = (unsigned)n_tracks;
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_hist, g, dim3(AMX_BLOCK), 0, st, spans, hop, hops, max_hops, bounds,
                       hist, st_hist);
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

}  // namespace amx

