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
    TileRegs<1, ROWS> R;
    tile_fetch<1, ROWS>(R, x, rb, nullptr, rl, 0);
    for (int k = 0; k < L; k += AMX_TF) {
        tile_put<1, ROWS>(s_in, R, nullptr, rl, k);
        __syncthreads();
        if (k + AMX_TF < L) tile_fetch<1, ROWS>(R, x, rb, nullptr, rl, k + AMX_TF);
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

// per-hop sum of the segment pieces: one wave per hop, lanes over the hop's
// segments, then a fixed butterfly (deterministic for a given segment grid)
__global__ void __launch_bounds__(AMX_BLOCK) k_hops(const SpanDev *__restrict__ spans,
                                                    const KwSegDev *__restrict__ ks, int L,
                                                    int hop, const double *__restrict__ parts,
                                                    const int64_t *__restrict__ part_hop,
                                                    double *__restrict__ hops, int64_t max_hops) {
    const int t = blockIdx.y;
    const SpanDev sp = spans[t];
    if (sp.nkseg == 0) return;
    const int lane = threadIdx.x & 63;
    const int64_t hfirst = sp.tframe0 / hop;
    const int64_t hlast = (sp.tframe0 + sp.out_n - 1) / hop;
    const int64_t h = hfirst + (int64_t)blockIdx.x * (AMX_BLOCK / 64) + (threadIdx.x >> 6);
    if (h > hlast || h >= max_hops) return;          // wave-uniform
    // span-local frame range of hop h
    int64_t a = h * hop - sp.tframe0, bnd = (h + 1) * hop - sp.tframe0;
    if (a < 0) a = 0;
    if (bnd > sp.out_n) bnd = sp.out_n;
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
    dim3 g = grid1(max_hops);
    g.y = (unsigned)n_tracks;
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_hist, g, dim3(AMX_BLOCK), 0, st, spans, hop, hops, max_hops, bounds,
                       hist, st_hist);
    return hipGetLastError();
}


// Sample peak per track from the per-(segment, channel) maxima k_front2 wrote
// when it ran the loudness pass-1 work fused (pk[j][ch] = max |x|).
__global__ void __launch_bounds__(AMX_BLOCK) k_peak_reduce(const SpanDev *__restrict__ spans,
                                                           const uint32_t *__restrict__ pk,
                                                           unsigned long long *__restrict__ peak) {
    __shared__ int red[2][AMX_BLOCK / 64];
    const int t = blockIdx.x;
    const SpanDev sp = spans[t];
    int m0 = 0, m1 = 0;
    for (int q = threadIdx.x; q < sp.nkseg; q += AMX_BLOCK) {
        const int64_t j = (int64_t)sp.kseg0 + q;
        m0 = max(m0, (int)pk[j * 2]);
        m1 = max(m1, (int)pk[j * 2 + 1]);
    }
    for (int o = 32; o > 0; o >>= 1) {
        m0 = max(m0, __shfl_xor(m0, o));
        m1 = max(m1, __shfl_xor(m1, o));
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = m0;
        red[1][threadIdx.x >> 6] = m1;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        int m = 0;
        for (int w = 0; w < AMX_BLOCK / 64; w++) m = max(m, red[threadIdx.x][w]);
        const double p = (double)m * (1.0 / 32768.0);
        peak[2 * t + threadIdx.x] = (unsigned long long)__double_as_longlong(p);
    }
}

hipError_t launch_peak_reduce(const SpanDev *spans, int n_tracks, const uint32_t *pk,
                              unsigned long long *peak, hipStream_t st) {
    if (n_tracks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_peak_reduce, dim3(n_tracks), dim3(AMX_BLOCK), 0, st, spans, pk, peak);
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

// "%.2f" then float(): the exact decimal rounding (half-even on exact ties) of v
__device__ double round2(double v) {
    if (!isfinite(v)) return v;
    const double p = v * 100.0;
    const double err = fma(v, 100.0, -p);        // v*100 == p + err exactly
    double k = rint(p);
    if (fabs(p - k) == 0.5 && err != 0.0) k = err > 0.0 ? floor(p) + 1.0 : floor(p);
    return k / 100.0;
}

__device__ __forceinline__ double lufs_of(double e) { return 10 * log10(e) - 0.691; }

// Non-empty bins of h in ascending order -> nz (index), nc (count as double, exact
// below 2^53) and np (count * energy, the product libebur128 adds); returns how many.
__device__ int compact_bins(const unsigned long long *h, const double *E, short *nz, double *nc,
                            double *np) {
    constexpr int NB = (AMX_HIST_BINS + 63) / 64;
    const int lane = threadIdx.x;
    unsigned long long v[NB];
#pragma unroll
    for (int c = 0; c < NB; c++) {                 // every load in flight before the first use
        const int j = c * 64 + lane;
        v[c] = h[j < AMX_HIST_BINS ? j : AMX_HIST_BINS - 1];
        if (j >= AMX_HIST_BINS) v[c] = 0ull;
    }
    int n = 0;
#pragma unroll
    for (int c = 0; c < NB; c++) {
        const int j = c * 64 + lane;
        const unsigned long long m = __ballot(v[c] != 0ull);
        const int pos = __popcll(m & ((1ull << lane) - 1ull));
        if (v[c]) {
            nz[n + pos] = (short)j;
            nc[n + pos] = (double)v[c];
            np[n + pos] = (double)v[c] * E[j];
        }
        n += __popcll(m);
    }
    __syncthreads();
    return n;
}

__global__ void __launch_bounds__(64) k_decide(DecideArgs a) {
    __shared__ short nz[AMX_HIST_BINS];
    __shared__ double nc[AMX_HIST_BINS], np[AMX_HIST_BINS];
    const int t = blockIdx.x;
    const unsigned long long *H = a.hist + (int64_t)t * AMX_HIST_BINS;
    const unsigned long long *S = a.st_hist + (int64_t)t * AMX_HIST_BINS;
    const double *E = a.energies;
    double I = -INFINITY, thr = -70.0, lra = 0.0;
    if (a.lufs_on) {
        const int n = compact_bins(H, E, nz, nc, np);
        if (threadIdx.x == 0) {
            double rel = 0.0, cnt = 0.0;
            for (int q = 0; q < n; q++) {
                rel += np[q];
                cnt += nc[q];                          // exact: integer-valued < 2^53
            }
            if (cnt != 0.0) {
                rel /= cnt;
                rel *= 0.1;                            // pow(10, -10/10)
                thr = lufs_of(rel);
                int start;
                if (rel < a.bounds[0]) start = 0;
                else {
                    start = find_bin(a.bounds, rel);
                    if (rel > E[start]) ++start;
                }
                double g = 0.0, above = 0.0;
                for (int q = 0; q < n; q++) {
                    if (nz[q] < start) continue;
                    g += np[q];
                    above += nc[q];
                }
                if (above != 0.0) I = lufs_of(g / above);
            }
        }
        __syncthreads();
        const int m = compact_bins(S, E, nz, nc, np);
        if (threadIdx.x == 0) {
            double size = 0.0, power = 0.0;
            for (int q = 0; q < m; q++) {
                size += nc[q];
                power += np[q];
            }
            if (size != 0.0) {
                power /= size;
                const double integ = 0.01 * power;      // pow(10, -20/10)
                int index;
                if (integ < a.bounds[0]) index = 0;
                else {
                    index = find_bin(a.bounds, integ);
                    if (integ > E[index]) ++index;
                }
                size = 0.0;
                int q0 = 0;
                while (q0 < m && nz[q0] < index) q0++;
                for (int q = q0; q < m; q++) size += nc[q];
                if (size != 0.0) {
                    const double plo = (double)(int64_t)((size - 1) * 0.1 + 0.5);
                    const double phi = (double)(int64_t)((size - 1) * 0.95 + 0.5);
                    double acc = 0.0;
                    int q = q0, last = index;
                    while (acc <= plo) { last = nz[q]; acc += nc[q]; q++; }
                    const double l_en = E[last];
                    while (acc <= phi) { last = nz[q]; acc += nc[q]; q++; }
                    const double h_en = E[last];
                    lra = lufs_of(h_en) - lufs_of(l_en);
                }
            }
        }
    }
    if (threadIdx.x != 0) return;
    const double pk = fmax(a.peak[2 * t], a.peak[2 * t + 1]);
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
    const double m16 = rint(pk * 32768.0);
    double amax = m16 / 32768.0;
    if (gain > 0.0) amax = fmin(rint(((m16 * (1.0 / 32768.0)) * gain) * 32768.0), 32768.0) / 32768.0;
    const bool fast = amax * a.level_in <= a.limit;
    double *o = a.stats + (int64_t)t * AMX_STATS;
    o[0] = I; o[1] = lra; o[2] = thr; o[3] = tp;
    o[4] = si; o[5] = stp; o[6] = slra; o[7] = sthr;
    o[8] = (double)mode; o[9] = gain; o[10] = fast ? 1.0 : 0.0; o[11] = pk;
    a.gains[t] = gain;
    a.ctl[t] = (fast ? AMX_CTL_FAST : 0) | (mode << 4);
}

hipError_t launch_decide(const DecideArgs &a, hipStream_t st) {
    if (a.n_tracks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_decide, dim3(a.n_tracks), dim3(64), 0, st, a);
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

}  // namespace amx

