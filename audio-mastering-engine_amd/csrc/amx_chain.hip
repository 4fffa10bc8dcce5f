// amx_chain.hip -- the per-chunk linear chain on CDNA4 (gfx950):
//   quantise (A.1) -> analog character (:258-266) -> 4-stage EQ (:272-298)
//   -> width (:267-271) -> int16 (:254-257) [-> crossover bands (:300-305)]
//
// Every IIR runs time-parallel by a 2-pass state-space method:
// pass 1 = zero-state end state of each segment as a GEMV e = G x (independent
// FMAs, G rows wave-uniform -> scalar loads); a Kogge-Stone affine scan with
// precomputed powers of M = A^L gives the exact segment start states; pass 2
// re-runs the recursion from the true state.  Chunks restart from rest
// (:185-204).  Memory-less stages keep the reference's float32/float64 operation
// order exactly (-ffp-contract=off; FMAs only inside the IIR recursions).
// Segment kernels stream their rows through LDS tiles (amx_dev.hpp tile_load /
// tile_store): coalesced dword traffic, recursion reads from LDS.
#include "amx_dev.hpp"

namespace amx {

__device__ __forceinline__ void decode_in(const ChainDev &cd, const uint32_t *row, int f,
                                          int win, int16_t &l, int16_t &r) {
    if (win == 2) {
        l = q_f32_to_s16_ffmpeg(__uint_as_float(row[2 * f]));
        r = q_f32_to_s16_ffmpeg(__uint_as_float(row[2 * f + 1]));
    } else {
        const uint32_t w = row[f];
        if (cd.in_s16) {
            l = lo16(w);
            r = hi16(w);
        } else {
            l = r = q_f32_to_s16_ffmpeg(__uint_as_float(w));   // mono duplicated (:190)
        }
    }
}

// ------------------------------------------------ pass 1: quantise/analog + GEMV
template <int MASK, int WIN>
__global__ void __launch_bounds__(AMX_BLOCK) k_front1(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const SegDev *__restrict__ segs, int n_seg,
                                                      int L, const uint32_t *__restrict__ in,
                                                      const float *__restrict__ lut,
                                                      uint32_t *__restrict__ a16,
                                                      const double *__restrict__ G,
                                                      double *__restrict__ e) {
    constexpr int D = EqDim<MASK>::v;
    __shared__ uint32_t s_in[Tile<WIN>::WORDS];
    __shared__ uint32_t s_out[Tile<1>::WORDS];
    __shared__ int64_t rb_in[AMX_BLOCK], rb_out[AMX_BLOCK];
    __shared__ int rl[AMX_BLOCK];
    const ChainDev &cd = *cdp;
    const int t = threadIdx.x;
    const int j = blockIdx.x * AMX_BLOCK + t;
    bool need_e = false;
    rb_in[t] = 0;
    rb_out[t] = 0;
    rl[t] = 0;
    if (j < n_seg) {
        const SegDev sg = segs[j];
        const ChunkDev ch = chunks[sg.chunk];
        rb_in[t] = (ch.in_off + sg.pos) * WIN;
        rb_out[t] = ch.loc_off + sg.pos;
        rl[t] = sg.len;
        need_e = !sg.last;
    }
    double e0[D > 0 ? D : 1], e1[D > 0 ? D : 1];
#pragma unroll
    for (int d = 0; d < D; d++) { e0[d] = 0.0; e1[d] = 0.0; }
    const int analog = cd.analog_on;
    __syncthreads();
    for (int k = 0; k < L; k += AMX_TF) {
        tile_load<WIN>(s_in, in, rb_in, nullptr, rl, k);
        __syncthreads();
        const uint32_t *row = s_in + t * Tile<WIN>::PITCH;
        uint32_t *orow = s_out + t * Tile<1>::PITCH;
        for (int f = 0; f < AMX_TF; f++) {
            int16_t l, r;
            decode_in(cd, row, f, WIN, l, r);
            if (analog) analog_frame(cd, lut, l, r, l, r);
            orow[f] = pack2(l, r);
            if constexpr (D > 0) {
                const double *g = G + (int64_t)(k + f) * D;   // wave-uniform row
                const double x0 = (double)((float)l / 32768.0f);
                const double x1 = (double)((float)r / 32768.0f);
#pragma unroll
                for (int d = 0; d < D; d++) {
                    e0[d] = fma(g[d], x0, e0[d]);
                    e1[d] = fma(g[d], x1, e1[d]);
                }
            }
        }
        __syncthreads();
        tile_store<1>(s_out, a16, rb_out, rl, k);
    }
    if constexpr (D > 0) {
        if (need_e) {
            double *o = e + (int64_t)j * 2 * D;
#pragma unroll
            for (int d = 0; d < D; d++) { o[d] = e0[d]; o[D + d] = e1[d]; }
        }
    }
}

// ------------------------------------------------------ Kogge-Stone affine scan
// x_j = carry (j == first) or e_{j-1};   s_j = sum_{k<K} M^k x_{j-k}  (same stream)
// One block = 256 consecutive entries of one lane; the first K-1 are halo.  Each
// thread keeps its entry's D-vector in registers; LDS only publishes it per level.
template <int D>
__global__ void __launch_bounds__(AMX_BLOCK) k_scan(const double *__restrict__ e,
                                                    double *__restrict__ s,
                                                    const int32_t *__restrict__ seg_first,
                                                    const int32_t *__restrict__ seg_stream,
                                                    int n_seg, int lanes,
                                                    const double *__restrict__ Mp, int levels,
                                                    const double *__restrict__ carry) {
    __shared__ double lds[AMX_BLOCK * D];
    const int K = 1 << levels;
    const int HALO = K - 1;
    const int OUT = blockDim.x - HALO;
    const int lane = blockIdx.y;
    const int t = threadIdx.x;
    const int64_t j = (int64_t)blockIdx.x * OUT - HALO + t;
    double v[D], nb[D];
    int first = 0x7fffffff;
    const bool in = j >= 0 && j < n_seg;
    if (in) first = seg_first[j];
#pragma unroll
    for (int d = 0; d < D; d++) {
        double x = 0.0;
        if (in) {
            if (j == first) x = carry ? carry[((int64_t)seg_stream[j] * lanes + lane) * D + d] : 0.0;
            else x = e[((j - 1) * lanes + lane) * D + d];
        }
        v[d] = x;
    }
    for (int l = 0; l < levels; l++) {
        const int off = 1 << l;
#pragma unroll
        for (int d = 0; d < D; d++) lds[t * D + d] = v[d];
        __syncthreads();
        const bool use = (t - off >= 0) && (j - off >= first) && in;
        if (use) {
#pragma unroll
            for (int d = 0; d < D; d++) nb[d] = lds[(t - off) * D + d];
        }
        __syncthreads();
        if (use) {
            const double *M = Mp + (int64_t)l * D * D;
#pragma unroll
            for (int i = 0; i < D; i++) {
                double acc = v[i];
#pragma unroll
                for (int k = 0; k < D; k++) acc = fma(M[i * D + k], nb[k], acc);
                v[i] = acc;
            }
        }
    }
    if (t >= HALO && in)
#pragma unroll
        for (int d = 0; d < D; d++) s[(j * lanes + lane) * D + d] = v[d];
}

// ------------------------------------------- pass 2: EQ from true state -> int16
// MB: also accumulate the crossover's zero-state end state (GEMV) for its scan.
template <int MASK, bool MB>
__global__ void __launch_bounds__(AMX_BLOCK) k_front2(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const SegDev *__restrict__ segs, int n_seg,
                                                      int L, const uint32_t *__restrict__ a16,
                                                      const double *__restrict__ s_eq,
                                                      uint32_t *__restrict__ dst, int to_out,
                                                      const double *__restrict__ Gx,
                                                      double *__restrict__ e_x) {
    constexpr int D = EqDim<MASK>::v;
    __shared__ uint32_t s_in[Tile<1>::WORDS];
    __shared__ uint32_t s_out[Tile<1>::WORDS];
    __shared__ int64_t rb_in[AMX_BLOCK], rb_out[AMX_BLOCK];
    __shared__ int rl[AMX_BLOCK];
    const ChainDev &cd = *cdp;
    const int t = threadIdx.x;
    const int j = blockIdx.x * AMX_BLOCK + t;
    bool need_x = false;
    rb_in[t] = 0;
    rb_out[t] = 0;
    rl[t] = 0;
    double z0[D > 0 ? D : 1], z1[D > 0 ? D : 1];
#pragma unroll
    for (int d = 0; d < D; d++) { z0[d] = 0.0; z1[d] = 0.0; }
    if (j < n_seg) {
        const SegDev sg = segs[j];
        const ChunkDev ch = chunks[sg.chunk];
        rb_in[t] = ch.loc_off + sg.pos;
        rb_out[t] = (to_out ? ch.out_off : ch.loc_off) + sg.pos;
        rl[t] = sg.len;
        need_x = MB && !sg.last;
        if constexpr (D > 0) {
            const double *s = s_eq + (int64_t)j * 2 * D;
#pragma unroll
            for (int d = 0; d < D; d++) { z0[d] = s[d]; z1[d] = s[D + d]; }
        }
    }
    double x0v[MB ? AMX_XO_DIM : 1], x1v[MB ? AMX_XO_DIM : 1];
#pragma unroll
    for (int d = 0; d < (MB ? AMX_XO_DIM : 1); d++) { x0v[d] = 0.0; x1v[d] = 0.0; }
    const float w = cd.width;
    const int won = cd.width_on;
    __syncthreads();
    for (int k = 0; k < L; k += AMX_TF) {
        tile_load<1>(s_in, a16, rb_in, nullptr, rl, k);
        __syncthreads();
        const uint32_t *row = s_in + t * Tile<1>::PITCH;
        uint32_t *orow = s_out + t * Tile<1>::PITCH;
        for (int f = 0; f < AMX_TF; f++) {
            const uint32_t p = row[f];
            float l = (float)lo16(p) / 32768.0f, r = (float)hi16(p) / 32768.0f;
            l = eq_chain<MASK>(cd, z0, l);
            r = eq_chain<MASK>(cd, z1, r);
            if (won) width_frame(w, l, r);
            const int16_t ql = f32_to_s16(l), qr = f32_to_s16(r);
            orow[f] = pack2(ql, qr);
            if constexpr (MB) {
                const double *g = Gx + (int64_t)(k + f) * AMX_XO_DIM;
                const double xl = (double)((float)ql / 32768.0f);
                const double xr = (double)((float)qr / 32768.0f);
#pragma unroll
                for (int d = 0; d < AMX_XO_DIM; d++) {
                    x0v[d] = fma(g[d], xl, x0v[d]);
                    x1v[d] = fma(g[d], xr, x1v[d]);
                }
            }
        }
        __syncthreads();
        tile_store<1>(s_out, dst, rb_out, rl, k);
    }
    if constexpr (MB) {
        if (need_x) {
            double *o = e_x + (int64_t)j * 2 * AMX_XO_DIM;
#pragma unroll
            for (int d = 0; d < AMX_XO_DIM; d++) { o[d] = x0v[d]; o[AMX_XO_DIM + d] = x1v[d]; }
        }
    }
}

// ------------------------------------------------ crossover pass 2 -> 3 bands
__global__ void __launch_bounds__(AMX_BLOCK) k_xover2(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const SegDev *__restrict__ segs, int n_seg,
                                                      int L, const uint32_t *__restrict__ p16,
                                                      const double *__restrict__ s_x,
                                                      uint32_t *__restrict__ bands, int64_t nloc) {
    __shared__ uint32_t s_in[Tile<1>::WORDS];
    __shared__ uint32_t s_lo[Tile<1>::WORDS], s_mi[Tile<1>::WORDS], s_hi[Tile<1>::WORDS];
    __shared__ int64_t rb[AMX_BLOCK];
    __shared__ int rl[AMX_BLOCK];
    const ChainDev &cd = *cdp;
    const int t = threadIdx.x;
    const int j = blockIdx.x * AMX_BLOCK + t;
    double z[2][AMX_XO_DIM];
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int d = 0; d < AMX_XO_DIM; d++) z[c][d] = 0.0;
    rb[t] = 0;
    rl[t] = 0;
    if (j < n_seg) {
        const SegDev sg = segs[j];
        const ChunkDev ch = chunks[sg.chunk];
        rb[t] = ch.loc_off + sg.pos;
        rl[t] = sg.len;
        const double *s = s_x + (int64_t)j * 2 * AMX_XO_DIM;
#pragma unroll
        for (int c = 0; c < 2; c++)
#pragma unroll
            for (int d = 0; d < AMX_XO_DIM; d++) z[c][d] = s[c * AMX_XO_DIM + d];
    }
    __syncthreads();
    for (int k = 0; k < L; k += AMX_TF) {
        tile_load<1>(s_in, p16, rb, nullptr, rl, k);
        __syncthreads();
        const uint32_t *row = s_in + t * Tile<1>::PITCH;
        const int o = t * Tile<1>::PITCH;
        for (int f = 0; f < AMX_TF; f++) {
            const uint32_t p = row[f];
            int16_t lo[2], mi[2], hi[2];
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const int16_t v = c ? hi16(p) : lo16(p);
                const double x = (double)((float)v / 32768.0f);   // :300 float32 then float64
                double l = sos_step(cd.xlo, z[c][0], z[c][1], x);
                l = sos_step(cd.xlo + 6, z[c][2], z[c][3], l);
                double h = sos_step(cd.xhi, z[c][4], z[c][5], x);
                h = sos_step(cd.xhi + 6, z[c][6], z[c][7], h);
                const double m = (x - l) - h;                    // :304
                lo[c] = f64_to_s16(l);
                mi[c] = f64_to_s16(m);
                hi[c] = f64_to_s16(h);
            }
            s_lo[o + f] = pack2(lo[0], lo[1]);
            s_mi[o + f] = pack2(mi[0], mi[1]);
            s_hi[o + f] = pack2(hi[0], hi[1]);
        }
        __syncthreads();
        tile_store<1>(s_lo, bands, rb, rl, k);
        tile_store<1>(s_mi, bands + nloc, rb, rl, k);
        tile_store<1>(s_hi, bands + 2 * nloc, rb, rl, k);
    }
}

// ================================================================ launchers
template <int MASK, int WIN>
static hipError_t front1_t(const Launch &l, const uint32_t *in, const float *lut, uint32_t *a16,
                           const double *G, double *e) {
    hipLaunchKernelGGL((k_front1<MASK, WIN>), grid1(l.n_seg), dim3(AMX_BLOCK), 0, l.stream, l.cd,
                       l.chunks, l.segs, l.n_seg, l.L, in, lut, a16, G, e);
    return hipGetLastError();
}

template <int MASK, bool MB>
static hipError_t front2_t(const Launch &l, const uint32_t *a16, const double *s_eq,
                           uint32_t *dst, int to_out, const double *Gx, double *e_x) {
    hipLaunchKernelGGL((k_front2<MASK, MB>), grid1(l.n_seg), dim3(AMX_BLOCK), 0, l.stream, l.cd,
                       l.chunks, l.segs, l.n_seg, l.L, a16, s_eq, dst, to_out, Gx, e_x);
    return hipGetLastError();
}

#define AMX_MASK_CASES(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

hipError_t launch_front1_lut(const Launch &l, int mask, int win, const float *in, const float *lut,
                             int16_t *a16, const double *G, double *e) {
    if (l.n_seg <= 0) return hipSuccess;
    const uint32_t *i32 = reinterpret_cast<const uint32_t *>(in);
    uint32_t *a = reinterpret_cast<uint32_t *>(a16);
    if (win == 2) {
        switch (mask) {
#define C1(M) case M: return front1_t<M, 2>(l, i32, lut, a, G, e);
            AMX_MASK_CASES(C1)
#undef C1
        }
    } else {
        switch (mask) {
#define C1(M) case M: return front1_t<M, 1>(l, i32, lut, a, G, e);
            AMX_MASK_CASES(C1)
#undef C1
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_front2(const Launch &l, int mask, const int16_t *a16, const double *s_eq,
                         int16_t *dst, int to_out, const double *Gx, double *e_x) {
    if (l.n_seg <= 0) return hipSuccess;
    const uint32_t *a = reinterpret_cast<const uint32_t *>(a16);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    const bool mb = Gx != nullptr;
    switch (mask) {
#define C2(M) case M: return mb ? front2_t<M, true>(l, a, s_eq, d, to_out, Gx, e_x) \
                                : front2_t<M, false>(l, a, s_eq, d, to_out, Gx, e_x);
        AMX_MASK_CASES(C2)
#undef C2
    }
    return hipErrorInvalidValue;
}

template <int D>
static hipError_t scan_t(const double *e, double *s, const int32_t *seg_first,
                         const int32_t *seg_stream, int n_seg, int lanes, const double *Mp,
                         int levels, const double *carry, hipStream_t st) {
    const int K = 1 << levels;
    const int OUT = AMX_BLOCK - (K - 1);
    if (OUT <= 0) return hipErrorInvalidValue;
    dim3 grid((unsigned)((n_seg + OUT - 1) / OUT), (unsigned)lanes);
    hipLaunchKernelGGL(k_scan<D>, grid, dim3(AMX_BLOCK), 0, st, e, s, seg_first, seg_stream,
                       n_seg, lanes, Mp, levels, carry);
    return hipGetLastError();
}

hipError_t launch_scan(const double *e, double *s, const int32_t *seg_first,
                       const int32_t *seg_stream, int n_seg, int D, int lanes,
                       const double *Mp, int levels, const double *carry, hipStream_t st) {
    if (n_seg <= 0 || D <= 0) return hipSuccess;
    switch (D) {
#define SC(DD) case DD: return scan_t<DD>(e, s, seg_first, seg_stream, n_seg, lanes, Mp, levels, carry, st);
        SC(2) SC(4) SC(8) SC(10) SC(12) SC(16) SC(18) SC(20)
#undef SC
    }
    return hipErrorInvalidValue;
}

hipError_t launch_xover2(const Launch &l, const int16_t *p16, const double *s_x,
                         int16_t *bands, int64_t nloc) {
    if (l.n_seg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_xover2, grid1(l.n_seg), dim3(AMX_BLOCK), 0, l.stream, l.cd, l.chunks,
                       l.segs, l.n_seg, l.L, reinterpret_cast<const uint32_t *>(p16), s_x,
                       reinterpret_cast<uint32_t *>(bands), nloc);
    return hipGetLastError();
}

}  // namespace amx
