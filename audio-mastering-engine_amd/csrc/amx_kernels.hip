// amx_kernels.hip -- CDNA4 (gfx950) kernels of the mastering hot path.
//
// Design:
//  * Every IIR (EQ cascade :277-298, crossover :301-304, K-weighting) is run
//    time-parallel by a 2-pass state-space method: pass 1 computes each
//    segment's zero-state end state as a GEMV e = G x (no recursion, all FMAs
//    independent), a Kogge-Stone affine scan with precomputed powers of
//    M = A^L turns those into the exact segment start states, pass 2 re-runs the
//    recursion from the true state.  Chunks restart from zero state (:185-204).
//  * Memory-less stages (quantise A.1, analog character :258-266, width :267-271,
//    int16 conversions :254-257, overlay :309) reproduce the reference's
//    float32/float64 operation order exactly (built with -ffp-contract=off;
//    FMAs are written explicitly only inside the IIR recursions).
//  * The pydub compressor envelope (:306-308) is a non-linear recurrence: it is
//    evaluated speculatively per segment from a warm-up guess, then a per
//    (chunk, band) wave verifies segment hand-offs and re-runs mismatching
//    segments until the re-run coincides with the old trajectory.  The result is
//    bit-identical to the sequential loop.
//  * One thread owns both channels of a segment: interleaved stereo s16 frames are
//    one 32-bit load/store, float32 stereo input one 64-bit load.
#include "amx_internal.hpp"
#include <math.h>

namespace amx {

// ------------------------------------------------------------ helpers
__device__ __forceinline__ int16_t q_f32_to_s16_ffmpeg(float x) {
    // libswresample f32->s16: av_clip_int16(lrintf(x * 32768))   
    float v = rintf(x * 32768.0f);
    v = fminf(fmaxf(v, -32768.0f), 32767.0f);
    return (int16_t)(int)v;
}
__device__ __forceinline__ int16_t f32_to_s16(float x) {
    // float_array_to_audio_segment (:255-256) on float32 arrays
    float v = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
    v = v * 32767.0f;
    return (int16_t)(int)v;
}
__device__ __forceinline__ int16_t f64_to_s16(double x) {
    double v = x < -1.0 ? -1.0 : (x > 1.0 ? 1.0 : x);
    v = v * 32767.0;
    return (int16_t)(int)v;
}
__device__ __forceinline__ int16_t sat16(int v) {
    return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}
__device__ __forceinline__ uint32_t pack2(int16_t a, int16_t b) {
    return (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16);
}
__device__ __forceinline__ int16_t lo16(uint32_t v) { return (int16_t)(v & 0xffff); }
__device__ __forceinline__ int16_t hi16(uint32_t v) { return (int16_t)(v >> 16); }

// lfilter DF-II-T biquad step (scipy _linear_filter order, fused)
__device__ __forceinline__ double lf_step(const double *c, double &z0, double &z1, double x) {
    double y = fma(c[0], x, z0);
    z0 = fma(-c[4], y, fma(c[1], x, z1));
    z1 = fma(-c[5], y, c[2] * x);
    return y;
}
// sosfilt section step (scipy _sosfilt order, fused)
__device__ __forceinline__ double sos_step(const double *c, double &z0, double &z1, double x) {
    double y = fma(c[0], x, z0);
    z0 = fma(-c[4], y, fma(c[1], x, z1));
    z1 = fma(-c[5], y, c[2] * x);
    return y;
}

// analog character for one frame, exact reference op order (no FMA):
// lfilter along the channel axis (:264-265) = a length-2 sequence per frame.
__device__ __forceinline__ void analog_frame(const ChainDev &cd, const float *lut, int16_t l,
                                             int16_t r, int16_t &ol, int16_t &orr) {
    double x0, x1;
    if (lut) {
        x0 = (double)lut[(int)l + 32768];
        x1 = (double)lut[(int)r + 32768];
    } else {
        float a = ((float)l / 32768.0f) * cd.drive, b = ((float)r / 32768.0f) * cd.drive;
        x0 = (double)(float)tanh((double)a);
        x1 = (double)(float)tanh((double)b);
    }
    const double *b1 = cd.an_lo, *b2 = cd.an_hi;
    // first shelf (120 Hz low, +cf dB): y0 = 0 + b0*x0 ; Z0 = (0 + x0*b1) - y0*a1 ; y1 = Z0 + b0*x1
    double y0 = 0.0 + b1[0] * x0;
    double z0 = (0.0 + x0 * b1[1]) - y0 * b1[4];
    double y1 = z0 + b1[0] * x1;
    double u0 = x0 + (y0 - x0) * cd.an_glo1;
    double u1 = x1 + (y1 - x1) * cd.an_glo1;
    double v0 = 0.0 + b2[0] * u0;
    double w = (0.0 + u0 * b2[1]) - v0 * b2[4];
    double v1 = w + b2[0] * u1;
    double o0 = u0 + (v0 - u0) * cd.an_ghi1;
    double o1 = u1 + (v1 - u1) * cd.an_ghi1;
    ol = f64_to_s16(o0);
    orr = f64_to_s16(o1);
}

// chain input frame: quantise (A.1, mono duplicated :190) + analog (:192)
__device__ __forceinline__ uint32_t front_frame(const ChainDev &cd, const float *lut,
                                                const float *in, int64_t f) {
    int16_t l, r;
    if (cd.in_s16) {
        const int16_t *in16 = reinterpret_cast<const int16_t *>(in);
        if (cd.chin == 2) {
            uint32_t v = *reinterpret_cast<const uint32_t *>(in16 + 2 * f);
            l = lo16(v);
            r = hi16(v);
        } else {
            l = r = in16[f];
        }
    } else if (cd.chin == 2) {
        float2 v = *reinterpret_cast<const float2 *>(in + 2 * f);
        l = q_f32_to_s16_ffmpeg(v.x);
        r = q_f32_to_s16_ffmpeg(v.y);
    } else {
        l = r = q_f32_to_s16_ffmpeg(in[f]);
    }
    if (cd.analog_on) analog_frame(cd, lut, l, r, l, r);
    return pack2(l, r);
}

// --------------------------------------------------------------- EQ chain
template <int MASK>
struct EqDim {
    static constexpr int v = ((MASK & 1) ? 2 : 0) + ((MASK & 2) ? 8 : 0) + ((MASK & 4) ? 8 : 0) +
                             ((MASK & 8) ? 2 : 0);
};

// One channel: z holds the compact state (active stages in order).
// Stage k is the first active stage (float32 input) iff no lower bit of MASK is set.
template <int MASK>
__device__ __forceinline__ float eq_chain(const ChainDev &cd, double *z, float xf) {
    double x = (double)xf;
    int o = 0;
    if constexpr ((MASK & 1) != 0) {
        const EqStageDev &s = cd.st[0];
        double y = lf_step(s.c, z[o], z[o + 1], x);
        if (!s.neg) x = x + (y - x) * s.gm1;
        else { double xg = (double)(xf * s.gf); x = xg + (y - xg); }
        o += 2;
    }
    if constexpr ((MASK & 2) != 0) {
        const EqStageDev &s = cd.st[1];
        double b = x;
#pragma unroll
        for (int k = 0; k < 4; k++) b = sos_step(s.c + 6 * k, z[o + 2 * k], z[o + 2 * k + 1], b);
        x = x + b * s.gm1;
        o += 8;
    }
    if constexpr ((MASK & 4) != 0) {
        const EqStageDev &s = cd.st[2];
        double b = x;
#pragma unroll
        for (int k = 0; k < 4; k++) b = sos_step(s.c + 6 * k, z[o + 2 * k], z[o + 2 * k + 1], b);
        x = x + b * s.gm1;
        o += 8;
    }
    if constexpr ((MASK & 8) != 0) {
        const EqStageDev &s = cd.st[3];
        double y = lf_step(s.c, z[o], z[o + 1], x);
        if (!s.neg) x = x + (y - x) * s.gm1;
        else if constexpr ((MASK & 7) == 0) { double xg = (double)(xf * s.gf); x = xg + (y - xg); }
        else { double xg = x * s.g; x = xg + (y - xg); }
        o += 2;
    }
    (void)o;
    if constexpr (MASK == 0) return xf;
    return (float)x;
}
// stage-1/2 "first" cases: a peak stage has no float32-sensitive op, and the
// stage-0 shelf is always first; only stage 3 needs the (MASK & 7) test above.

__device__ __forceinline__ void width_frame(float w, float &l, float &r) {
    // apply_stereo_width (:269-270), float32, exact order
    float mid = (l + r) / 2.0f, side = (l - r) / 2.0f;
    side = side * w;
    float nl = mid + side, nr = mid - side;
    l = nl < -1.0f ? -1.0f : (nl > 1.0f ? 1.0f : nl);
    r = nr < -1.0f ? -1.0f : (nr > 1.0f ? 1.0f : nr);
}

// ------------------------------------------------ pass 1: quantise/analog + GEMV
// e[seg][ch][D] = sum_n G[n][:] * x_n   (zero-state end state of the chain)
template <int MASK>
__global__ void __launch_bounds__(AMX_BLOCK) k_front1(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const SegDev *__restrict__ segs, int n_seg,
                                                      int L, const float *__restrict__ in,
                                                      const float *__restrict__ lut,
                                                      uint32_t *__restrict__ a16,
                                                      const double *__restrict__ G,
                                                      double *__restrict__ e) {
    constexpr int D = EqDim<MASK>::v;
    const ChainDev &cd = *cdp;
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_seg) return;
    const SegDev sg = segs[j];
    const ChunkDev ch = chunks[sg.chunk];
    const int64_t f0 = ch.in_off + sg.pos;
    uint32_t *dst = a16 + ch.loc_off + sg.pos;
    double e0[D > 0 ? D : 1], e1[D > 0 ? D : 1];
#pragma unroll
    for (int d = 0; d < D; d++) { e0[d] = 0.0; e1[d] = 0.0; }
    const bool need_e = (D > 0) && !sg.last;
    const int len = sg.len;
    for (int n = 0; n < len; n++) {
        uint32_t p = front_frame(cd, lut, in, f0 + n);
        dst[n] = p;
        if constexpr (D > 0) {
            if (need_e) {
                double x0 = (double)((float)lo16(p) / 32768.0f);
                double x1 = (double)((float)hi16(p) / 32768.0f);
                const double *g = G + (int64_t)n * D;
#pragma unroll
                for (int d = 0; d < D; d++) {
                    e0[d] = fma(g[d], x0, e0[d]);
                    e1[d] = fma(g[d], x1, e1[d]);
                }
            }
        }
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
                                                      const uint32_t *__restrict__ a16,
                                                      const double *__restrict__ s_eq,
                                                      uint32_t *__restrict__ dst, int to_out,
                                                      const double *__restrict__ Gx,
                                                      double *__restrict__ e_x) {
    constexpr int D = EqDim<MASK>::v;
    const ChainDev &cd = *cdp;
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_seg) return;
    const SegDev sg = segs[j];
    const ChunkDev ch = chunks[sg.chunk];
    const uint32_t *src = a16 + ch.loc_off + sg.pos;
    uint32_t *out = dst + (to_out ? ch.out_off : ch.loc_off) + sg.pos;
    double z0[D > 0 ? D : 1], z1[D > 0 ? D : 1];
    if constexpr (D > 0) {
        const double *s = s_eq + (int64_t)j * 2 * D;
#pragma unroll
        for (int d = 0; d < D; d++) { z0[d] = s[d]; z1[d] = s[D + d]; }
    }
    double x0v[AMX_XO_DIM], x1v[AMX_XO_DIM];
#pragma unroll
    for (int d = 0; d < AMX_XO_DIM; d++) { x0v[d] = 0.0; x1v[d] = 0.0; }
    const bool need_x = MB && !sg.last;
    const int len = sg.len;
    const float w = cd.width;
    const int won = cd.width_on;
    for (int n = 0; n < len; n++) {
        uint32_t p = src[n];
        float l = (float)lo16(p) / 32768.0f, r = (float)hi16(p) / 32768.0f;
        l = eq_chain<MASK>(cd, z0, l);
        r = eq_chain<MASK>(cd, z1, r);
        if (won) width_frame(w, l, r);
        int16_t ql = f32_to_s16(l), qr = f32_to_s16(r);
        out[n] = pack2(ql, qr);
        if constexpr (MB) {
            if (need_x) {
                double xl = (double)((float)ql / 32768.0f), xr = (double)((float)qr / 32768.0f);
                const double *g = Gx + (int64_t)n * AMX_XO_DIM;
#pragma unroll
                for (int d = 0; d < AMX_XO_DIM; d++) {
                    x0v[d] = fma(g[d], xl, x0v[d]);
                    x1v[d] = fma(g[d], xr, x1v[d]);
                }
            }
        }
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
                                                      const uint32_t *__restrict__ p16,
                                                      const double *__restrict__ s_x,
                                                      uint32_t *__restrict__ bands, int64_t nloc) {
    const ChainDev &cd = *cdp;
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_seg) return;
    const SegDev sg = segs[j];
    const ChunkDev ch = chunks[sg.chunk];
    double z[2][AMX_XO_DIM];
    const double *s = s_x + (int64_t)j * 2 * AMX_XO_DIM;
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int d = 0; d < AMX_XO_DIM; d++) z[c][d] = s[c * AMX_XO_DIM + d];
    const int64_t base = ch.loc_off + sg.pos;
    for (int n = 0; n < sg.len; n++) {
        uint32_t p = p16[base + n];
        int16_t lo[2], mi[2], hi[2];
#pragma unroll
        for (int c = 0; c < 2; c++) {
            int16_t v = c ? hi16(p) : lo16(p);
            double x = (double)((float)v / 32768.0f);      // :300 float32 then float64
            double l = sos_step(cd.xlo, z[c][0], z[c][1], x);
            l = sos_step(cd.xlo + 6, z[c][2], z[c][3], l);
            double h = sos_step(cd.xhi, z[c][4], z[c][5], x);
            h = sos_step(cd.xhi + 6, z[c][6], z[c][7], h);
            double m = (x - l) - h;                        // :304
            lo[c] = f64_to_s16(l);
            mi[c] = f64_to_s16(m);
            hi[c] = f64_to_s16(h);
        }
        bands[base + n] = pack2(lo[0], lo[1]);
        bands[nloc + base + n] = pack2(mi[0], mi[1]);
        bands[2 * nloc + base + n] = pack2(hi[0], hi[1]);
    }
}

// --------------------------------------------- compressor RMS detector (exact)
// r_i = audioop.rms of frames [max(i-look,0), i) of the band, both channels:
// (unsigned)sqrt(S / count) with S the exact integer sum of squares.
__global__ void __launch_bounds__(AMX_BLOCK) k_rms(const ChainDev *__restrict__ cdp,
                                                   const ChunkDev *__restrict__ chunks,
                                                   const SegDev *__restrict__ segs, int n_seg,
                                                   const uint32_t *__restrict__ bands,
                                                   uint16_t *__restrict__ rr, int64_t nloc) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    int b = blockIdx.y;
    if (j >= n_seg) return;
    const int look = cdp->look;
    const SegDev sg = segs[j];
    const ChunkDev ch = chunks[sg.chunk];
    const uint32_t *x = bands + b * nloc + ch.loc_off;
    uint16_t *r = rr + b * nloc + ch.loc_off;
    const int64_t p0 = sg.pos;
    int64_t lo = p0 - look < 0 ? 0 : p0 - look;
    int64_t S = 0;
    for (int64_t f = lo; f < p0; f++) {
        uint32_t v = x[f];
        int64_t a = lo16(v), c = hi16(v);
        S += a * a + c * c;
    }
    for (int n = 0; n < sg.len; n++) {
        int64_t i = p0 + n;
        int64_t wlo = i - look < 0 ? 0 : i - look;
        int64_t cnt = 2 * (i - wlo);
        uint32_t rms = cnt ? (uint32_t)sqrt((double)S / (double)cnt) : 0u;
        r[i] = (uint16_t)(rms > 65535u ? 65535u : rms);
        // slide: add frame i, drop frame i-look
        uint32_t v = x[i];
        int64_t a = lo16(v), c = hi16(v);
        S += a * a + c * c;
        if (i - look >= 0) {
            uint32_t u = x[i - look];
            int64_t a2 = lo16(u), c2 = hi16(u);
            S -= a2 * a2 + c2 * c2;
        }
    }
}

// pydub envelope step (compress_dynamic_range inner loop), exact.
__device__ __forceinline__ double env_step(double att, bool over, double m, double inc,
                                           double dec) {
    if (over && att <= m) {
        att = att + inc;
        att = (m < att) ? m : att;          // min(attenuation, max_attenuation)
    } else {
        att = att - dec;
        att = (0.0 > att) ? 0.0 : att;      // max(attenuation, 0)
    }
    return att;
}

#define AMX_TAB 32769
// speculative envelope: guess from a warm-up started at att = 0
__global__ void __launch_bounds__(AMX_BLOCK) k_env(const ChainDev *__restrict__ cdp,
                                                   const ChunkDev *__restrict__ chunks,
                                                   const SegDev *__restrict__ segs, int n_seg,
                                                   const uint16_t *__restrict__ rr,
                                                   const double *__restrict__ tabs,
                                                   double *__restrict__ att_out,
                                                   double *__restrict__ guess,
                                                   double *__restrict__ endv, int64_t nloc,
                                                   int warm) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    int b = blockIdx.y;
    if (j >= n_seg) return;
    const SegDev sg = segs[j];
    const ChunkDev ch = chunks[sg.chunk];
    const uint16_t *r = rr + b * nloc + ch.loc_off;
    double *ao = att_out + b * nloc + ch.loc_off;
    const double *mt = tabs + (int64_t)b * 3 * AMX_TAB;
    const double *it = mt + AMX_TAB, *dt = mt + 2 * AMX_TAB;
    const int rthr = cdp->rthr[b];
    double att = 0.0;
    int64_t w0 = sg.pos - warm;
    if (w0 < 0) w0 = 0;
    for (int64_t f = w0; f < sg.pos; f++) {
        int rv = r[f];
        att = env_step(att, rv >= rthr, mt[rv], it[rv], dt[rv]);
    }
    guess[(int64_t)b * n_seg + j] = att;
    for (int n = 0; n < sg.len; n++) {
        int rv = r[sg.pos + n];
        att = env_step(att, rv >= rthr, mt[rv], it[rv], dt[rv]);
        ao[sg.pos + n] = att;
    }
    endv[(int64_t)b * n_seg + j] = att;
}

// verification / fix-up: one wave per (chunk, band).  Walks the chunk's segment
// hand-offs; each mismatch (guess_j != end_{j-1}) is re-run from the exact start
// until the new trajectory coincides with the stored one.
__global__ void __launch_bounds__(64) k_fix(const ChainDev *__restrict__ cdp,
                                            const ChunkDev *__restrict__ chunks,
                                            const SegDev *__restrict__ segs, int n_seg,
                                            const uint16_t *__restrict__ rr,
                                            const double *__restrict__ tabs,
                                            double *__restrict__ att_arr,
                                            double *__restrict__ guess,
                                            double *__restrict__ endv, int64_t nloc) {
    const int c = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    const ChunkDev ch = chunks[c];
    const uint16_t *r = rr + b * nloc + ch.loc_off;
    double *aa = att_arr + b * nloc + ch.loc_off;
    double *gs = guess + (int64_t)b * n_seg;
    double *en = endv + (int64_t)b * n_seg;
    const double *mt = tabs + (int64_t)b * 3 * AMX_TAB;
    const double *it = mt + AMX_TAB, *dt = mt + 2 * AMX_TAB;
    const int rthr = cdp->rthr[b];
    const int s0 = ch.seg0, s1 = ch.seg0 + ch.nseg;
    int cur = s0 + 1;
    while (true) {
        int found = 0x7fffffff;
        for (int base = cur; base < s1; base += 64) {
            int jj = base + lane;
            bool bad = false;
            if (jj < s1) bad = !(gs[jj] == en[jj - 1]);
            unsigned long long m = __ballot(bad);
            if (m) { found = base + __ffsll((long long)m) - 1; break; }
        }
        if (found >= s1) break;
        const SegDev sg = segs[found];
        double att = en[found - 1];
        bool coincided = false;
        for (int base = 0; base < sg.len && !coincided; base += 64) {
            const int n = base + lane;
            const bool valid = n < sg.len;
            const int64_t f = sg.pos + n;
            int rv = valid ? (int)r[f] : 0;
            double mv = mt[rv], iv = it[rv], dv = dt[rv];
            bool over = valid && rv >= rthr;
            double old = valid ? aa[f] : 0.0;
            double nv;
            if (__ballot(over) == 0ull) {
                nv = att;                       // below threshold: state held
            } else {
                nv = 0.0;
                const int cnt = sg.len - base < 64 ? sg.len - base : 64;
                for (int k = 0; k < cnt; k++) {
                    double mk = __shfl(mv, k), ik = __shfl(iv, k), dk = __shfl(dv, k);
                    int ok = __shfl((int)over, k);
                    att = env_step(att, ok != 0, mk, ik, dk);
                    if (lane == k) nv = att;
                }
            }
            unsigned long long same = __ballot(valid && nv == old);
            if (same) {
                int k = __ffsll((long long)same) - 1;
                if (valid && lane < k) aa[f] = nv;
                coincided = true;
            } else if (valid) {
                aa[f] = nv;
            }
        }
        if (!coincided && lane == 0) en[found] = att;
        if (lane == 0) gs[found] = en[found - 1];
        __threadfence_block();
        __syncthreads();
        cur = found + 1;
    }
}

// audioop.mul clamp + floor (CPython Modules/audioop.c fbound)
__device__ __forceinline__ int mul16(int v, double f) {
    double val = (double)v * f;
    if (val > 32767.0) val = 32767.0;
    else if (val < -32768.0 + 1.0) val = -32768.0;
    return (int)floor(val);
}

// gains + overlay (:306-309) -> chunk output (pydub ms-rounded length)
__global__ void __launch_bounds__(AMX_BLOCK) k_apply(const ChunkDev *__restrict__ chunks,
                                                     const uint32_t *__restrict__ bands,
                                                     const double *__restrict__ att,
                                                     uint32_t *__restrict__ out, int64_t nloc,
                                                     const int64_t *__restrict__ n2tab) {
    const int c = blockIdx.y;
    const ChunkDev ch = chunks[c];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n2 = ch.out_n;            // final (second overlay) length
    if (i >= n2) return;
    const int64_t n1 = n2tab[c];            // first overlay length
    uint32_t res = 0;
    if (i < ch.n) {
        int acc[3][2];
#pragma unroll
        for (int b = 0; b < 3; b++) {
            uint32_t v = bands[b * nloc + ch.loc_off + i];
            double a = att[b * nloc + ch.loc_off + i];
            int l = lo16(v), r = hi16(v);
            if (a != 0.0) {
                double f = exp10(-a / 20.0);
                l = mul16(l, f);
                r = mul16(r, f);
            }
            acc[b][0] = l;
            acc[b][1] = r;
        }
        int16_t o[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            int s1 = i < n1 ? (int)sat16(acc[0][k] + acc[1][k]) : 0;
            o[k] = sat16(s1 + acc[2][k]);
        }
        res = pack2(o[0], o[1]);
    }
    out[ch.out_off + i] = res;
}

// ----------------------------------------------------------------- loudness
// K-weighting pass 1: zero-state end state GEMV + sample peak
__global__ void __launch_bounds__(AMX_BLOCK) k_kw1(const KwSegDev *__restrict__ ks, int n_kseg,
                                                   int L, const uint32_t *__restrict__ x,
                                                   const double *__restrict__ G,
                                                   double *__restrict__ e,
                                                   unsigned long long *__restrict__ peak) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_kseg) return;
    const KwSegDev sg = ks[j];
    double e0[AMX_KW_DIM], e1[AMX_KW_DIM];
#pragma unroll
    for (int d = 0; d < AMX_KW_DIM; d++) { e0[d] = 0.0; e1[d] = 0.0; }
    int m0 = 0, m1 = 0;
    const uint32_t *src = x + sg.out_pos;
    const int shift = L - sg.len;   // partial segment: use the tail of G
    for (int n = 0; n < sg.len; n++) {
        uint32_t p = src[n];
        int a = lo16(p), b = hi16(p);
        m0 = max(m0, abs(a));
        m1 = max(m1, abs(b));
        double xa = (double)a * (1.0 / 32768.0), xb = (double)b * (1.0 / 32768.0);
        const double *g = G + (int64_t)(n + shift) * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) {
            e0[d] = fma(g[d], xa, e0[d]);
            e1[d] = fma(g[d], xb, e1[d]);
        }
    }
    double *o = e + (int64_t)j * 2 * AMX_KW_DIM;
#pragma unroll
    for (int d = 0; d < AMX_KW_DIM; d++) { o[d] = e0[d]; o[AMX_KW_DIM + d] = e1[d]; }
    double p0 = (double)m0 * (1.0 / 32768.0), p1 = (double)m1 * (1.0 / 32768.0);
    atomicMax(peak + 2 * sg.track, (unsigned long long)__double_as_longlong(p0));
    atomicMax(peak + 2 * sg.track + 1, (unsigned long long)__double_as_longlong(p1));
}

// K-weighting pass 2: filter from the true state, y^2 summed per 100 ms hop piece.
// parts[j][piece][ch], part_hop[j] = whole-track hop index of piece 0.
__global__ void __launch_bounds__(AMX_BLOCK) k_kw2(const ChainDev *__restrict__ cdp,
                                                   const KwSegDev *__restrict__ ks, int n_kseg,
                                                   int hop, const uint32_t *__restrict__ x,
                                                   const double *__restrict__ s,
                                                   double *__restrict__ parts,
                                                   int64_t *__restrict__ part_hop) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_kseg) return;
    const ChainDev &cd = *cdp;
    const KwSegDev sg = ks[j];
    double v[2][4];
    const double *st = s + (int64_t)j * 2 * AMX_KW_DIM;
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int d = 0; d < 4; d++) v[c][d] = st[c * 4 + d];
    const int64_t h0 = sg.tframe / hop;
    int64_t next_b = (h0 + 1) * hop;   // next hop boundary (whole-track frame)
    double acc[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    int piece = 0;
    const uint32_t *src = x + sg.out_pos;
    for (int n = 0; n < sg.len; n++) {
        if (sg.tframe + n == next_b) { piece = 1; next_b += hop; }
        uint32_t p = src[n];
#pragma unroll
        for (int c = 0; c < 2; c++) {
            double xs = (double)(c ? hi16(p) : lo16(p)) * (1.0 / 32768.0);
            double u = sos_step(cd.kw1, v[c][0], v[c][1], xs);
            double y = sos_step(cd.kw2, v[c][2], v[c][3], u);
            acc[piece][c] = fma(y, y, acc[piece][c]);
        }
    }
    double *o = parts + (int64_t)j * 4;
    o[0] = acc[0][0]; o[1] = acc[0][1]; o[2] = acc[1][0]; o[3] = acc[1][1];
    part_hop[j] = h0;
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

// ----------------------------------------------------------------- finalize
__device__ __forceinline__ int16_t clip_llrint(double v) {
    double q = rint(v);
    q = q > 32767.0 ? 32767.0 : (q < -32768.0 ? -32768.0 : q);
    return (int16_t)(int)q;
}
__device__ __forceinline__ int16_t gain16(int16_t x, double g) {
    // loudnorm linear mode: dst = src * gain on doubles x/32768 ; s16 llrint(x*32768)
    if (g <= 0.0) return x;
    double v = ((double)x * (1.0 / 32768.0)) * g;
    return clip_llrint(v * 32768.0);
}

// limiter never engages (host-proven max|x| <= limit): att == 1, delta == 0 for
// every frame, so out[n] = level-scaled input[n - (B-1)] (B = ring frames).
__global__ void __launch_bounds__(AMX_BLOCK) k_final_fast(const SpanDev *__restrict__ spans,
                                                          const uint32_t *__restrict__ x,
                                                          const uint32_t *__restrict__ halo,
                                                          int halo_frames,
                                                          const double *__restrict__ gains,
                                                          double level_in, double level,
                                                          double level_out, double limit,
                                                          uint32_t *__restrict__ y) {
    const int t = blockIdx.y;
    const SpanDev sp = spans[t];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= sp.out_n) return;
    const int64_t src = i - halo_frames;      // span-local source frame (delay B-1)
    const int64_t tsrc = sp.tframe0 + src;   // whole-track source frame
    uint32_t p = 0;
    bool zero = tsrc < 0;
    if (!zero) p = src >= 0 ? x[sp.out_off + src] : halo[(int64_t)t * halo_frames + (halo_frames + src)];
    const double g = gains[t];
    int16_t o[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        if (zero) { o[c] = 0; continue; }
        int16_t v = gain16(c ? hi16(p) : lo16(p), g);
        double smp = ((double)v * (1.0 / 32768.0)) * level_in;
        double d = smp * 1.0;
        d = d < -limit ? -limit : (d > limit ? limit : d);
        d = d * level * level_out;
        o[c] = clip_llrint(d * 32768.0);
    }
    y[sp.out_off + i] = pack2(o[0], o[1]);
}

// General alimiter (af_alimiter.c filter_frame, asc off), one thread per track
// span, sequential.  State layout (doubles): [0] att [1] delta [2] pos [3] nextiter
// [4] nextlen [5] valid  [8 .. 8+bs) buffer  [8+bs .. 8+2bs) nextdelta
// [8+2bs .. 8+3bs) nextpos (stored as doubles).
__global__ void k_final_general(const SpanDev *__restrict__ spans, int n_tracks,
                                const uint32_t *__restrict__ x,
                                const uint32_t *__restrict__ halo, int halo_frames,
                                const double *__restrict__ gains, int fs, double level_in,
                                double level, double level_out, double limit, double release,
                                int bs, double *__restrict__ state, int64_t state_doubles,
                                uint32_t *__restrict__ y) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tracks) return;
    const SpanDev sp = spans[t];
    const int channels = 2;
    double *S = state + (int64_t)t * state_doubles;
    double *buffer = S + 8, *nextdelta = S + 8 + bs, *nextposd = S + 8 + 2 * bs;
    double att, delta;
    int pos, nextiter, nextlen;
    if (sp.tframe0 == 0 || S[5] == 0.0) {
        att = 1.0; delta = 0.0; pos = 0; nextiter = 0; nextlen = 0;
        for (int k = 0; k < bs; k++) { buffer[k] = 0.0; nextdelta[k] = 0.0; nextposd[k] = -1.0; }
        if (sp.tframe0 != 0) {
            // no carried state: prime the ring with the halo (limiter assumed idle)
            for (int h = 0; h < halo_frames; h++) {
                uint32_t p = halo[(int64_t)t * halo_frames + h];
                const double g = gains[t];
                for (int c = 0; c < channels; c++)
                    buffer[pos + c] = ((double)gain16(c ? hi16(p) : lo16(p), g) * (1.0 / 32768.0)) * level_in;
                pos = (pos + channels) % bs;
            }
        }
    } else {
        att = S[0]; delta = S[1]; pos = (int)S[2]; nextiter = (int)S[3]; nextlen = (int)S[4];
    }
#define NEXTPOS(k) ((int)nextposd[(k)])
    const double g = gains[t];
    for (int64_t n = 0; n < sp.out_n; n++) {
        uint32_t p = x[sp.out_off + n];
        double dst[2];
        double peak = 0;
        for (int c = 0; c < channels; c++) {
            double sample = ((double)gain16(c ? hi16(p) : lo16(p), g) * (1.0 / 32768.0)) * level_in;
            buffer[pos + c] = sample;
            peak = fmax(peak, fabs(sample));
        }
        if (peak > limit) {
            double patt = fmin(limit / peak, 1.);
            double rdelta = (1.0 - patt) / (fs * release);
            double d = (limit / peak - att) / bs * channels;
            int found = 0, i;
            if (d < delta) {
                delta = d;
                nextposd[0] = pos;
                nextposd[1] = -1;
                nextdelta[0] = rdelta;
                nextlen = 1;
                nextiter = 0;
            } else {
                for (i = nextiter; i < nextiter + nextlen; i++) {
                    int jx = i % bs;
                    double ppeak = 0, pdelta;
                    for (int c = 0; c < channels; c++) ppeak = fmax(ppeak, fabs(buffer[NEXTPOS(jx) + c]));
                    pdelta = (limit / peak - limit / ppeak) /
                             (((bs - NEXTPOS(jx) + pos) % bs) / channels);
                    if (pdelta < nextdelta[jx]) {
                        nextdelta[jx] = pdelta;
                        found = 1;
                        break;
                    }
                }
                if (found) {
                    nextlen = i - nextiter + 1;
                    nextposd[(nextiter + nextlen) % bs] = pos;
                    nextdelta[(nextiter + nextlen) % bs] = rdelta;
                    nextposd[(nextiter + nextlen + 1) % bs] = -1;
                    nextlen++;
                }
            }
        }
        const double *buf = &buffer[(pos + channels) % bs];
        peak = 0;
        for (int c = 0; c < channels; c++) peak = fmax(peak, fabs(buf[c]));
        att += delta;
        for (int c = 0; c < channels; c++) dst[c] = buf[c] * att;
        if ((pos + channels) % bs == NEXTPOS(nextiter)) {
            delta = nextdelta[nextiter];
            att = limit / peak;
            nextlen -= 1;
            nextposd[nextiter] = -1;
            nextiter = (nextiter + 1) % bs;
        }
        if (att > 1.) { att = 1.; delta = 0.; nextiter = 0; nextlen = 0; nextposd[0] = -1; }
        if (att <= 0.) { att = 0.0000000000001; delta = (1.0 - att) / (fs * release); }
        if (att != 1. && (1. - att) < 0.0000000000001) att = 1.;
        if (delta != 0. && fabs(delta) < 0.00000000000001) delta = 0.;
        int16_t o[2];
        for (int c = 0; c < channels; c++) {
            double v = dst[c];
            v = v < -limit ? -limit : (v > limit ? limit : v);
            v = v * level * level_out;
            o[c] = clip_llrint(v * 32768.0);
        }
        y[sp.out_off + n] = pack2(o[0], o[1]);
        pos = (pos + channels) % bs;
    }
#undef NEXTPOS
    S[0] = att; S[1] = delta; S[2] = pos; S[3] = nextiter; S[4] = nextlen; S[5] = 1.0;
}

// ================================================================ launchers
static inline dim3 grid1(int64_t n) { return dim3((unsigned)((n + AMX_BLOCK - 1) / AMX_BLOCK)); }
static inline bool empty(dim3 g) { return g.x == 0 || g.y == 0 || g.z == 0; }

template <int MASK>
static hipError_t front1_t(const Launch &l, const float *in, const float *lut, uint32_t *a16,
                           const double *G, double *e) {
    hipLaunchKernelGGL(k_front1<MASK>, grid1(l.n_seg), dim3(AMX_BLOCK), 0, l.stream, l.cd,
                       l.chunks, l.segs, l.n_seg, l.L, in, lut, a16, G, e);
    return hipGetLastError();
}

template <int MASK, bool MB>
static hipError_t front2_t(const Launch &l, const uint32_t *a16, const double *s_eq,
                           uint32_t *dst, int to_out, const double *Gx, double *e_x) {
    hipLaunchKernelGGL((k_front2<MASK, MB>), grid1(l.n_seg), dim3(AMX_BLOCK), 0, l.stream, l.cd,
                       l.chunks, l.segs, l.n_seg, a16, s_eq, dst, to_out, Gx, e_x);
    return hipGetLastError();
}

#define AMX_MASK_CASES(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

hipError_t launch_front1_lut(const Launch &l, int mask, const float *in, const float *lut,
                             int16_t *a16, const double *G, double *e) {
    uint32_t *a = reinterpret_cast<uint32_t *>(a16);
    switch (mask) {
#define C1(M) case M: return front1_t<M>(l, in, lut, a, G, e);
        AMX_MASK_CASES(C1)
#undef C1
    }
    return hipErrorInvalidValue;
}

hipError_t launch_front2(const Launch &l, int mask, const int16_t *a16, const double *s_eq,
                         int16_t *dst, int to_out, const double *Gx, double *e_x) {
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
    hipLaunchKernelGGL(k_xover2, grid1(l.n_seg), dim3(AMX_BLOCK), 0, l.stream, l.cd, l.chunks,
                       l.segs, l.n_seg, reinterpret_cast<const uint32_t *>(p16), s_x,
                       reinterpret_cast<uint32_t *>(bands), nloc);
    return hipGetLastError();
}

hipError_t launch_rms(const Launch &l, const int16_t *bands, uint16_t *r, int64_t nloc) {
    dim3 g = grid1(l.n_seg);
    g.y = 3;
    hipLaunchKernelGGL(k_rms, g, dim3(AMX_BLOCK), 0, l.stream, l.cd, l.chunks, l.segs, l.n_seg,
                       reinterpret_cast<const uint32_t *>(bands), r, nloc);
    return hipGetLastError();
}

hipError_t launch_env(const Launch &l, const uint16_t *r, const double *tabs, double *att,
                      double *guess, double *endv, int64_t nloc, int warm) {
    dim3 g = grid1(l.n_seg);
    g.y = 3;
    hipLaunchKernelGGL(k_env, g, dim3(AMX_BLOCK), 0, l.stream, l.cd, l.chunks, l.segs, l.n_seg,
                       r, tabs, att, guess, endv, nloc, warm);
    return hipGetLastError();
}

hipError_t launch_fix(const Launch &l, const uint16_t *r, const double *tabs, double *att,
                      double *guess, double *endv, int64_t nloc) {
    if (l.n_chunks <= 0) return hipSuccess;
    dim3 g((unsigned)l.n_chunks, 3);
    hipLaunchKernelGGL(k_fix, g, dim3(64), 0, l.stream, l.cd, l.chunks, l.segs, l.n_seg, r, tabs,
                       att, guess, endv, nloc);
    return hipGetLastError();
}

hipError_t launch_apply_n1(const Launch &l, const int16_t *bands, const double *att,
                           int16_t *out, int64_t nloc, int64_t max_chunk_out,
                           const int64_t *n1tab) {
    dim3 g = grid1(max_chunk_out);
    g.y = (unsigned)l.n_chunks;
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_apply, g, dim3(AMX_BLOCK), 0, l.stream, l.chunks,
                       reinterpret_cast<const uint32_t *>(bands), att,
                       reinterpret_cast<uint32_t *>(out), nloc, n1tab);
    return hipGetLastError();
}

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
    (void)L;
    if (n_kseg <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_kw2, grid1(n_kseg), dim3(AMX_BLOCK), 0, st, cd, ks, n_kseg, hop,
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

hipError_t launch_final_fast(const SpanDev *spans, int n_tracks, int64_t max_span,
                             const int16_t *x, const int16_t *halo, int halo_frames,
                             const double *gains, double level_in, double level,
                             double level_out, double limit, int16_t *y, hipStream_t st) {
    dim3 g = grid1(max_span);
    g.y = (unsigned)n_tracks;
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_final_fast, g, dim3(AMX_BLOCK), 0, st, spans,
                       reinterpret_cast<const uint32_t *>(x),
                       reinterpret_cast<const uint32_t *>(halo), halo_frames, gains, level_in,
                       level, level_out, limit, reinterpret_cast<uint32_t *>(y));
    return hipGetLastError();
}

hipError_t launch_final_general(const SpanDev *spans, int n_tracks, const int16_t *x,
                                const int16_t *halo, int halo_frames, const double *gains,
                                int fs, double level_in, double level, double level_out,
                                double limit, double release, int buffer_size,
                                double *state, int64_t state_doubles, int16_t *y,
                                hipStream_t st) {
    if (n_tracks <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_final_general, dim3((n_tracks + 63) / 64), dim3(64), 0, st, spans,
                       n_tracks, reinterpret_cast<const uint32_t *>(x),
                       reinterpret_cast<const uint32_t *>(halo), halo_frames, gains, fs,
                       level_in, level, level_out, limit, release, buffer_size, state,
                       state_doubles, reinterpret_cast<uint32_t *>(y));
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
