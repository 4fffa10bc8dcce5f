// amx_loud192.hip -- loudnorm pass 1 measured the way ffmpeg measures it: on the
// track resampled to 192 kHz (audio_mastering_engine.py:229 passes no measured_*
// values, so af_loudnorm runs in dynamic mode, whose query_formats asks for 192 kHz;
// ffmpeg inserts libswresample with its defaults).  The 192 kHz stream is never
// materialised: every kernel recomputes the samples it needs from the s16 track.
//
// Resampler (restated in oracle/amx_oracle.c, "libswresample"): exact-rational
// polyphase FIR, L phases, step M input samples per L outputs (48 kHz: L 4, M 1;
// 96 kHz: 2, 1; 44.1 kHz: 640, 147), 32 Kaiser-windowed taps, float32 bank and float32
// arithmetic (s16 in + dbl out -> FLTP internal format).  Output j = dot of the bank
// row (j M) % L with inputs floor(j M / L) - 15 .. + 16, summed in the order of the
// x86 FMA3 kernel: 8 fused chains over taps k, k+8, k+16, k+24, then
// ((a0+a4) + (a2+a6)) + ((a1+a5) + (a3+a7)).  Inputs are mirrored at the track's
// ends (x[-k] = x[k], x[n+k] = x[n-1-k]); a span that does not start / end its track
// reads the neighbouring rank's frames from the edge buffer instead.
//
// Both channels of a frame travel packed in one float2, so one v_pk_fma_f32 does a
// tap of both channels.  One lane per K-filter segment (Lin input frames = Lout
// outputs); all segments of a plan share the phase pattern (the plan checks it), so
// the bank row and the GEMV row of an output are wave-uniform (scalar loads).
//   k_up1: pass 1 -- zero-state end state of the K filter per segment: a GEMV over
//          the segment's outputs (G[n] = A^{Lout-1-n} B), for the scan; and the
//          sample peaks (192 kHz, loudnorm's input_tp; d_out's own, the limiter's).
//   k_up1_part: the same for a span's last, partial segment (row alignment differs).
//   k_up2: pass 2 -- the K filter (two DF-II-T biquads) from the exact segment start
//          state, y^2 summed per 100 ms hop piece.
// M == 1 rates (48, 96, 32 kHz ...) take the unrolled path STATIC = L: every input
// frame has outputs at phases 0 .. L-1 and phase 0 is the identity (the bank's
// phase-0 row is a unit impulse: u = x exactly).
#include "amx_dev.hpp"

namespace amx {

typedef float f2 __attribute__((ext_vector_type(2)));

#define UP_TAPS 32
#define UP_C 15            // center tap
#define UP_TB 8            // input frames per window block (STATIC path)

__device__ __forceinline__ f2 up_frame(uint32_t w) {
    return f2{(float)lo16(w) * (1.0f / 32768.0f), (float)hi16(w) * (1.0f / 32768.0f)};
}

__device__ __forceinline__ int64_t up_reflect(int64_t k, int64_t n) {
    for (int it = 0; it < 64; it++) {
        if (k < 0) k = -k;
        else if (k >= n) k = 2 * n - 1 - k;
        else return k;
    }
    return 0;
}

// span-local input frame g of the stream the resampler sees
__device__ __forceinline__ uint32_t up_word(const uint32_t *__restrict__ x,
                                            const uint32_t *__restrict__ edge, const SpanDev &sp,
                                            int t, int64_t g) {
    const int64_t n = sp.out_n;
    if (g >= 0 && g < n) return x[sp.out_off + g];
    if (g < 0 && sp.edge_lo && g >= -AMX_UP_EDGE) return edge[((int64_t)t * 2) * AMX_UP_EDGE + AMX_UP_EDGE + g];
    if (g >= n && sp.edge_hi && g < n + AMX_UP_EDGE) return edge[((int64_t)t * 2 + 1) * AMX_UP_EDGE + (g - n)];
    return n > 0 ? x[sp.out_off + up_reflect(g, n)] : 0u;
}

// the FMA3 kernel's order, both channels at once
__device__ __forceinline__ f2 up_dot(const f2 *w, const float *__restrict__ h) {
    f2 a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        f2 acc = w[k] * h[k];
        acc = __builtin_elementwise_fma(w[k + 8], f2{h[k + 8], h[k + 8]}, acc);
        acc = __builtin_elementwise_fma(w[k + 16], f2{h[k + 16], h[k + 16]}, acc);
        acc = __builtin_elementwise_fma(w[k + 24], f2{h[k + 24], h[k + 24]}, acc);
        a[k] = acc;
    }
    const f2 b0 = a[0] + a[4], b1 = a[1] + a[5], b2 = a[2] + a[6], b3 = a[3] + a[7];
    return (b0 + b2) + (b1 + b3);
}

// ------------------------------------------------------------ pass 1 (GEMV)
// pass 1 also takes the sample peaks (loudnorm's input_tp from the 192 kHz samples,
// and d_out's own peak for the limiter decision), so they are known -- and, at N > 1,
// exchanged -- before pass 2.  xc = the input frame the output's window is centred on.
struct Up1Acc {
    double e0[AMX_KW_DIM], e1[AMX_KW_DIM];
    f2 pk, px;
    int len;
    __device__ void init(int n_out) {
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) { e0[d] = 0.0; e1[d] = 0.0; }
        pk = f2{0.0f, 0.0f};
        px = f2{0.0f, 0.0f};
        len = n_out;
    }
    __device__ __forceinline__ void add(int n, const double *__restrict__ g, f2 u, f2 xc) {
        const double u0 = (double)u.x, u1 = (double)u.y;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) {
            e0[d] = fma(g[d], u0, e0[d]);
            e1[d] = fma(g[d], u1, e1[d]);
        }
        const bool in = n < len;
        pk = in ? f2{fmaxf(pk.x, fabsf(u.x)), fmaxf(pk.y, fabsf(u.y))} : pk;
        px = in ? f2{fmaxf(px.x, fabsf(xc.x)), fmaxf(px.y, fabsf(xc.y))} : px;
    }
};

// ------------------------------------------------------------ pass 2 (filter)
struct Up2Acc {
    double c1[5], c2[5];
    double v0[4], v1[4];       // [biquad1 z0 z1, biquad2 z0 z1] per channel
    double p00, p01, p10, p11; // y^2 per (piece, channel)
    int split;                 // first output of hop piece 1
    int len;                   // outputs of this segment
    __device__ __forceinline__ void add(int n, const double *, f2 u, f2) {
        const bool in = n < len;
        const double u0 = (double)u.x, u1 = (double)u.y;
        const double a0 = bq_step(c1, v0[0], v0[1], u0);
        double y0 = bq_step(c2, v0[2], v0[3], a0);
        const double a1 = bq_step(c1, v1[0], v1[1], u1);
        double y1 = bq_step(c2, v1[2], v1[3], a1);
        y0 = in ? y0 : 0.0;
        y1 = in ? y1 : 0.0;
        if (n < split) { p00 = fma(y0, y0, p00); p01 = fma(y1, y1, p01); }
        else { p10 = fma(y0, y0, p10); p11 = fma(y1, y1, p11); }
    }
};

// a bank row as an opaque per-iteration pointer: without it the compiler hoists every
// phase's 32 coefficients out of the block loop into SGPRs at once and spills them
__device__ __forceinline__ const float *up_row(const float *bank, int ph) {
    const float *h = bank + ph * UP_TAPS;
    asm volatile("" : "+s"(h));
    return h;
}

// STATIC = L (M == 1): unrolled window blocks of UP_TB input frames, outputs at phases
// 0 .. L-1 of every frame; 0: general phase pattern from the tables
template <int STATIC, class Acc, bool P1>
__device__ __forceinline__ void up_run(const UpArgs &a, const SpanDev &sp, int t, int64_t g0,
                                       bool edge, Acc &acc) {
    const uint32_t *__restrict__ x = a.x;
    if constexpr (STATIC > 0) {
        constexpr int W = UP_TB + UP_TAPS - 1;                 // inputs [k0 - 15, k0 + TB + 16)
        f2 w[W];
        const uint32_t *xp = x + sp.out_off + g0 - UP_C;       // frame g0 - 15
#pragma unroll
        for (int i = 0; i < W; i++)
            w[i] = up_frame(edge ? up_word(x, a.edge, sp, t, g0 - UP_C + i) : xp[i]);
        const int nblk = a.Lin / UP_TB;
        for (int b = 0; b < nblk; b++) {
            // next block's new inputs in flight while this block computes
            uint32_t nx[UP_TB];
            const bool more = b + 1 < nblk;
#pragma unroll
            for (int i = 0; i < UP_TB; i++) {
                // (past the last block: frame g0 - 15 again, in range, unused)
                const int o = more ? (b + 1) * UP_TB + (W - UP_TB) + i : 0;
                nx[i] = edge ? up_word(x, a.edge, sp, t, g0 - UP_C + o) : xp[o];
            }
            const int nb0 = b * UP_TB * STATIC;
            if constexpr (P1) {
                // GEMV and peaks are order-free: phase-outer, one bank row live at a time
#pragma unroll
                for (int ph = 0; ph < STATIC; ph++) {
                    const float *h = up_row(a.bank, ph);
#pragma unroll
                    for (int kb = 0; kb < UP_TB; kb++) {
                        const int n = nb0 + kb * STATIC + ph;
                        const f2 u = ph == 0 ? w[kb + UP_C] : up_dot(w + kb, h);
                        acc.add(n, a.G + (int64_t)n * AMX_KW_DIM, u, w[kb + UP_C]);
                    }
                }
            } else {
                // the recursion needs output order: the block's samples first (phase
                // outer), then the filter over them in order
                f2 u[UP_TB][STATIC > 1 ? STATIC - 1 : 1];
#pragma unroll
                for (int ph = 1; ph < STATIC; ph++) {
                    const float *h = up_row(a.bank, ph);
#pragma unroll
                    for (int kb = 0; kb < UP_TB; kb++) u[kb][ph - 1] = up_dot(w + kb, h);
                }
#pragma unroll
                for (int kb = 0; kb < UP_TB; kb++)
#pragma unroll
                    for (int ph = 0; ph < STATIC; ph++)
                        acc.add(nb0 + kb * STATIC + ph, nullptr, ph == 0 ? w[kb + UP_C] : u[kb][ph - 1],
                                w[kb + UP_C]);
            }
#pragma unroll
            for (int i = 0; i < W - UP_TB; i++) w[i] = w[i + UP_TB];
#pragma unroll
            for (int i = 0; i < UP_TB; i++) w[W - UP_TB + i] = up_frame(nx[i]);
        }
    } else {
        f2 w[UP_TAPS];
#pragma unroll
        for (int i = 0; i < UP_TAPS; i++) w[i] = up_frame(up_word(x, a.edge, sp, t, g0 - UP_C + i));
        int cur = 0;
        for (int n = 0; n < a.Lout; n++) {
            const int kb = a.obase[n];
            if (kb > cur) {                                    // wave-uniform: one frame on
#pragma unroll
                for (int i = 0; i < UP_TAPS - 1; i++) w[i] = w[i + 1];
                w[UP_TAPS - 1] = up_frame(up_word(x, a.edge, sp, t, g0 + cur + UP_TAPS - UP_C));
                cur++;
            }
            const f2 u = up_dot(w, a.bank + a.oph[n] * UP_TAPS);
            acc.add(n, a.G + (int64_t)n * AMX_KW_DIM, u, w[UP_C]);
        }
    }
}

template <int STATIC>
__global__ void __launch_bounds__(AMX_UP_BLOCK) k_up1(UpArgs a) {
    const int j = blockIdx.x * AMX_UP_BLOCK + threadIdx.x;
    const bool valid = j < a.n_kseg;
    const KwSegDev sg = a.ks[valid ? j : a.n_kseg - 1];
    const SpanDev sp = a.spans[sg.track];
    const int64_t g0 = sg.out_pos - sp.out_off;
    const bool edge = g0 - UP_C < 0 || g0 + a.Lin + UP_TAPS - UP_C > sp.out_n;
    Up1Acc acc;
    acc.init(valid ? sg.len : 0);
    up_run<STATIC, Up1Acc, true>(a, sp, sg.track, g0, edge, acc);
    // a span's partial last segment is k_up1_part's (its GEMV rows are right-aligned)
    if (valid && sg.len == a.Lout) {
        double *o = a.e + (int64_t)j * 2 * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) { o[d] = acc.e0[d]; o[AMX_KW_DIM + d] = acc.e1[d]; }
    }
    if (valid) {
        uint32_t *q = a.pk + (int64_t)j * 4;
        q[0] = __float_as_uint(acc.pk.x);
        q[1] = __float_as_uint(acc.pk.y);
        q[2] = (uint32_t)(acc.px.x * 32768.0f);      // |s16| / 32768: exact
        q[3] = (uint32_t)(acc.px.y * 32768.0f);
    }
}

// one wave per span: its last segment when partial (len < Lout): lane l takes the
// outputs n = l, l + 64, ... with its own window, rows G[n + Lout - len]
__global__ void __launch_bounds__(64) k_up1_part(UpArgs a) {
    const SpanDev sp = a.spans[blockIdx.x];
    if (sp.nkseg == 0) return;
    const int j = sp.kseg0 + sp.nkseg - 1;
    const KwSegDev sg = a.ks[j];
    if (sg.len == a.Lout) return;
    const int lane = threadIdx.x;
    const int64_t g0 = sg.out_pos - sp.out_off;
    const int sh = a.Lout - sg.len;
    Up1Acc acc;
    acc.init(sg.len);
    for (int n = lane; n < sg.len; n += 64) {
        const int base = a.obase[n], ph = a.oph[n];
        f2 w[UP_TAPS];
#pragma unroll
        for (int i = 0; i < UP_TAPS; i++)
            w[i] = up_frame(up_word(a.x, a.edge, sp, (int)blockIdx.x, g0 + base - UP_C + i));
        const f2 u = (a.static_l > 0 && ph == 0) ? w[UP_C] : up_dot(w, a.bank + ph * UP_TAPS);
        acc.add(n, a.G + (int64_t)(n + sh) * AMX_KW_DIM, u, w[UP_C]);
    }
#pragma unroll
    for (int d = 0; d < AMX_KW_DIM; d++)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            acc.e0[d] += __shfl_xor(acc.e0[d], o);
            acc.e1[d] += __shfl_xor(acc.e1[d], o);
        }
    if (lane == 0) {
        double *o = a.e + (int64_t)j * 2 * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) { o[d] = acc.e0[d]; o[AMX_KW_DIM + d] = acc.e1[d]; }
    }
}

template <int STATIC>
__global__ void __launch_bounds__(AMX_UP_BLOCK) k_up2(UpArgs a) {
    const int j = blockIdx.x * AMX_UP_BLOCK + threadIdx.x;
    const bool valid = j < a.n_kseg;
    const KwSegDev sg = a.ks[valid ? j : a.n_kseg - 1];
    const SpanDev sp = a.spans[sg.track];
    const int64_t g0 = sg.out_pos - sp.out_off;
    const bool edge = g0 - UP_C < 0 || g0 + a.Lin + UP_TAPS - UP_C > sp.out_n;
    Up2Acc acc;
#pragma unroll
    for (int i = 0; i < 3; i++) { acc.c1[i] = a.cd->kw1[i]; acc.c2[i] = a.cd->kw2[i]; }
    acc.c1[3] = a.cd->kw1[4]; acc.c1[4] = a.cd->kw1[5];
    acc.c2[3] = a.cd->kw2[4]; acc.c2[4] = a.cd->kw2[5];
    const double *s = a.s + (int64_t)(valid ? j : 0) * 2 * AMX_KW_DIM;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        acc.v0[d] = valid ? s[d] : 0.0;
        acc.v1[d] = valid ? s[AMX_KW_DIM + d] : 0.0;
    }
    acc.p00 = acc.p01 = acc.p10 = acc.p11 = 0.0;
    acc.len = valid ? sg.len : 0;
    const int64_t h0 = sg.tframe / a.hop;
    acc.split = (int)((h0 + 1) * a.hop - sg.tframe);
    up_run<STATIC, Up2Acc, false>(a, sp, sg.track, g0, edge, acc);
    if (valid) {
        double *o = a.parts + (int64_t)j * 4;
        o[0] = acc.p00; o[1] = acc.p01; o[2] = acc.p10; o[3] = acc.p11;
        a.part_hop[j] = h0;
    }
}

hipError_t launch_up1(const UpArgs &a, int n_spans, hipStream_t st) {
    if (a.n_kseg <= 0) return hipSuccess;
    const dim3 g((unsigned)((a.n_kseg + AMX_UP_BLOCK - 1) / AMX_UP_BLOCK));
    switch (a.static_l) {
    case 0: hipLaunchKernelGGL(k_up1<0>, g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_up1<2>, g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    case 4: hipLaunchKernelGGL(k_up1<4>, g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    default: return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(k_up1_part, dim3((unsigned)n_spans), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_up2(const UpArgs &a, hipStream_t st) {
    if (a.n_kseg <= 0) return hipSuccess;
    const dim3 g((unsigned)((a.n_kseg + AMX_UP_BLOCK - 1) / AMX_UP_BLOCK));
    switch (a.static_l) {
    case 0: hipLaunchKernelGGL(k_up2<0>, g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_up2<2>, g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    case 4: hipLaunchKernelGGL(k_up2<4>, g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace amx
