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
// outputs, Lout dividing the 100 ms hop where the rate allows); all segments of a
// plan share the phase pattern (the plan checks it), so a bank row is wave-uniform.
//   k_up<P1>: pass 1 -- the K filter (two DF-II-T biquads) over the segment from
//          rest: its end state is the zero-state end state the scan needs; and the
//          sample peaks (192 kHz, loudnorm's input_tp; d_out's own, the limiter's).
//   k_up<P2>: pass 2 -- the K filter from the exact segment start state, y^2
//          summed per 100 ms hop piece.
// M == 1 rates (48, 96, 32 kHz ...) take the unrolled path STATIC = L: every input
// frame has outputs at phases 0 .. L-1 and phase 0 is the identity (the bank's
// phase-0 row is a unit impulse: u = x exactly).
#include "amx_dev.hpp"

namespace amx {

typedef float f2 __attribute__((ext_vector_type(2)));

#define UP_TAPS 32
#define UP_C 15            // center tap
// input frames per window block of the STATIC path: the window (TB + 31 frames) and the
// block's samples (TB (L - 1)) live in registers
#ifndef AMX_UP_TB4
#define AMX_UP_TB4 4
#endif
template <int L> struct UpTB { static constexpr int v = L >= 4 ? AMX_UP_TB4 : 8; };
#ifndef AMX_UP_WAVES
#define AMX_UP_WAVES 3     // waves per SIMD the register budget must allow
#endif

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

// ------------------------------------------------------------ accumulators
// Both passes run the K filter (two DF-II-T biquads per channel, the state order of
// the scan's model [bq1 z0 z1, bq2 z0 z1]) over the segment's 192 kHz samples in
// order: pass 1 from rest -- its end state IS the zero-state end state the scan
// needs -- and pass 2 from the exact start state, summing y^2 per hop piece.
// FAST: every lane of the wave has a whole segment inside one hop and away from the
// span ends -- no masks, no hop split, no edge reads (all but ~one wave per span).
template <bool P1, bool FAST>
struct UpAcc {
    double c1[5], c2[5];
    double v0[4], v1[4];
    double p00, p01, p10, p11;   // pass 2: y^2 per (piece, channel)
    f2 pk, px;                   // pass 1: 192 kHz |u| max, d_out |x| max
    int split, len;
    __device__ __forceinline__ void add(int n, f2 u, f2 xc) {
        const double u0 = (double)u.x, u1 = (double)u.y;
        if constexpr (P1 && !FAST) {
            double w0[4], w1[4];
#pragma unroll
            for (int d = 0; d < 4; d++) { w0[d] = v0[d]; w1[d] = v1[d]; }
            const double a0 = bq_step(c1, v0[0], v0[1], u0);
            (void)bq_step(c2, v0[2], v0[3], a0);
            const double a1 = bq_step(c1, v1[0], v1[1], u1);
            (void)bq_step(c2, v1[2], v1[3], a1);
            const bool in = n < len;              // past a partial segment's end: state held
#pragma unroll
            for (int d = 0; d < 4; d++) { v0[d] = in ? v0[d] : w0[d]; v1[d] = in ? v1[d] : w1[d]; }
            pk = in ? f2{fmaxf(pk.x, fabsf(u.x)), fmaxf(pk.y, fabsf(u.y))} : pk;
            px = in ? f2{fmaxf(px.x, fabsf(xc.x)), fmaxf(px.y, fabsf(xc.y))} : px;
        } else if constexpr (P1) {
            const double a0 = bq_step(c1, v0[0], v0[1], u0);
            (void)bq_step(c2, v0[2], v0[3], a0);
            const double a1 = bq_step(c1, v1[0], v1[1], u1);
            (void)bq_step(c2, v1[2], v1[3], a1);
            pk = f2{fmaxf(pk.x, fabsf(u.x)), fmaxf(pk.y, fabsf(u.y))};
            px = f2{fmaxf(px.x, fabsf(xc.x)), fmaxf(px.y, fabsf(xc.y))};
        } else {
            const double a0 = bq_step(c1, v0[0], v0[1], u0);
            double y0 = bq_step(c2, v0[2], v0[3], a0);
            const double a1 = bq_step(c1, v1[0], v1[1], u1);
            double y1 = bq_step(c2, v1[2], v1[3], a1);
            if constexpr (FAST) {
                p00 = fma(y0, y0, p00);
                p01 = fma(y1, y1, p01);
            } else {
                const bool in = n < len;
                y0 = in ? y0 : 0.0;
                y1 = in ? y1 : 0.0;
                if (n < split) { p00 = fma(y0, y0, p00); p01 = fma(y1, y1, p01); }
                else { p10 = fma(y0, y0, p10); p11 = fma(y1, y1, p11); }
            }
        }
    }
};

// STATIC = L (M == 1): unrolled window blocks of UP_TB input frames, outputs at phases
// 0 .. L-1 of every frame; 0: general phase pattern from the tables.
// sb: the bank in LDS (STATIC); zp: an LDS word holding 0, read every block so the
// compiler cannot hoist the bank rows out of the block loop (all rows live at once
// would not fit the registers)
template <int STATIC, bool FAST, class Acc>
__device__ __forceinline__ void up_run(const UpArgs &a, const SpanDev &sp, int t, int64_t g0,
                                       bool vec, const float *sb, const int *zp, Acc &acc) {
    const uint32_t *__restrict__ x = a.x;
    if constexpr (STATIC > 0) {
        constexpr int UP_TB = UpTB<STATIC>::v;
        constexpr int W = UP_TB + UP_TAPS - 1;                 // inputs [k0 - 15, k0 + TB + 16)
        f2 w[W];
        const uint32_t *xp = x + sp.out_off + g0 - UP_C;       // frame g0 - 15
#pragma unroll
        for (int i = 0; i < W; i++)
            w[i] = up_frame(FAST ? xp[i] : up_word(x, a.edge, sp, t, g0 - UP_C + i));
        const int nblk = a.Lin / UP_TB;
        for (int b = 0; b < nblk; b++) {
            // next block's new frames in flight while this block computes (past the
            // last block: frames of this one again, in range, unused)
            uint32_t nx[UP_TB];
            const int o0 = (b + 1 < nblk ? (b + 1) * UP_TB : b * UP_TB) + (W - UP_TB);
            if (FAST && vec) {                                  // 16-B aligned rows
#pragma unroll
                for (int i = 0; i < UP_TB; i += 4) {
                    const uint4 q = *reinterpret_cast<const uint4 *>(xp + o0 + i);
                    nx[i] = q.x; nx[i + 1] = q.y; nx[i + 2] = q.z; nx[i + 3] = q.w;
                }
            } else {
#pragma unroll
                for (int i = 0; i < UP_TB; i++)
                    nx[i] = FAST ? xp[o0 + i] : up_word(x, a.edge, sp, t, g0 - UP_C + o0 + i);
            }
            const int nb0 = b * UP_TB * STATIC;
            // the bank row through scalar loads (SGPR operands of the FMAs); the
            // offset read from LDS (always 0) keeps the compiler from hoisting every
            // row out of the loop at once
            const float *bk = a.bank + __builtin_amdgcn_readfirstlane(zp[b & 1]);
            f2 u[UP_TB][STATIC > 1 ? STATIC - 1 : 1];
#pragma unroll
            for (int ph = 1; ph < STATIC; ph++) {
                const float *h = bk + ph * UP_TAPS;
#pragma unroll
                for (int kb = 0; kb < UP_TB; kb++) u[kb][ph - 1] = up_dot(w + kb, h);
            }
#pragma unroll
            for (int kb = 0; kb < UP_TB; kb++)
#pragma unroll
                for (int ph = 0; ph < STATIC; ph++)
                    acc.add(nb0 + kb * STATIC + ph, ph == 0 ? w[kb + UP_C] : u[kb][ph - 1], w[kb + UP_C]);
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
            acc.add(n, up_dot(w, a.bank + a.oph[n] * UP_TAPS), w[UP_C]);
        }
    }
}

// both passes: P1 = pass 1 (from rest: end state + peaks), else pass 2 (hop pieces)
template <int STATIC, bool P1>
__global__ void __launch_bounds__(AMX_UP_BLOCK) __attribute__((amdgpu_waves_per_eu(AMX_UP_WAVES)))
k_up(UpArgs a) {
    __shared__ __attribute__((aligned(16))) float sb[STATIC > 0 ? STATIC * UP_TAPS : 4];
    __shared__ int zp[2];
    const int lane = threadIdx.x;
    if constexpr (STATIC > 0) {
        for (int i = lane; i < STATIC * UP_TAPS; i += AMX_UP_BLOCK) sb[i] = a.bank[i];
    }
    if (lane < 2) zp[lane] = 0;
    __syncthreads();
    const int j = blockIdx.x * AMX_UP_BLOCK + lane;
    const bool valid = j < a.n_kseg;
    const KwSegDev sg = a.ks[valid ? j : a.n_kseg - 1];
    const SpanDev sp = a.spans[sg.track];
    const int64_t g0 = sg.out_pos - sp.out_off;
    const bool edge = g0 - UP_C < 0 || g0 + a.Lin + UP_TAPS - UP_C > sp.out_n;
    const int64_t h0 = sg.tframe / a.hop;
    const int split = (int)((h0 + 1) * a.hop - sg.tframe);
    const int len = valid ? sg.len : 0;
    const bool fast = valid && !edge && len == a.Lout && (P1 || split >= a.Lout);
    // 16-B loads when every lane's window rows are 16-B aligned
    const bool vec = __ballot(((sp.out_off + g0 - UP_C + (UP_TAPS - 1)) & 3) != 0) == 0;
    UpAcc<P1, true> af;
    UpAcc<P1, false> ag;
    auto setup = [&](auto &acc) {
#pragma unroll
        for (int i = 0; i < 3; i++) { acc.c1[i] = a.cd->kw1[i]; acc.c2[i] = a.cd->kw2[i]; }
        acc.c1[3] = a.cd->kw1[4]; acc.c1[4] = a.cd->kw1[5];
        acc.c2[3] = a.cd->kw2[4]; acc.c2[4] = a.cd->kw2[5];
        const double *s0 = a.s + (int64_t)(valid ? j : 0) * 2 * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < 4; d++) {
            acc.v0[d] = (!P1 && valid) ? s0[d] : 0.0;
            acc.v1[d] = (!P1 && valid) ? s0[AMX_KW_DIM + d] : 0.0;
        }
        acc.p00 = acc.p01 = acc.p10 = acc.p11 = 0.0;
        acc.pk = f2{0.0f, 0.0f};
        acc.px = f2{0.0f, 0.0f};
        acc.split = split;
        acc.len = len;
    };
    double v0[4], v1[4], p[4];
    f2 pk, px;
    auto take = [&](auto &acc) {
#pragma unroll
        for (int d = 0; d < 4; d++) { v0[d] = acc.v0[d]; v1[d] = acc.v1[d]; }
        p[0] = acc.p00; p[1] = acc.p01; p[2] = acc.p10; p[3] = acc.p11;
        pk = acc.pk;
        px = acc.px;
    };
    if (__ballot(!fast) == 0) {
        setup(af);
        up_run<STATIC, true>(a, sp, sg.track, g0, vec, sb, zp, af);
        take(af);
    } else {
        setup(ag);
        up_run<STATIC, false>(a, sp, sg.track, g0, vec, sb, zp, ag);
        take(ag);
    }
    if (!valid) return;
    if constexpr (P1) {
        double *o = a.e + (int64_t)j * 2 * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) { o[d] = v0[d]; o[AMX_KW_DIM + d] = v1[d]; }
        uint32_t *q = a.pk + (int64_t)j * 4;
        q[0] = __float_as_uint(pk.x);
        q[1] = __float_as_uint(pk.y);
        q[2] = (uint32_t)(px.x * 32768.0f);      // |s16| / 32768: exact
        q[3] = (uint32_t)(px.y * 32768.0f);
    } else {
        double *o = a.parts + (int64_t)j * 4;
        o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; o[3] = p[3];
        a.part_hop[j] = h0;
    }
}

template <bool P1>
static hipError_t up_launch(const UpArgs &a, hipStream_t st) {
    if (a.n_kseg <= 0) return hipSuccess;
    const dim3 g((unsigned)((a.n_kseg + AMX_UP_BLOCK - 1) / AMX_UP_BLOCK));
    switch (a.static_l) {
    case 0: hipLaunchKernelGGL((k_up<0, P1>), g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_up<2, P1>), g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    case 4: hipLaunchKernelGGL((k_up<4, P1>), g, dim3(AMX_UP_BLOCK), 0, st, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_up1(const UpArgs &a, int n_spans, hipStream_t st) {
    (void)n_spans;
    return up_launch<true>(a, st);
}

hipError_t launch_up2(const UpArgs &a, hipStream_t st) { return up_launch<false>(a, st); }

}  // namespace amx
