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
// One lane per (K-filter segment, channel): lanes 2i / 2i+1 are the L / R channel of
// segment i (Lin input frames = Lout outputs, Lout dividing the 100 ms hop where the
// rate allows).  A lane's window of 32 + TB - 1 float samples, its filter state and
// accumulators fit ~90 VGPRs, so 4+ waves per SIMD hide the dependent latencies (one
// lane per segment with both channels packed in float2 needed ~150: two waves per
// SIMD, measured 1.2-1.4x slower).  All segments of a plan share the phase pattern
// (the plan checks it), so a bank row is wave-uniform: scalar operands of the FMAs.
//   k_up: the one pass over the samples -- the K filter (two DF-II-T biquads) over
//          the segment from rest: its end state is the zero-state end state the scan
//          needs; the sample peaks (192 kHz, loudnorm's input_tp; d_out's own, the
//          limiter's); and, per 100 ms hop piece, what the piece's energy needs once
//          the exact start state s is known: the filter is linear, y_n = yz_n +
//          C A^n s (yz = the response from rest computed here), so
//            sum y^2 = sum yz^2 + 2 s . sum yz_n (C A^n)^T + s^T Q s,
//          Q = sum (C A^n)^T (C A^n) a plan constant.  The pass over the samples is
//          therefore not repeated after the scan:
//   k_up_energy: per (segment, channel), the hop pieces' energies from s (after
//          the scan, with the carry from the previous rank at N > 1).
// M == 1 rates (48, 96, 32 kHz ...) take the unrolled path STATIC = L: every input
// frame has outputs at phases 0 .. L-1 and phase 0 is the identity (the bank's
// phase-0 row is a unit impulse: u = x exactly).
#include "amx_dev.hpp"

namespace amx {

#define UP_TAPS 32
#define UP_C 15            // center tap
#ifndef AMX_UP_TB
#define AMX_UP_TB 8        // input frames per window block (STATIC path)
#endif
#ifndef AMX_UP_SB
#define AMX_UP_SB 6        // sched_barrier mask: VALU + SALU may cross, scalar loads may not
#endif
#ifndef UP_DOT
#define UP_DOT up_dot2      // packed-pair form of the fast kernel's dot products
#endif
#ifndef AMX_UP_WAVES
#define AMX_UP_WAVES 4     // waves per SIMD the register budget must allow
#endif

__device__ __forceinline__ float up_sample(uint32_t w, int ch) {
    return (float)(ch ? hi16(w) : lo16(w)) * (1.0f / 32768.0f);
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

typedef float up_f2 __attribute__((ext_vector_type(2)));

// the FMA3 kernel's order with the 8 chains as 4 packed pairs (v_pk_fma_f32 / v_pk_add_f32):
// the same operations, lane by lane, as up_dot
__device__ __forceinline__ float up_dot2(const float *w, const float *__restrict__ h) {
    up_f2 a[4];
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
        up_f2 acc = up_f2{w[k], w[k + 1]} * up_f2{h[k], h[k + 1]};
        acc = __builtin_elementwise_fma(up_f2{w[k + 8], w[k + 9]}, up_f2{h[k + 8], h[k + 9]}, acc);
        acc = __builtin_elementwise_fma(up_f2{w[k + 16], w[k + 17]}, up_f2{h[k + 16], h[k + 17]}, acc);
        acc = __builtin_elementwise_fma(up_f2{w[k + 24], w[k + 25]}, up_f2{h[k + 24], h[k + 25]}, acc);
        a[k >> 1] = acc;
    }
    const up_f2 b01 = a[0] + a[2], b23 = a[1] + a[3];     // (a0+a4, a1+a5), (a2+a6, a3+a7)
    const up_f2 c = b01 + b23;                            // (b0+b2, b1+b3)
    return c.x + c.y;
}

// the FMA3 kernel's order
__device__ __forceinline__ float up_dot(const float *w, const float *__restrict__ h) {
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float acc = w[k] * h[k];
        acc = fmaf(w[k + 8], h[k + 8], acc);
        acc = fmaf(w[k + 16], h[k + 16], acc);
        acc = fmaf(w[k + 24], h[k + 24], acc);
        a[k] = acc;
    }
    const float b0 = a[0] + a[4], b1 = a[1] + a[5], b2 = a[2] + a[6], b3 = a[3] + a[7];
    return (b0 + b2) + (b1 + b3);
}

// libebur128's second K section, the RLB high-pass: b = (1, -2, 1) always, so the
// DF-II-T step is bq_step's arithmetic without its two unit multiplies (same values)
__device__ __forceinline__ double hp_step(const double *q, double &z0, double &z1, double x) {
    const double y = x + z0;
    z0 = fma(-q[3], y, fma(-2.0, x, z1));
    z1 = fma(-q[4], y, x);
    return y;
}

// ------------------------------------------------------------ accumulator
// FAST: every lane of the wave has a whole segment inside one hop and away from the
// span ends -- no masks, no hop split, no edge reads (all but ~one wave per span).
template <bool FAST>
struct UpAcc {
    double c1[5], c2[5];
    double v[4];                 // K-filter state (the scan model's order)
    double z0, z1;               // sum yz^2 per hop piece
    double q0[4], q1[4];         // sum yz_n (C A^n)^T per hop piece
    float pk, px;                // 192 kHz |u| max, d_out |x| max
    int split, len;
    const double *wc;            // rows C A^n (plan table)
    __device__ __forceinline__ void add(int n, float u, float xc) {
        add_row(n, u, xc, wc + (int64_t)n * AMX_KW_DIM);              // wave-uniform row
    }
    __device__ __forceinline__ void add_row(int n, float u, float xc, const double *r) {
        const double ud = (double)u;
        if constexpr (FAST) {
            const double a = bq_step(c1, v[0], v[1], ud);
            const double y = hp_step(c2, v[2], v[3], a);
            z0 = fma(y, y, z0);
#pragma unroll
            for (int d = 0; d < 4; d++) q0[d] = fma(y, r[d], q0[d]);
            pk = fmaxf(pk, fabsf(u));
            px = fmaxf(px, fabsf(xc));
        } else {
            const double w0 = v[0], w1 = v[1], w2 = v[2], w3 = v[3];
            const double a = bq_step(c1, v[0], v[1], ud);
            double y = hp_step(c2, v[2], v[3], a);
            const bool in = n < len;              // past a partial segment's end: state held
            v[0] = in ? v[0] : w0; v[1] = in ? v[1] : w1;
            v[2] = in ? v[2] : w2; v[3] = in ? v[3] : w3;
            y = in ? y : 0.0;
            if (n < split) {
                z0 = fma(y, y, z0);
#pragma unroll
                for (int d = 0; d < 4; d++) q0[d] = fma(y, r[d], q0[d]);
            } else {
                z1 = fma(y, y, z1);
#pragma unroll
                for (int d = 0; d < 4; d++) q1[d] = fma(y, r[d], q1[d]);
            }
            pk = in ? fmaxf(pk, fabsf(u)) : pk;
            px = in ? fmaxf(px, fabsf(xc)) : px;
        }
    }
};

// The fast kernel: STATIC = L (M == 1), a segment that is whole, inside one hop and
// away from the span ends (the plan lists the others for k_up_slow): unrolled window
// blocks of TB input frames, outputs at phases 0 .. L-1 of every frame, phase 0 the
// frame itself.  zp: an LDS word holding 0, read every block so LLVM cannot hoist the
// bank rows out of the block loop (all rows at once would not fit the SGPRs).
template <int STATIC>
__device__ __forceinline__ void up_run_fast(const UpArgs &a, const SpanDev &sp, int ch, int64_t g0,
                                            bool vec, const int *zp, UpAcc<true> &acc) {
    constexpr int TB = AMX_UP_TB;
    constexpr int W = TB + UP_TAPS - 1;                        // inputs [k0 - 15, k0 + TB + 16)
    float w[W];
    const uint32_t *xp = a.x + sp.out_off + g0 - UP_C;         // frame g0 - 15
#pragma unroll
    for (int i = 0; i < W; i++) w[i] = up_sample(xp[i], ch);
    const int nblk = a.Lin / TB;
    for (int b = 0; b < nblk; b++) {
        // next block's new frames in flight while this block computes (past the last
        // block: frames of this one again, in range, unused)
        uint32_t nx[TB];
        const int o0 = (b + 1 < nblk ? (b + 1) * TB : b * TB) + (W - TB);
        if (vec) {                                              // 16-B aligned rows
#pragma unroll
            for (int i = 0; i < TB; i += 4) {
                const uint4 q = *reinterpret_cast<const uint4 *>(xp + o0 + i);
                nx[i] = q.x; nx[i + 1] = q.y; nx[i + 2] = q.z; nx[i + 3] = q.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < TB; i++) nx[i] = xp[o0 + i];
        }
        const int nb0 = b * TB * STATIC;
        const float *bk = a.bank + __builtin_amdgcn_readfirstlane(zp[b & 1]);
#pragma unroll
        for (int kb = 0; kb < TB; kb++) {
            // outputs of frame kb in order; the scheduling barriers keep one output's
            // scalar rows (bank row, C A^n row) in its own region: pulled ahead, the
            // block's rows would not fit the SGPRs
            __builtin_amdgcn_sched_barrier(AMX_UP_SB);
            const int n0 = nb0 + kb * STATIC;
            acc.add(n0, w[kb + UP_C], w[kb + UP_C]);
#pragma unroll
            for (int ph = 1; ph < STATIC; ph++) {
                __builtin_amdgcn_sched_barrier(AMX_UP_SB);
                acc.add(n0 + ph, UP_DOT(w + kb, bk + ph * UP_TAPS), w[kb + UP_C]);
            }
        }
        __builtin_amdgcn_sched_barrier(AMX_UP_SB);
#pragma unroll
        for (int i = 0; i < W - TB; i++) w[i] = w[i + TB];
#pragma unroll
        for (int i = 0; i < TB; i++) w[W - TB + i] = up_sample(nx[i], ch);
    }
}

template <class Acc>
__device__ __forceinline__ void acc_init(const UpArgs &a, Acc &acc, int split, int len) {
#pragma unroll
    for (int i = 0; i < 3; i++) { acc.c1[i] = a.cd->kw1[i]; acc.c2[i] = a.cd->kw2[i]; }
    acc.c1[3] = a.cd->kw1[4]; acc.c1[4] = a.cd->kw1[5];
    acc.c2[3] = a.cd->kw2[4]; acc.c2[4] = a.cd->kw2[5];
#pragma unroll
    for (int d = 0; d < 4; d++) { acc.v[d] = 0.0; acc.q0[d] = 0.0; acc.q1[d] = 0.0; }
    acc.z0 = acc.z1 = 0.0;
    acc.pk = acc.px = 0.0f;
    acc.split = split;
    acc.len = len;
    acc.wc = a.G;
}

template <class Acc>
__device__ __forceinline__ void acc_store(const UpArgs &a, const Acc &acc, int64_t j, int ch) {
    double *o = a.e + (j * 2 + ch) * AMX_KW_DIM;
#pragma unroll
    for (int d = 0; d < AMX_KW_DIM; d++) o[d] = acc.v[d];
    uint32_t *q = a.pk + j * 4;
    q[ch] = __float_as_uint(acc.pk);
    q[2 + ch] = (uint32_t)(acc.px * 32768.0f);      // |s16| / 32768: exact
    // energy terms: [piece][sum yz^2, sum yz (C A^n)^T (4)]
    double *t = a.eterms + (j * 2 + ch) * 10;
    t[0] = acc.z0;
    t[5] = acc.z1;
#pragma unroll
    for (int d = 0; d < 4; d++) { t[1 + d] = acc.q0[d]; t[6 + d] = acc.q1[d]; }
}

__device__ __forceinline__ bool up_fast_seg(const UpArgs &a, const KwSegDev &sg, const SpanDev &sp) {
    const int64_t g0 = sg.out_pos - sp.out_off;
    const int64_t h0 = sg.tframe / a.hop;
    const int64_t split = (h0 + 1) * a.hop - sg.tframe;
    return g0 - UP_C >= 0 && g0 + a.Lin + UP_TAPS - UP_C <= sp.out_n && sg.len == a.Lout &&
           split >= a.Lout;
}

// k_up_edge's work in chunks of AMX_UPE_CH outputs, for the first workgroups of k_up
// (below): a left-over segment's frames in LDS, the resampled samples and the K filter's
// outputs of one chunk at a time (5 KB instead of k_up_edge's 12 KB, so the fast
// kernel's own workgroups keep their occupancy).  Every sum keeps k_up_edge's order:
// lane l still accumulates outputs l, l + 64, ... in turn (chunks are multiples of 64),
// and the K filter runs on, serially, from chunk to chunk.  A k_up_edge beside k_up
// needed a fork and a join in the step's graph; the join alone cost ~10 us.
#define AMX_UPE_CH 128
#define AMX_UPE_NF 544            // frames staged: Lin + 32 <= 544 (static paths: Lin <= 480)
__device__ __forceinline__ void up_edge_chunked(const UpArgs &a, int64_t j, uint32_t *fr, float *us,
                                                double *ys) {
    const int lane = threadIdx.x & 63;
    const KwSegDev sg = a.ks[j];
    const SpanDev sp = a.spans[sg.track];
    const int t = sg.track;
    const int64_t g0 = sg.out_pos - sp.out_off;
    const int nf = a.Lin + UP_TAPS;                               // frames g0 - 15 + [0, nf)
    for (int i = lane; i < nf; i += 64) fr[i] = up_word(a.x, a.edge, sp, t, g0 - UP_C + i);
    __syncthreads();
    const int len = sg.len;
    const int ch = lane & 1;
    float pk = 0.0f, px = 0.0f;
    double c1[5], c2[5];
#pragma unroll
    for (int k = 0; k < 3; k++) { c1[k] = a.cd->kw1[k]; c2[k] = a.cd->kw2[k]; }
    c1[3] = a.cd->kw1[4]; c1[4] = a.cd->kw1[5];
    c2[3] = a.cd->kw2[4]; c2[4] = a.cd->kw2[5];
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    const int64_t h0 = sg.tframe / a.hop;
    const int split = (int)((h0 + 1) * a.hop - sg.tframe);
    double acc[2][2][5] = {};                                     // [ch][piece][term]
    for (int n0 = 0; n0 < a.Lout; n0 += AMX_UPE_CH) {
        const int nc = a.Lout - n0 < AMX_UPE_CH ? a.Lout - n0 : AMX_UPE_CH;
        for (int i = lane; i < 2 * nc; i += 64) {                 // i & 1 == ch
            const int n = n0 + (i >> 1);
            const int kb = a.obase[n], ph = a.oph[n];
            float w[UP_TAPS];
#pragma unroll
            for (int k = 0; k < UP_TAPS; k++) w[k] = up_sample(fr[kb + k], ch);
            const float u = (a.static_l > 0 && ph == 0) ? w[UP_C] : up_dot(w, a.bank + ph * UP_TAPS);
            us[i] = u;
            if (n < len) {
                pk = fmaxf(pk, fabsf(u));
                px = fmaxf(px, fabsf(w[UP_C]));
            }
        }
        __syncthreads();
        // the K filter recursion, one lane per channel, on from the previous chunk
        if (lane < 2) {
            for (int k = 0; k < nc; k++) {
                const int n = n0 + k;
                ys[2 * k + ch] = n < len ? hp_step(c2, v[2], v[3], bq_step(c1, v[0], v[1], (double)us[2 * k + ch]))
                                         : 0.0;
            }
        }
        __syncthreads();
        for (int k = lane; k < nc; k += 64) {
            const int n = n0 + k;
            if (n >= len) continue;
            const double *r = a.G + (int64_t)n * AMX_KW_DIM;
            const int pc = n < split ? 0 : 1;
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const double y = ys[2 * k + c];
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const double yy = q == pc ? y : 0.0;
                    acc[c][q][0] = fma(yy, yy, acc[c][q][0]);
#pragma unroll
                    for (int d = 0; d < 4; d++) acc[c][q][1 + d] = fma(yy, r[d], acc[c][q][1 + d]);
                }
            }
        }
        __syncthreads();                                          // us / ys are rewritten next chunk
    }
#pragma unroll
    for (int o = 2; o < 64; o <<= 1) {                            // max over the channel's lanes
        pk = fmaxf(pk, __shfl_xor(pk, o));
        px = fmaxf(px, __shfl_xor(px, o));
    }
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
            for (int k = 0; k < 5; k++) {
                double x = acc[c][q][k];
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o);
                acc[c][q][k] = x;
            }
    if (lane < 2) {
        double *o = a.e + (j * 2 + ch) * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) o[d] = v[d];
        uint32_t *pq = a.pk + j * 4;
        pq[ch] = __float_as_uint(pk);
        pq[2 + ch] = (uint32_t)(px * 32768.0f);
        double *te = a.eterms + (j * 2 + ch) * 10;
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
            for (int k = 0; k < 5; k++) te[q * 5 + k] = ch ? acc[1][q][k] : acc[0][q][k];
    }
}

// one lane per (segment, channel); lanes of segments k_up_slow owns return at once
template <int STATIC>
__global__ void __launch_bounds__(AMX_UP_BLOCK) __attribute__((amdgpu_waves_per_eu(AMX_UP_WAVES)))
k_up(UpArgs a, int n_edge) {
    __shared__ int zp[2];
    const int lane = threadIdx.x;
    if ((int)blockIdx.x < n_edge) {                      // the left-over segments first
        __shared__ __attribute__((aligned(16))) uint32_t fr[AMX_UPE_NF];
        __shared__ __attribute__((aligned(16))) float us[2 * AMX_UPE_CH];
        __shared__ __attribute__((aligned(16))) double ys[2 * AMX_UPE_CH];
        up_edge_chunked(a, a.slow[blockIdx.x], fr, us, ys);
        return;
    }
    if (lane < 2) zp[lane] = 0;
    __syncthreads();
    const int ch = lane & 1;
    const int64_t j = (int64_t)(blockIdx.x - n_edge) * (AMX_UP_BLOCK / 2) + (lane >> 1);
    if (j >= a.n_kseg) return;
    const KwSegDev sg = a.ks[j];
    const SpanDev sp = a.spans[sg.track];
    if (!up_fast_seg(a, sg, sp)) return;
    const int64_t g0 = sg.out_pos - sp.out_off;
    // 16-B loads when every lane's window rows are 16-B aligned
    const bool vec = __ballot(((sp.out_off + g0 - UP_C + (UP_TAPS - 1)) & 3) != 0) == 0;
    UpAcc<true> acc;
    acc_init(a, acc, a.Lout, a.Lout);
    up_run_fast<STATIC>(a, sp, ch, g0, vec, zp, acc);
    acc_store(a, acc, j, ch);
}

// M > 1 rates (44.1 / 88.2 / 176.4 kHz) and the M == 1 rates without an unrolled phase
// loop (32 / 64 kHz): k_up's register window of TB + 31 frames, taken frame by frame.
// Frame kb of a block is the base of cnt consecutive outputs (CMIN <= cnt <= CMAX, the
// plan's per-frame table fcnt: the phase pattern is the same for every segment, so the
// count is wave-uniform).  Output n's bank row is row n of the plan's table in output
// order (bankn[n] = bank[oph[n]]): a scalar load at an address the output counter gives,
// where k_up_slow first loads obase[n] and oph[n] and only then the row, and moves its
// window one frame at a time through masked, bounds-tested loads.  The segments this
// kernel leaves (span ends, partial segments, hop splits) go to k_up_edge, as for k_up.
template <int CMIN, int CMAX, int TB>
__global__ void __launch_bounds__(AMX_UP_BLOCK) __attribute__((amdgpu_waves_per_eu(AMX_UP_WAVES)))
k_up_poly(UpArgs a) {
    static_assert(CMIN >= 1 && CMIN <= CMAX, "every frame is the base of >= 1 output");
    const int lane = threadIdx.x;
    const int ch = lane & 1;
    const int64_t j = (int64_t)blockIdx.x * (AMX_UP_BLOCK / 2) + (lane >> 1);
    if (j >= a.n_kseg) return;
    const KwSegDev sg = a.ks[j];
    const SpanDev sp = a.spans[sg.track];
    if (!up_fast_seg(a, sg, sp)) return;
    const int64_t g0 = sg.out_pos - sp.out_off;
    UpAcc<true> acc;
    acc_init(a, acc, a.Lout, a.Lout);
    constexpr int W = TB + UP_TAPS - 1;                        // inputs [k0 - 15, k0 + TB + 16)
    float w[W];
    const uint32_t *xp = a.x + sp.out_off + g0 - UP_C;         // frame g0 - 15
#pragma unroll
    for (int i = 0; i < W; i++) w[i] = up_sample(xp[i], ch);
    const int nblk = a.Lin / TB;
    int n = 0;                                                 // next output (wave-uniform)
    // the rows of output n (bank row, C A^n row) are loaded while output n - 1 computes:
    // 40 scalar registers in flight instead of a scalar-cache miss on every output (the
    // 640 rows of 44.1 kHz are 80 KB)
    float h[UP_TAPS];
    double r[AMX_KW_DIM];
#pragma unroll
    for (int i = 0; i < UP_TAPS; i++) h[i] = a.bankn[i];
#pragma unroll
    for (int d = 0; d < AMX_KW_DIM; d++) r[d] = a.G[d];
    for (int b = 0; b < nblk; b++) {
        uint32_t nx[TB];
        const int o0 = (b + 1 < nblk ? (b + 1) * TB : b * TB) + (W - TB);
#pragma unroll
        for (int i = 0; i < TB; i++) nx[i] = xp[o0 + i];
        const int32_t *cn = a.fcnt + b * TB;
#pragma unroll
        for (int kb = 0; kb < TB; kb++) {
            const int c = cn[kb];
#pragma unroll
            for (int o = 0; o < CMAX; o++) {
                if (o < CMIN || o < c) {
                    __builtin_amdgcn_sched_barrier(AMX_UP_SB);
                    const int nn = n + 1 < a.Lout ? n + 1 : n;
                    float hn[UP_TAPS];
                    double rn[AMX_KW_DIM];
                    const float *hp = a.bankn + (int64_t)nn * UP_TAPS;
                    const double *rp = a.G + (int64_t)nn * AMX_KW_DIM;
#pragma unroll
                    for (int i = 0; i < UP_TAPS; i++) hn[i] = hp[i];
#pragma unroll
                    for (int d = 0; d < AMX_KW_DIM; d++) rn[d] = rp[d];
                    acc.add_row(n, UP_DOT(w + kb, h), w[kb + UP_C], r);
#pragma unroll
                    for (int i = 0; i < UP_TAPS; i++) h[i] = hn[i];
#pragma unroll
                    for (int d = 0; d < AMX_KW_DIM; d++) r[d] = rn[d];
                    n++;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(AMX_UP_SB);
#pragma unroll
        for (int i = 0; i < W - TB; i++) w[i] = w[i + TB];
#pragma unroll
        for (int i = 0; i < TB; i++) w[W - TB + i] = up_sample(nx[i], ch);
    }
    acc_store(a, acc, j, ch);
}

// the (CMIN, CMAX, TB) forms k_up_poly is built for
#define AMX_UP_POLY_FORMS(X) X(4, 5, 7) X(2, 3, 7) X(1, 2, 7) X(6, 6, 8) X(3, 3, 8)

int up_poly_form(int cmin, int cmax, int tb) {
#define AMX_UP_POLY_HAS(c0, c1, t) if (cmin == c0 && cmax == c1 && tb == t) return AMX_UP_POLY(c0, c1, t);
    AMX_UP_POLY_FORMS(AMX_UP_POLY_HAS)
#undef AMX_UP_POLY_HAS
    return 0;
}

// The general kernel, over the plan's list of the segments k_up does not take (span
// ends, partial segments, hop splits) -- or over every segment when the rate has no
// unrolled form (M > 1, e.g. 44.1 kHz: phase pattern from the tables, the window
// moves one frame at a time): neighbour / mirrored frames, masks, two hop pieces.
__global__ void __launch_bounds__(AMX_UP_BLOCK) k_up_slow(UpArgs a) {
    const int lane = threadIdx.x;
    const int ch = lane & 1;
    const int64_t q = (int64_t)blockIdx.x * (AMX_UP_BLOCK / 2) + (lane >> 1);
    if (q >= a.n_slow) return;
    const int64_t j = a.slow ? a.slow[q] : q;
    const KwSegDev sg = a.ks[j];
    const SpanDev sp = a.spans[sg.track];
    const int t = sg.track;
    const int64_t g0 = sg.out_pos - sp.out_off;
    const int64_t h0 = sg.tframe / a.hop;
    UpAcc<false> acc;
    acc_init(a, acc, (int)((h0 + 1) * a.hop - sg.tframe), sg.len);
    float w[UP_TAPS];
    for (int i = 0; i < UP_TAPS; i++) {
        const float v = up_sample(up_word(a.x, a.edge, sp, t, g0 - UP_C + i), ch);
#pragma unroll
        for (int k = 0; k < UP_TAPS; k++) w[k] = k == i ? v : w[k];
    }
    int cur = 0;
    for (int n = 0; n < a.Lout; n++) {
        const int kb = a.obase[n];
        if (kb > cur) {                                         // one frame on
#pragma unroll
            for (int i = 0; i < UP_TAPS - 1; i++) w[i] = w[i + 1];
            w[UP_TAPS - 1] = up_sample(up_word(a.x, a.edge, sp, t, g0 + cur + UP_TAPS - UP_C), ch);
            cur++;
        }
        const int ph = a.oph[n];
        const float u = a.lin ? swr_dot_lin(w, a.bank + ph * UP_TAPS, a.bank + (ph + 1) * UP_TAPS, a.owt[n])
                        : (a.static_l > 0 && ph == 0) ? w[UP_C] : up_dot(w, a.bank + ph * UP_TAPS);
        acc.add(n, u, w[UP_C]);
    }
    acc_store(a, acc, j, ch);
}

// The static path's left-over segments (span ends, partial segments, hop splits: a
// few per span), one wave per segment: the lane-per-segment form above would run each
// of them as one serial lane over Lout outputs, all taps and edge tests included --
// longer than the whole fast kernel.  Here the wave stages the segment's frames in LDS,
// computes the 2 x Lout resampled samples and the peaks in parallel, and only the K
// filter recursion (one lane per channel) stays serial.
__global__ void __launch_bounds__(64) k_up_edge(UpArgs a) {
    extern __shared__ uint32_t sh[];
    const int lane = threadIdx.x;
    const int64_t j = a.slow[blockIdx.x];
    const KwSegDev sg = a.ks[j];
    const SpanDev sp = a.spans[sg.track];
    const int t = sg.track;
    const int64_t g0 = sg.out_pos - sp.out_off;
    const int nf = a.Lin + UP_TAPS;                               // frames g0 - 15 + [0, nf)
    uint32_t *fr = sh;
    float *us = reinterpret_cast<float *>(sh + nf);               // [n][ch]
    for (int i = lane; i < nf; i += 64) fr[i] = up_word(a.x, a.edge, sp, t, g0 - UP_C + i);
    __syncthreads();
    const int len = sg.len;
    const int ch = lane & 1;
    float pk = 0.0f, px = 0.0f;
    for (int i = lane; i < 2 * a.Lout; i += 64) {                 // i & 1 == ch
        const int n = i >> 1;
        const int kb = a.obase[n], ph = a.oph[n];
        float w[UP_TAPS];
#pragma unroll
        for (int k = 0; k < UP_TAPS; k++) w[k] = up_sample(fr[kb + k], ch);
        const float u = a.lin ? swr_dot_lin(w, a.bank + ph * UP_TAPS, a.bank + (ph + 1) * UP_TAPS, a.owt[n])
                        : (a.static_l > 0 && ph == 0) ? w[UP_C] : up_dot(w, a.bank + ph * UP_TAPS);
        us[i] = u;
        if (n < len) {
            pk = fmaxf(pk, fabsf(u));
            px = fmaxf(px, fabsf(w[UP_C]));
        }
    }
#pragma unroll
    for (int o = 2; o < 64; o <<= 1) {                            // max over the channel's lanes
        pk = fmaxf(pk, __shfl_xor(pk, o));
        px = fmaxf(px, __shfl_xor(px, o));
    }
    __syncthreads();
    // the K filter recursion, one lane per channel: y_n into LDS (0 past len)
    double *ys = reinterpret_cast<double *>(sh + ((nf + 2 * a.Lout + 1) & ~1));   // [n][ch]
    if (lane < 2) {
        double c1[5], c2[5];
#pragma unroll
        for (int k = 0; k < 3; k++) { c1[k] = a.cd->kw1[k]; c2[k] = a.cd->kw2[k]; }
        c1[3] = a.cd->kw1[4]; c1[4] = a.cd->kw1[5];
        c2[3] = a.cd->kw2[4]; c2[4] = a.cd->kw2[5];
        double v[4] = {0.0, 0.0, 0.0, 0.0};
        int n = 0;
        for (; n + 8 <= len; n += 8) {
            float ub[8];
#pragma unroll
            for (int k = 0; k < 8; k++) ub[k] = us[2 * (n + k) + ch];
#pragma unroll
            for (int k = 0; k < 8; k++)
                ys[2 * (n + k) + ch] = hp_step(c2, v[2], v[3], bq_step(c1, v[0], v[1], (double)ub[k]));
        }
        for (; n < len; n++)
            ys[2 * n + ch] = hp_step(c2, v[2], v[3], bq_step(c1, v[0], v[1], (double)us[2 * n + ch]));
        for (; n < a.Lout; n++) ys[2 * n + ch] = 0.0;
        double *o = a.e + (j * 2 + ch) * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) o[d] = v[d];
        uint32_t *pq = a.pk + j * 4;
        pq[ch] = __float_as_uint(pk);
        pq[2 + ch] = (uint32_t)(px * 32768.0f);
    }
    __syncthreads();
    // energy terms per hop piece, all lanes: sum y^2, sum y (C A^n)^T
    const int64_t h0 = sg.tframe / a.hop;
    const int split = (int)((h0 + 1) * a.hop - sg.tframe);
    double acc[2][2][5] = {};                                     // [ch][piece][term]
    for (int n = lane; n < len; n += 64) {
        const double *r = a.G + (int64_t)n * AMX_KW_DIM;
        const int pc = n < split ? 0 : 1;
#pragma unroll
        for (int c = 0; c < 2; c++) {
            const double y = ys[2 * n + c];
#pragma unroll
            for (int p = 0; p < 2; p++) {
                const double yy = p == pc ? y : 0.0;
                acc[c][p][0] = fma(yy, yy, acc[c][p][0]);
#pragma unroll
                for (int d = 0; d < 4; d++) acc[c][p][1 + d] = fma(yy, r[d], acc[c][p][1 + d]);
            }
        }
    }
#pragma unroll
    for (int c = 0; c < 2; c++)
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int k = 0; k < 5; k++) {
                double x = acc[c][p][k];
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o);
                acc[c][p][k] = x;
            }
    if (lane < 2) {
        double *te = a.eterms + (j * 2 + ch) * 10;
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int k = 0; k < 5; k++) te[p * 5 + k] = ch ? acc[1][p][k] : acc[0][p][k];
    }
}

// the FMA3 kernel's order over a row of `alloc` taps (a multiple of 8: the downsampling
// filters of inputs above 192 kHz), the window's frames read from LDS: 8 chains over taps
// k, k + 8, ..., then the common horizontal sum
__device__ __forceinline__ float up_dot_wide(const uint32_t *fr, int ch, const float *__restrict__ h, int alloc) {
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float acc = up_sample(fr[k], ch) * h[k];
        for (int q = 8; q < alloc; q += 8) acc = fmaf(up_sample(fr[k + q], ch), h[k + q], acc);
        a[k] = acc;
    }
    const float b0 = a[0] + a[4], b1 = a[1] + a[5], b2 = a[2] + a[6], b3 = a[3] + a[7];
    return (b0 + b2) + (b1 + b3);
}

// Every K segment of a downsampling rate (an input above 192 kHz / 0.97: 352.8, 384,
// 705.6, 768 kHz; the filter has `taps` > 32 taps in rows of `alloc`), one wave per
// segment as k_up_edge: the segment's frames staged in LDS from g0 - center, the 2 x Lout
// outputs in parallel, the K filter on one lane per channel, the energy terms reduced
// over the wave.  The window of output n is frames obase[n] - center .. + alloc - 1 (the
// row's zero padding multiplies the frames after it, as the x86 kernel does).
__global__ void __launch_bounds__(64) k_up_wide(UpArgs a) {
    extern __shared__ uint32_t sh[];
    const int lane = threadIdx.x;
    const int64_t j = a.slow ? a.slow[blockIdx.x] : (int64_t)blockIdx.x;
    const KwSegDev sg = a.ks[j];
    const SpanDev sp = a.spans[sg.track];
    const int t = sg.track;
    const int64_t g0 = sg.out_pos - sp.out_off;
    const int c = (a.taps - 1) / 2;
    const int nf = a.Lin + a.alloc;                               // frames g0 - c + [0, nf)
    uint32_t *fr = sh;
    float *us = reinterpret_cast<float *>(sh + nf);               // [n][ch]
    for (int i = lane; i < nf; i += 64) fr[i] = up_word(a.x, a.edge, sp, t, g0 - c + i);
    __syncthreads();
    const int len = sg.len;
    const int ch = lane & 1;
    float pk = 0.0f, px = 0.0f;
    for (int i = lane; i < 2 * a.Lout; i += 64) {                 // i & 1 == ch
        const int n = i >> 1;
        const int kb = a.obase[n], ph = a.oph[n];
        const float u = up_dot_wide(fr + kb, ch, a.bank + (int64_t)ph * a.alloc, a.alloc);
        us[i] = u;
        if (n < len) {
            pk = fmaxf(pk, fabsf(u));
            px = fmaxf(px, fabsf(up_sample(fr[kb + c], ch)));
        }
    }
#pragma unroll
    for (int o = 2; o < 64; o <<= 1) {                            // max over the channel's lanes
        pk = fmaxf(pk, __shfl_xor(pk, o));
        px = fmaxf(px, __shfl_xor(px, o));
    }
    __syncthreads();
    double *ys = reinterpret_cast<double *>(sh + ((nf + 2 * a.Lout + 1) & ~1));   // [n][ch]
    if (lane < 2) {
        double c1[5], c2[5];
#pragma unroll
        for (int k = 0; k < 3; k++) { c1[k] = a.cd->kw1[k]; c2[k] = a.cd->kw2[k]; }
        c1[3] = a.cd->kw1[4]; c1[4] = a.cd->kw1[5];
        c2[3] = a.cd->kw2[4]; c2[4] = a.cd->kw2[5];
        double v[4] = {0.0, 0.0, 0.0, 0.0};
        int n = 0;
        for (; n < len; n++)
            ys[2 * n + ch] = hp_step(c2, v[2], v[3], bq_step(c1, v[0], v[1], (double)us[2 * n + ch]));
        for (; n < a.Lout; n++) ys[2 * n + ch] = 0.0;
        double *o = a.e + (j * 2 + ch) * AMX_KW_DIM;
#pragma unroll
        for (int d = 0; d < AMX_KW_DIM; d++) o[d] = v[d];
        uint32_t *pq = a.pk + j * 4;
        pq[ch] = __float_as_uint(pk);
        pq[2 + ch] = (uint32_t)(px * 32768.0f);
    }
    __syncthreads();
    const int64_t h0 = sg.tframe / a.hop;
    const int split = (int)((h0 + 1) * a.hop - sg.tframe);
    double acc[2][2][5] = {};                                     // [ch][piece][term]
    for (int n = lane; n < len; n += 64) {
        const double *r = a.G + (int64_t)n * AMX_KW_DIM;
        const int pc = n < split ? 0 : 1;
#pragma unroll
        for (int cc = 0; cc < 2; cc++) {
            const double y = ys[2 * n + cc];
#pragma unroll
            for (int p = 0; p < 2; p++) {
                const double yy = p == pc ? y : 0.0;
                acc[cc][p][0] = fma(yy, yy, acc[cc][p][0]);
#pragma unroll
                for (int d = 0; d < 4; d++) acc[cc][p][1 + d] = fma(yy, r[d], acc[cc][p][1 + d]);
            }
        }
    }
#pragma unroll
    for (int cc = 0; cc < 2; cc++)
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int k = 0; k < 5; k++) {
                double x = acc[cc][p][k];
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) x += __shfl_xor(x, o);
                acc[cc][p][k] = x;
            }
    if (lane < 2) {
        double *te = a.eterms + (j * 2 + ch) * 10;
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int k = 0; k < 5; k++) te[p * 5 + k] = ch ? acc[1][p][k] : acc[0][p][k];
    }
}

// hop pieces' energies from the exact start states: E = sum yz^2 + 2 s.q + s^T Q s,
// Q the piece's Gram matrix of the rows C A^n (plan tables: head Qh[k] = sum_{n<k},
// tail Qt[k] = sum_{k<=n<Lout}); one thread per (segment, channel)
__global__ void __launch_bounds__(AMX_BLOCK) k_up_energy(UpArgs a) {
    const int64_t i = (int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x;
    if (i >= 2 * (int64_t)a.n_kseg) return;
    const int64_t j = i >> 1;
    const int ch = (int)(i & 1);
    const KwSegDev sg = a.ks[j];
    const int64_t h0 = sg.tframe / a.hop;
    const int split = (int)((h0 + 1) * a.hop - sg.tframe);
    const int len = sg.len;
    const double *s = a.s + (j * 2 + ch) * AMX_KW_DIM;
    const double *t = a.eterms + (j * 2 + ch) * 10;
    double sv[4];
#pragma unroll
    for (int d = 0; d < 4; d++) sv[d] = s[d];
    auto quad = [&](const double *Q) {           // s^T Q s
        double r = 0.0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            double row = 0.0;
#pragma unroll
            for (int w = 0; w < 4; w++) row = fma(Q[u * 4 + w], sv[w], row);
            r = fma(sv[u], row, r);
        }
        return r;
    };
    const int e0 = split < len ? split : len;    // piece 0 = outputs [0, e0)
    const double *Qh = a.qh + (int64_t)e0 * 16;
    double E0 = t[0], E1 = 0.0;
    double c0 = 0.0, c1 = 0.0;
#pragma unroll
    for (int d = 0; d < 4; d++) { c0 = fma(sv[d], t[1 + d], c0); c1 = fma(sv[d], t[6 + d], c1); }
    E0 = E0 + 2.0 * c0 + quad(Qh);
    if (split < len) {                           // piece 1 = outputs [split, len)
        double Q[16];
        const double *Qa = a.qt + (int64_t)split * 16, *Qb = a.qt + (int64_t)len * 16;
#pragma unroll
        for (int k = 0; k < 16; k++) Q[k] = Qa[k] - Qb[k];
        E1 = t[5] + 2.0 * c1 + quad(Q);
    }
    double *o = a.parts + j * 4;
    o[ch] = E0;
    o[2 + ch] = E1;
    if (ch == 0) a.part_hop[j] = h0;
}

hipError_t launch_up1(const UpArgs &a, hipStream_t st, hipStream_t aux, hipEvent_t fork, hipEvent_t join) {
    if (a.n_kseg <= 0) return hipSuccess;
    const unsigned nblk = (unsigned)((a.n_kseg + AMX_UP_BLOCK / 2 - 1) / (AMX_UP_BLOCK / 2));
    if (a.static_l > 0 && !a.lin && a.Lin + UP_TAPS <= AMX_UPE_NF && a.n_slow < (1 << 20)) {
        // the left-over segments are k_up's first workgroups (dispatched first, so their
        // serial K filter overlaps the fast segments): no second stream, no join
        const unsigned ne = (unsigned)a.n_slow;
        switch (a.static_l) {
        case 1: hipLaunchKernelGGL(k_up<1>, dim3(ne + nblk), dim3(AMX_UP_BLOCK), 0, st, a, (int)ne); break;
        case 2: hipLaunchKernelGGL(k_up<2>, dim3(ne + nblk), dim3(AMX_UP_BLOCK), 0, st, a, (int)ne); break;
        case 4: hipLaunchKernelGGL(k_up<4>, dim3(ne + nblk), dim3(AMX_UP_BLOCK), 0, st, a, (int)ne); break;
        default: return hipErrorInvalidValue;
        }
    } else if (a.static_l > 0 || a.poly > 0) {
        // the left-over segments' kernel is latency-bound (a serial K-filter lane per
        // channel): it runs on the plan's second stream beside the fast kernel
        const bool side = a.n_slow > 0 && aux && fork && join;
        if (a.n_slow > 0) {
            hipStream_t es = side ? aux : st;
            if (side) {
                hipError_t e = hipEventRecord(fork, st);
                if (e == hipSuccess) e = hipStreamWaitEvent(aux, fork, 0);
                if (e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(k_up_edge, dim3((unsigned)a.n_slow), dim3(64),
                               (size_t)((a.Lin + UP_TAPS + 2 * a.Lout + 1) & ~1) * 4 + (size_t)a.Lout * 16,
                               es, a);
            if (side) {
                hipError_t e = hipEventRecord(join, aux);
                if (e != hipSuccess) return e;
            }
        }
        switch (a.static_l > 0 ? a.static_l : a.poly) {
        case 1: hipLaunchKernelGGL(k_up<1>, dim3(nblk), dim3(AMX_UP_BLOCK), 0, st, a, 0); break;
        case 2: hipLaunchKernelGGL(k_up<2>, dim3(nblk), dim3(AMX_UP_BLOCK), 0, st, a, 0); break;
        case 4: hipLaunchKernelGGL(k_up<4>, dim3(nblk), dim3(AMX_UP_BLOCK), 0, st, a, 0); break;
#define AMX_UP_POLY_CASE(c0, c1, t)                                                                  \
        case AMX_UP_POLY(c0, c1, t):                                                                 \
            hipLaunchKernelGGL((k_up_poly<c0, c1, t>), dim3(nblk), dim3(AMX_UP_BLOCK), 0, st, a); break;
        AMX_UP_POLY_FORMS(AMX_UP_POLY_CASE)
#undef AMX_UP_POLY_CASE
        default: return hipErrorInvalidValue;
        }
        if (side) {
            hipError_t e = hipStreamWaitEvent(st, join, 0);
            if (e != hipSuccess) return e;
        }
    } else if (a.taps != UP_TAPS) {
        const size_t nf = (size_t)a.Lin + a.alloc;
        hipLaunchKernelGGL(k_up_wide, dim3((unsigned)a.n_slow), dim3(64),
                           ((nf + 2 * (size_t)a.Lout + 1) & ~(size_t)1) * 4 + (size_t)a.Lout * 16, st, a);
    } else {
        hipLaunchKernelGGL(k_up_slow, dim3((unsigned)((a.n_slow + AMX_UP_BLOCK / 2 - 1) / (AMX_UP_BLOCK / 2))),
                           dim3(AMX_UP_BLOCK), 0, st, a);
    }
    return hipGetLastError();
}

hipError_t launch_up2(const UpArgs &a, hipStream_t st) {
    if (a.n_kseg <= 0) return hipSuccess;
    const int64_t n = 2 * (int64_t)a.n_kseg;
    hipLaunchKernelGGL(k_up_energy, dim3((unsigned)((n + AMX_BLOCK - 1) / AMX_BLOCK)), dim3(AMX_BLOCK), 0, st, a);
    return hipGetLastError();
}

}  // namespace amx
