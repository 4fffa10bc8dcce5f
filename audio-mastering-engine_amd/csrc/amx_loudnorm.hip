// amx_loudnorm.hip -- af_loudnorm's 192 kHz modes on one track (the reference's pass 1
// at :229 always runs them -- its target_offset is measured on their output -- and pass 2
// at :240 runs dynamic mode whenever the linear conditions fail).  Restated from FFmpeg
// af_loudnorm.c as the oracle does (oracle/amx_oracle.c orc_loudnorm, which cites the
// functions); this file follows the oracle's structure, not the reverse.
//
//   k_ln_upsample: the 192 kHz stream libswresample feeds the filter (the same float32
//     polyphase FIR, window and FMA3 summation order as amx_loud192.hip), stored once as
//     float32 [frames][2] -- the filter reads it up to 3 s behind its output.
//   k_ln_dyn: the filter itself, one workgroup per track.  af_loudnorm is a state machine
//     over 100 ms frames (the AGC gain of a frame depends on the previous frames'
//     decisions) whose true-peak limiter is a state machine over samples, so it runs in
//     order; the workgroup shares out the per-sample loops:
//       - the limiter ring fills (gain ramp x offset) and the output (clamp, s16);
//       - detect_peak: a block-wide minimum finds the first position that can be a peak
//         (prev <= |x| >= next, |x| > ceiling); only from there on is the scan serial
//         (a candidate that fails the 10-sample look-ahead keeps the previous sample,
//         so later positions depend on it);
//       - the envelope loops of ATTACK / SUSTAIN / RELEASE (each thread one sample);
//     and the scalar parts (Gaussian smoothing, statistics, delta, limiter state) are
//     carried by every thread alike.  The input-side loudness statistics af_loudnorm reads from r128_in
//     after each frame (3 s short-term, gated integrated, relative gate) come from the
//     hop energies loudness pass 1 measured on this same 192 kHz stream; the
//     histogram is rebuilt in LDS block by block.  r128_out (the output's short-term
//     loudness) is only read while above_threshold is 0; libebur128's K filter then runs
//     over the frame's output on two threads (one per channel).
// Floating point: no FMA contraction (the reference's C is compiled that way too,
// -ffp-contract=off in the oracle), so every expression keeps its operation order.
#include "amx_dev.hpp"

#pragma clang fp contract(off)

namespace amx {

#define LN_FR 19200          // frame_size(192000, 100)
#define LN_FIRST 576000      // frame_size(192000, 3000)
#define LN_LIMF 40320        // frame_size(192000, 210): limiter ring frames
#define LN_RSZ (2 * LN_LIMF) // limiter ring samples
#define LN_ATT 1920          // frame_size(192000, 10)
#define LN_TAPS 32
#define LN_C 15

// --------------------------------------------------------------- resampler
__device__ __forceinline__ int64_t ln_reflect(int64_t k, int64_t n) {
    for (int it = 0; it < 64; it++) {
        if (k < 0) k = -k;
        else if (k >= n) k = 2 * n - 1 - k;
        else return k;
    }
    return 0;
}

__device__ __forceinline__ float ln_dot(const float *w, const float *__restrict__ h) {
    float a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float acc = __builtin_fmaf(w[k], h[k], 0.0f);
        acc = __builtin_fmaf(w[k + 8], h[k + 8], acc);
        acc = __builtin_fmaf(w[k + 16], h[k + 16], acc);
        acc = __builtin_fmaf(w[k + 24], h[k + 24], acc);
        a[k] = acc;
    }
    const float b0 = a[0] + a[4], b1 = a[1] + a[5], b2 = a[2] + a[6], b3 = a[3] + a[7];
    return (b0 + b2) + (b1 + b3);
}

typedef float ln_f2 __attribute__((ext_vector_type(2)));
typedef unsigned lp_u4 __attribute__((ext_vector_type(4)));
#ifndef AMX_LP_HANDOFF
#define AMX_LP_HANDOFF 1     // k_lp_seg's boundary records: sc1 stores + one acquire (0: __threadfence form)
#endif

// ln_dot with the 8 chains as 4 packed pairs (v_pk_fma_f32 / v_pk_add_f32): the same
// operations lane by lane, the first term a fused multiply-add onto 0 as in ln_dot
template <class P>
__device__ __forceinline__ float ln_dot2(const float *w, P h) {
    ln_f2 acc4[4];
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
        ln_f2 acc = __builtin_elementwise_fma(ln_f2{w[k], w[k + 1]}, ln_f2{h[k], h[k + 1]}, ln_f2{0.0f, 0.0f});
        acc = __builtin_elementwise_fma(ln_f2{w[k + 8], w[k + 9]}, ln_f2{h[k + 8], h[k + 9]}, acc);
        acc = __builtin_elementwise_fma(ln_f2{w[k + 16], w[k + 17]}, ln_f2{h[k + 16], h[k + 17]}, acc);
        acc = __builtin_elementwise_fma(ln_f2{w[k + 24], w[k + 25]}, ln_f2{h[k + 24], h[k + 25]}, acc);
        acc4[k >> 1] = acc;
    }
    const ln_f2 b01 = acc4[0] + acc4[2], b23 = acc4[1] + acc4[3];
    const ln_f2 c = b01 + b23;
    return c.x + c.y;
}

// The M == 1 rates (192 kHz / L: 48 kHz L = 4, 96 kHz 2, 64 kHz 3, 32 kHz 6, 192 kHz 1):
// output j = frame j / L, phase j % L.  One thread per LN_UPF consecutive input frames:
// one window of 31 + LN_UPF frames (loaded once: 35 loads for 4 frames instead of 128),
// then every frame's L outputs with the bank rows as wave-uniform operands (k_ln_upsample's
// generic form pays two 64-bit divisions and a per-lane bank row for every output).
#define LN_UPF 4
// Stores (round 6): a thread's 4 frames are 32 L contiguous bytes, so the lanes' own
// stores had a 32 L-byte stride (one 16-B piece per 128-B line per instruction at 48 kHz:
// the writes, 461 MB for a 5-min track, ran at ~2.4 TB/s).  A workgroup whose 256 x 4
// frames are all in range stages its outputs in LDS and writes them as one contiguous
// block, 16 B per lane per instruction (AMX_LN_UPS_LDS; the others store directly).
#ifndef AMX_LN_UPS_LDS
#define AMX_LN_UPS_LDS 1
#endif
#ifndef AMX_LN_UPS_PH
#define AMX_LN_UPS_PH 1
#endif
template <int L>
__global__ void __launch_bounds__(AMX_BLOCK) k_ln_up_static(const uint32_t *__restrict__ x, int64_t n_in,
                                                            const float *__restrict__ bank, int64_t j0, int64_t j1,
                                                            float *__restrict__ u, const int32_t *__restrict__ gate) {
    if (AMX_LN_GATED(gate)) return;
    constexpr int NW = LN_TAPS + LN_UPF - 1;
    constexpr bool STAGE = AMX_LN_UPS_LDS && (L % 2 == 0);
    constexpr int TF = 2 * L * LN_UPF;                 // floats a thread produces
    __shared__ __attribute__((aligned(16))) float s_o[STAGE ? AMX_BLOCK * TF : 4];


    const int64_t f0 = j0 / L, f1 = (j1 + L - 1) / L;
    const int64_t nblk = (f1 - f0 + LN_UPF - 1) / LN_UPF;
    // workgroup-uniform iterations (the staged stores need the barriers)
    for (int64_t b0 = (int64_t)blockIdx.x * AMX_BLOCK; b0 < nblk; b0 += (int64_t)gridDim.x * AMX_BLOCK) {
        const int64_t bi = b0 + threadIdx.x;
        const bool act = bi < nblk;
        const int64_t fb = f0 + (act ? bi : b0) * LN_UPF;   // this thread's first frame
        float w0[NW], w1[NW];
        const int64_t g = fb - LN_C;
        static_assert(LN_UPF == 4 && LN_C % 4 == 3, "the 16-B window loads start one frame early");
        if (g >= 1 && g - 1 + NW + 1 <= n_in && ((reinterpret_cast<uintptr_t>(x + g - 1) & 15) == 0)) {
            // 16-B loads of frames g - 1 .. g + NW - 1 (g - 1 = fb - 16: 16-B aligned when x is)
            uint32_t wv[NW + 1];
#pragma unroll
            for (int i = 0; i < (NW + 1) / 4; i++) {
                const uint4 q = *reinterpret_cast<const uint4 *>(x + g - 1 + 4 * i);
                wv[4 * i] = q.x; wv[4 * i + 1] = q.y; wv[4 * i + 2] = q.z; wv[4 * i + 3] = q.w;
            }
#pragma unroll
            for (int i = 0; i < NW; i++) {
                w0[i] = (float)lo16(wv[i + 1]) * (1.0f / 32768.0f);
                w1[i] = (float)hi16(wv[i + 1]) * (1.0f / 32768.0f);
            }
        } else if (g >= 0 && g + NW <= n_in) {
#pragma unroll
            for (int i = 0; i < NW; i++) {
                const uint32_t v = x[g + i];
                w0[i] = (float)lo16(v) * (1.0f / 32768.0f);
                w1[i] = (float)hi16(v) * (1.0f / 32768.0f);
            }
        } else {
#pragma unroll
            for (int i = 0; i < NW; i++) {
                const uint32_t v = x[ln_reflect(g + i, n_in)];
                w0[i] = (float)lo16(v) * (1.0f / 32768.0f);
                w1[i] = (float)hi16(v) * (1.0f / 32768.0f);
            }
        }
        // the whole workgroup's outputs in range: frames f0 + 4 b0 .. + 4 * AMX_BLOCK
        const int64_t fw = f0 + b0 * LN_UPF;
        const bool whole = STAGE && b0 + AMX_BLOCK <= nblk && fw * L >= j0 &&
                           (fw + (int64_t)AMX_BLOCK * LN_UPF) * L <= j1 && fw + (int64_t)AMX_BLOCK * LN_UPF <= f1;
#if AMX_LN_UPS_PH
        // a (frame, phase)'s 32 bank taps are scalar operands loaded just before its two
        // dots: the load address depends on the previous dot's result, so the compiler
        // cannot hoist every frame's and phase's taps together (all 32 L at once: 128 SGPRs
        // at L = 4, spilled to VGPR lanes, 332 v_readlane per pass beside 512 v_pk_fma)
        typedef const __attribute__((address_space(4))) float *ConstF;
        float dep = 0.0f;
#endif
#pragma unroll
        for (int k = 0; k < LN_UPF; k++) {
            const int64_t f = fb + k;
            float o[2 * L];
#pragma unroll
            for (int ph = 0; ph < L; ph++) {
#if AMX_LN_UPS_PH
                uint64_t bp = reinterpret_cast<uint64_t>(bank + ph * LN_TAPS);
                asm volatile("" : "+s"(bp) : "v"(dep));
                const ConstF h = (ConstF)bp;
#else
                const float *h = bank + ph * LN_TAPS;
#endif
                o[2 * ph] = ln_dot2(w0 + k, h);
                o[2 * ph + 1] = ln_dot2(w1 + k, h);
#if AMX_LN_UPS_PH
                dep = o[2 * ph + 1];
#endif
            }
            if constexpr (STAGE) {
                if (whole) {
#pragma unroll
                    for (int q = 0; q < L / 2; q++)
                        *reinterpret_cast<float4 *>(s_o + threadIdx.x * TF + k * 2 * L + 4 * q) =
                            make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
                    continue;
                }
            }
            if (!act || f >= f1) continue;
            bool done = false;
            if constexpr (L % 2 == 0) {
                // the frame's L outputs are 8 L contiguous bytes: 16-B stores when all are
                // in range
                if (f * L >= j0 && f * L + L <= j1) {
#pragma unroll
                    for (int q = 0; q < L / 2; q++)
                        *reinterpret_cast<float4 *>(u + 2 * (f * L) + 4 * q) =
                            make_float4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
                    done = true;
                }
            }
            if (!done) {
#pragma unroll
                for (int ph = 0; ph < L; ph++) {
                    const int64_t j = f * L + ph;
                    if (j >= j0 && j < j1) *reinterpret_cast<float2 *>(u + 2 * j) = make_float2(o[2 * ph], o[2 * ph + 1]);
                }
            }
        }
        if constexpr (STAGE) {
            if (whole) {                                     // workgroup-uniform
                __syncthreads();
                float4 *dst = reinterpret_cast<float4 *>(u + 2 * fw * L);
                const float4 *src = reinterpret_cast<const float4 *>(s_o);
#pragma unroll
                for (int q = 0; q < TF / 4; q++) dst[q * AMX_BLOCK + threadIdx.x] = src[q * AMX_BLOCK + threadIdx.x];
                __syncthreads();                             // s_o is rewritten next pass
            }
        }
    }
}

// dispatch: the static form for M == 1 rates, else the generic one
static void ln_upsample(const uint32_t *x, int64_t n_in, const SwrDev &r, int64_t j0, int64_t j1, float *u,
                        const int32_t *gate, hipStream_t st);

// one thread per 192 kHz frame: both channels, frames [j0, j1).  Output j sits at phase
// position j dst / src past input frame 0 (exact rates: j M / L, frac 0)
__global__ void __launch_bounds__(AMX_BLOCK) k_ln_upsample(const uint32_t *__restrict__ x, int64_t n_in,
                                                           SwrDev r, int64_t j0, int64_t j1, float *__restrict__ u,
                                                           const int32_t *__restrict__ gate) {
    if (AMX_LN_GATED(gate)) return;
    for (int64_t j = j0 + (int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x; j < j1; j += (int64_t)gridDim.x * AMX_BLOCK) {
        const int64_t pos = j * r.dst, idx = pos / r.src;
        const int64_t base = idx / r.pc;
        const int ph = (int)(idx % r.pc);
        float w0[LN_TAPS], w1[LN_TAPS];
#pragma unroll
        for (int i = 0; i < LN_TAPS; i++) {
            const uint32_t v = x[ln_reflect(base - LN_C + i, n_in)];
            w0[i] = (float)lo16(v) * (1.0f / 32768.0f);
            w1[i] = (float)hi16(v) * (1.0f / 32768.0f);
        }
        const float *h = r.bank + (int64_t)ph * LN_TAPS;
        if (r.lin) {
            const float wf = (float)(pos - idx * r.src) * (1.0f / (float)r.src);
            u[2 * j] = swr_dot_lin(w0, h, h + LN_TAPS, wf);
            u[2 * j + 1] = swr_dot_lin(w1, h, h + LN_TAPS, wf);
        } else {
            u[2 * j] = ln_dot(w0, h);
            u[2 * j + 1] = ln_dot(w1, h);
        }
    }
}

// a downsampling rate's resampler (r.taps > 32 taps in rows of r.alloc): one thread per
// 192 kHz frame, both channels, the window x[base - center ..] read from memory (mirrored
// at the track's ends), the FMA3 kernel's 8 chains over the row
__global__ void __launch_bounds__(AMX_BLOCK) k_ln_upsample_wide(const uint32_t *__restrict__ x, int64_t n_in,
                                                                SwrDev r, int64_t j0, int64_t j1,
                                                                float *__restrict__ u,
                                                                const int32_t *__restrict__ gate) {
    if (AMX_LN_GATED(gate)) return;
    const int c = (r.taps - 1) / 2;
    for (int64_t j = j0 + (int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x; j < j1; j += (int64_t)gridDim.x * AMX_BLOCK) {
        const int64_t pos = j * r.dst, idx = pos / r.src;
        const int64_t base = idx / r.pc;
        const int ph = (int)(idx % r.pc);
        const float *h = r.bank + (int64_t)ph * r.alloc;
        float a0[8], a1[8];
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t v = x[ln_reflect(base - c + k, n_in)];
            a0[k] = __builtin_fmaf((float)lo16(v) * (1.0f / 32768.0f), h[k], 0.0f);
            a1[k] = __builtin_fmaf((float)hi16(v) * (1.0f / 32768.0f), h[k], 0.0f);
        }
        for (int q = 8; q < r.alloc; q += 8) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t v = x[ln_reflect(base - c + q + k, n_in)];
                a0[k] = __builtin_fmaf((float)lo16(v) * (1.0f / 32768.0f), h[q + k], a0[k]);
                a1[k] = __builtin_fmaf((float)hi16(v) * (1.0f / 32768.0f), h[q + k], a1[k]);
            }
        }
        const float b0 = a0[0] + a0[4], b1 = a0[1] + a0[5], b2 = a0[2] + a0[6], b3 = a0[3] + a0[7];
        const float e0 = a1[0] + a1[4], e1 = a1[1] + a1[5], e2 = a1[2] + a1[6], e3 = a1[3] + a1[7];
        u[2 * j] = (b0 + b2) + (b1 + b3);
        u[2 * j + 1] = (e0 + e2) + (e1 + e3);
    }
}

// ------------------------------------------------------------ block helpers
// The filter runs on one workgroup of LN_NT threads per track: every thread carries the
// (block-uniform) scalar state, the per-sample loops are shared out over the block.  One
// wave alone left every loop waiting on its own loads (HBM / L2 latency per 64 samples).
#define LN_NT 512
#define LN_NW (LN_NT / 64)

__device__ __forceinline__ double ln_wsum(double v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
    return v;
}

// block sum / max of one value per thread (s_red: LN_NW doubles); every thread gets it
__device__ __forceinline__ double ln_bsum(double v, double *s_red) {
    v = ln_wsum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
#pragma unroll
    for (int w = 0; w < LN_NW; w++) r += s_red[w];
    return r;
}
__device__ __forceinline__ double ln_bmax(double v, double *s_red) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = fmax(v, __shfl_xor(v, o));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = s_red[0];
#pragma unroll
    for (int w = 1; w < LN_NW; w++) r = fmax(r, s_red[w]);
    return r;
}

__device__ __forceinline__ int16_t ln_s16(double v) {            // av_clip_int16(llrint(v * 32768))
    const double r = rint(v * 32768.0);
    return (int16_t)(r > 32767.0 ? 32767 : (r < -32768.0 ? -32768 : (int)r));
}

// ln_s16 with the clamp as fmax / fmin (two fp64 operations instead of two compares and
// four selects; the same value for every non-NaN v)
__device__ __forceinline__ int16_t ln_s16_lim(double v) {
    return (int16_t)(int)fmin(fmax(rint(v * 32768.0), -32768.0), 32767.0);
}

__device__ __forceinline__ int ln_w(int i) { return i < LN_RSZ ? i : i - LN_RSZ; }
__device__ __forceinline__ int ln_wrap(int i) {
    while (i >= LN_RSZ) i -= LN_RSZ;
    return i;
}

struct LnShared {
    unsigned hist[1000];               // r128_in's gating-block histogram, rebuilt here
    double E[1000], B[1001];
    double th[2][LN_NT + 12];          // |x| of a scan group and the 12 positions after it
    double red[LN_NW];
    double oe[30];                     // r128_out: the last 30 frames' energies
    int first[LN_NW];
    double sbuf[1001];                 // ln_seq_sum
    int scan[LN_NW + 1];
};

__device__ __forceinline__ int ln_find_bin(const double *B, double e) {
    int lo = 0, hi = 1000;
    do {
        const int mid = (lo + hi) / 2;
        if (e >= B[mid]) lo = mid; else hi = mid;
    } while (hi - lo != 1);
    return lo;
}

// libebur128's sum over the bins j >= lo of hist[j] * E[j], in its sequential order
// (ebur128_gated_loudness's loop; k_decide's wave_seq_sum does the same): thread t owns
// bins [PER t, PER t + PER), the non-empty ones are compacted in bin order into sbuf
// (an empty bin adds 0.0, exactly) and thread 0 adds them one by one.  Every thread
// gets the sum.  sbuf: 1000 doubles; scan: NT / 64 + 1 ints.
template <int NT>
__device__ double ln_seq_sum(const unsigned *hist, const double *E, int lo, double *sbuf, int *scan) {
    constexpr int PER = (1000 + NT - 1) / NT;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    int mine = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int j = tid * PER + q;
        mine += (j < 1000 && j >= lo && hist[j] != 0u) ? 1 : 0;
    }
    int incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int up = __shfl_up(incl, o);
        if (lane >= o) incl += up;
    }
    __syncthreads();
    if (lane == 63) scan[w] = incl;
    __syncthreads();
    int off = incl - mine, tot = 0;
    for (int v = 0; v < NT / 64; v++) {
        off += v < w ? scan[v] : 0;
        tot += scan[v];
    }
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int j = tid * PER + q;
        if (j < 1000 && j >= lo && hist[j] != 0u) sbuf[off++] = (double)hist[j] * E[j];
    }
    __syncthreads();
    if (tid == 0) {
        double acc = 0.0;
        for (int k = 0; k < tot; k++) acc += sbuf[k];
        sbuf[1000] = acc;
    }
    __syncthreads();
    const double r = sbuf[1000];
    __syncthreads();
    return r;
}

// ebur128 gated loudness + relative threshold of the histogram (every thread)
__device__ void ln_global(LnShared &L, double &global, double &rel_thr) {
    const int tid = threadIdx.x;
    double c = 0.0;
    for (int j = tid; j < 1000; j += LN_NT) c += (double)L.hist[j];
    const double s = ln_seq_sum<LN_NT>(L.hist, L.E, 0, L.sbuf, L.scan);
    c = ln_bsum(c, L.red);
    if (c == 0.0) {
        global = -HUGE_VAL;
        rel_thr = -70.0;
        return;
    }
    double rel = s / c;
    rel *= 0.1;                                       // RELATIVE_GATE_FACTOR
    rel_thr = 10 * log10(rel) - 0.691;
    int start;
    if (rel < L.B[0]) start = 0;
    else {
        start = ln_find_bin(L.B, rel);
        if (rel > L.E[start]) ++start;
    }
    double a = 0.0;
    for (int j = start + tid; j < 1000; j += LN_NT) a += (double)L.hist[j];
    const double g = ln_seq_sum<LN_NT>(L.hist, L.E, start, L.sbuf, L.scan);
    a = ln_bsum(a, L.red);
    global = a == 0.0 ? -HUGE_VAL : 10 * log10(g / a) - 0.691;
}

// gating block ending at hop k (k >= 4): the mean square of hops k-4 .. k-1
__device__ __forceinline__ double ln_block_energy(const double *hops, int64_t k) {
    const double c0 = ((hops[2 * (k - 4)] + hops[2 * (k - 3)]) + hops[2 * (k - 2)]) + hops[2 * (k - 1)];
    const double c1 = ((hops[2 * (k - 4) + 1] + hops[2 * (k - 3) + 1]) + hops[2 * (k - 2) + 1]) + hops[2 * (k - 1) + 1];
    return (c0 + c1) / (double)(4 * LN_FR);
}
__device__ __forceinline__ void ln_add_block(LnShared &L, const double *hops, int64_t k) {
    const double en = ln_block_energy(hops, k);
    __syncthreads();
    if (threadIdx.x == 0 && en >= L.B[0]) L.hist[ln_find_bin(L.B, en)] += 1u;
    __syncthreads();
}

// 3 s short-term loudness ending at hop k (hops k-30 .. k-1)
__device__ __forceinline__ double ln_shortterm(const double *hops, int64_t k, double *s_red) {
    const int tid = threadIdx.x;
    double c0 = 0.0, c1 = 0.0;
    if (tid < 30 && k - 30 + tid >= 0) {
        c0 = hops[2 * (k - 30 + tid)];
        c1 = hops[2 * (k - 30 + tid) + 1];
    }
    const double e = (ln_bsum(c0, s_red) + ln_bsum(c1, s_red)) / (double)LN_FIRST;
    return 10 * log10(e) - 0.691;
}

// ------------------------------------------------------------ the filter
struct LnLim {                   // true_peak_limiter state (block-uniform)
    int state, env_cnt, env_index, peak_index, attack_length;
    double gr0, gr1, prev[2];
};

enum { LIM_OUT_, LIM_ATTACK_, LIM_SUSTAIN_, LIM_RELEASE_ };

// cycle counts of the kernel's parts (d_summary[2..]): where a track's time goes
struct LnProf {
    uint64_t fill = 0, detect = 0, env = 0, out = 0, stats = 0, feed = 0;
    uint64_t n_detect = 0, n_serial = 0;
};

// detect_peak from output offset `offset` over `count` positions: returns peak_delta
// (-1: none) and sets peak_value, peak_index, prev[].  Groups of LN_NT positions: each
// thread stages one position's |x| (and threads < 12 the positions after the group:
// the next sample and the 10-sample look-ahead read past a position; the ring always
// holds real samples there); the first position that is a candidate with the normal
// predecessor (the previous sample) is found by a block-wide minimum, and only from
// there on is the scan serial (a candidate that fails the look-ahead keeps the older
// predecessor, so later positions depend on it), every thread stepping it alike.
__device__ int ln_detect(const double *ring, LnLim &S, int lbi, int offset, int count, bool first,
                         double ceiling, double &peak_value, LnShared &L, LnProf &P) {
    P.n_detect++;
    const int tid = threadIdx.x;
    int index = lbi + (offset * 2) + (LN_ATT * 2);
    if (index >= LN_RSZ) index -= LN_RSZ;
    if (first) {
        S.prev[0] = fabs(ring[index - 2]);
        S.prev[1] = fabs(ring[index - 1]);
    }
    for (int base = 0; base < count; base += LN_NT) {
        {
            const int idx = ln_wrap(index + 2 * (base + tid));
            const double a0 = fabs(ring[idx]), a1 = fabs(ring[idx + 1]);
            double b0 = 0.0, b1 = 0.0;
            if (tid < 12) {
                const int jx = ln_wrap(index + 2 * (base + LN_NT + tid));
                b0 = fabs(ring[jx]);
                b1 = fabs(ring[jx + 1]);
            }
            __syncthreads();                          // the previous group's reads are done
            L.th[0][tid] = a0;
            L.th[1][tid] = a1;
            if (tid < 12) {
                L.th[0][LN_NT + tid] = b0;
                L.th[1][LN_NT + tid] = b1;
            }
            __syncthreads();
        }
        const int n = base + tid;
        const int last = (count - base < LN_NT ? count - base : LN_NT) - 1;
        bool cand = false;
        if (n < count) {
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const double th = L.th[c][tid], nx = L.th[c][tid + 1];
                const double pv = tid == 0 ? S.prev[c] : L.th[c][tid - 1];
                cand |= pv <= th && nx <= th && th > ceiling && n > 0;
            }
        }
        const unsigned long long m = __ballot(cand);
        if ((tid & 63) == 0) L.first[tid >> 6] = m ? (tid + __ffsll((long long)m) - 1) : LN_NT;
        __syncthreads();
        int L0 = LN_NT;
#pragma unroll
        for (int w = 0; w < LN_NW; w++) L0 = L.first[w] < L0 ? L.first[w] : L0;
        if (L0 == LN_NT) {
            S.prev[0] = L.th[0][last];
            S.prev[1] = L.th[1][last];
            continue;
        }
        P.n_serial++;
        if (L0 > 0) {
            S.prev[0] = L.th[0][L0 - 1];
            S.prev[1] = L.th[1][L0 - 1];
        }
        for (int k = L0; k <= last; k++) {
            const int nn = base + k;
            for (int c = 0; c < 2; c++) {
                const double t = L.th[c][k], nxt = L.th[c][k + 1];
                if ((S.prev[c] <= t) && (nxt <= t) && (t > ceiling) && (nn > 0)) {
                    bool detected = true;
                    for (int i = 2; i < 12; i++)
                        if (L.th[c][k + i] > t) { detected = false; break; }
                    if (!detected) continue;
                    const double p0 = L.th[0][k], p1 = L.th[1][k];
                    double mp = p0;
                    if (p1 > mp) mp = p1;
                    S.prev[0] = p0;
                    S.prev[1] = p1;
                    S.peak_index = ln_wrap(index + 2 * nn);
                    peak_value = mp;
                    return nn;
                }
                S.prev[c] = t;
            }
        }
    }
    return -1;
}

// apply env(i) to the k ring frames from env_index on (env_index may be the ring size
// itself, as in af_loudnorm: that first write falls outside the ring)
template <class F>
__device__ __forceinline__ void ln_env_apply(double *ring, int e0, int k, F env) {
    const int tid = threadIdx.x;
    constexpr int U = 4;
    for (int i0 = 0; i0 < k; i0 += LN_NT * U) {
        int sl[U];
        double r0[U], r1[U];
#pragma unroll
        for (int q = 0; q < U; q++) {
            const int i = i0 + LN_NT * q + tid;
            sl[q] = i > 0 ? ln_wrap(e0 + 2 * i) : e0;
            r0[q] = i < k ? ring[sl[q]] : 0.0;
            r1[q] = i < k ? ring[sl[q] + 1] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < U; q++) {
            const int i = i0 + LN_NT * q + tid;
            if (i < k) {
                const double g = env(i);
                ring[sl[q]] = r0[q] * g;
                ring[sl[q] + 1] = r1[q] * g;
            }
        }
    }
    __syncthreads();
}

__device__ __forceinline__ int ln_env_end(int e0, int k) {
    if (k <= 0) return e0;
    int e = e0 + 2 * (k - 1);
    if (k > 1) e = ln_wrap(e);
    e += 2;
    if (e >= LN_RSZ) e -= LN_RSZ;
    return e;
}

// true_peak_limiter: nb output frames from ring position lbi into y (s16)
__device__ void ln_limiter(double *ring, LnLim &S, int lbi, int nb, bool first, double ceiling,
                           int16_t *y, LnShared &L, LnProf &P) {
    const int tid = threadIdx.x;
    if (first) {
        double mx = 0.0;
        for (int i = tid; i < LN_ATT; i += LN_NT) mx = fmax(mx, fmax(fabs(ring[2 * i]), fabs(ring[2 * i + 1])));
        mx = ln_bmax(mx, L.red);
        if (mx > ceiling) {
            S.gr1 = ceiling / mx;
            S.state = LIM_SUSTAIN_;
            for (int i = tid; i < LN_ATT; i += LN_NT) {
                ring[2 * i] *= S.gr1;
                ring[2 * i + 1] *= S.gr1;
            }
            __syncthreads();
        }
    }
    int smp = 0;
    double pv = 0.0;
    do {
        switch (S.state) {
        case LIM_OUT_: {
            const uint64_t t0 = clock64();
            const int pd = ln_detect(ring, S, lbi, smp, nb - smp, first, ceiling, pv, L, P);
            P.detect += clock64() - t0;
            if (pd != -1) {
                S.env_cnt = 0;
                smp += (pd - S.attack_length);
                S.gr0 = 1.;
                S.gr1 = ceiling / pv;
                S.state = LIM_ATTACK_;
                S.env_index = S.peak_index - (S.attack_length * 2);
                if (S.env_index < 0) S.env_index += LN_RSZ;
                S.env_index += (S.env_cnt * 2);
                if (S.env_index > LN_RSZ) S.env_index -= LN_RSZ;
            } else {
                smp = nb;
            }
            break;
        }
        case LIM_ATTACK_: {
            int k = S.attack_length - S.env_cnt;
            if (k > nb - smp) k = nb - smp;
            if (k < 0) k = 0;
            const int c0 = S.env_cnt, al = S.attack_length;
            const double g0 = S.gr0, g1 = S.gr1;
            const uint64_t t0 = clock64();
            ln_env_apply(ring, S.env_index, k,
                         [&](int i) { return g0 - ((double)(c0 + i) / (al - 1) * (g0 - g1)); });
            P.env += clock64() - t0;
            S.env_index = ln_env_end(S.env_index, k);
            S.env_cnt += k;
            smp += k;
            if (smp < nb) {
                S.env_cnt = 0;
                S.attack_length = LN_ATT;
                S.state = LIM_SUSTAIN_;
            }
            break;
        }
        case LIM_SUSTAIN_: {
            const uint64_t t0 = clock64();
            const int pd = ln_detect(ring, S, lbi, smp, nb, first, ceiling, pv, L, P);
            P.detect += clock64() - t0;
            if (pd == -1) {
                S.state = LIM_RELEASE_;
                S.gr0 = S.gr1;
                S.gr1 = 1.;
                S.env_cnt = 0;
                break;
            }
            const double gain_reduction = ceiling / pv;
            if (gain_reduction < S.gr1) {
                S.state = LIM_ATTACK_;
                S.attack_length = pd;
                if (S.attack_length <= 1) S.attack_length = 2;
                S.gr0 = S.gr1;
                S.gr1 = gain_reduction;
                S.env_cnt = 0;
                break;
            }
            int k = pd;
            if (k > nb - smp) k = nb - smp;
            if (k < 0) k = 0;
            const double g1 = S.gr1;
            const uint64_t t1 = clock64();
            ln_env_apply(ring, S.env_index, k, [&](int) { return g1; });
            P.env += clock64() - t1;
            S.env_index = ln_env_end(S.env_index, k);
            S.env_cnt = k;
            smp += k;
            break;
        }
        default: {   // RELEASE
            const int rl = LN_FR;
            int k = rl - S.env_cnt;
            if (k > nb - smp) k = nb - smp;
            if (k < 0) k = 0;
            const int c0 = S.env_cnt;
            const double g0 = S.gr0, g1 = S.gr1;
            const uint64_t t0 = clock64();
            ln_env_apply(ring, S.env_index, k,
                         [&](int i) { return g0 + (((double)(c0 + i) / (rl - 1)) * (g1 - g0)); });
            P.env += clock64() - t0;
            S.env_index = ln_env_end(S.env_index, k);
            S.env_cnt += k;
            smp += k;
            if (smp < nb) {
                S.env_cnt = 0;
                S.state = LIM_OUT_;
            }
            break;
        }
        }
    } while (smp < nb);
    const uint64_t t_out = clock64();
    constexpr int U = 4;
    for (int i0 = 0; i0 < nb; i0 += LN_NT * U) {
        double r0[U], r1[U];
#pragma unroll
        for (int q = 0; q < U; q++) {
            const int i = i0 + LN_NT * q + tid;
            const int slot = ln_wrap(lbi + 2 * i);
            r0[q] = i < nb ? ring[slot] : 0.0;
            r1[q] = i < nb ? ring[slot + 1] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < U; q++) {
            const int i = i0 + LN_NT * q + tid;
            double o0 = r0[q], o1 = r1[q];
            if (fabs(o0) > ceiling) o0 = ceiling * (o0 < 0 ? -1 : 1);
            if (fabs(o1) > ceiling) o1 = ceiling * (o1 < 0 ? -1 : 1);
            if (i < nb) {
                y[2 * i] = ln_s16(o0);
                y[2 * i + 1] = ln_s16(o1);
            }
        }
    }
    P.out += clock64() - t_out;
}

// libebur128's K filter (direct form) over the frame's clamped output, threads 0 / 1 one
// channel each (r128_out, read only while above_threshold is 0): the frame's energy,
// both channels, to every thread; DBL_MIN flush at the end as ebur128_filter does per call
__device__ double ln_out_energy(const double *ring, int lbi, int nb, double ceiling, const double *kb,
                                const double *ka, double (&kv)[5], double *s_red) {
    const int tid = threadIdx.x;
    double e = 0.0;
    if (tid < 2) {
        double *v = kv;
        for (int i = 0; i < nb; i++) {
            const int slot = ln_wrap(lbi + 2 * i);
            double o = ring[slot + tid];
            if (fabs(o) > ceiling) o = ceiling * (o < 0 ? -1 : 1);
            v[0] = o - ka[1] * v[1] - ka[2] * v[2] - ka[3] * v[3] - ka[4] * v[4];
            const double yv = kb[0] * v[0] + kb[1] * v[1] + kb[2] * v[2] + kb[3] * v[3] + kb[4] * v[4];
            e += yv * yv;
            v[4] = v[3]; v[3] = v[2]; v[2] = v[1]; v[1] = v[0];
        }
        for (int k = 1; k < 5; k++) v[k] = fabs(v[k]) < 2.2250738585072014e-308 ? 0.0 : v[k];
    }
    __syncthreads();
    if (tid < 2) s_red[tid] = e;
    __syncthreads();
    const double r = s_red[0] + s_red[1];
    __syncthreads();
    return r;
}

// phase 0 (after k_lp_stats): the tracks the parallel form does not start -- the < 3 s
// linear fallback, a quiet start (handed over at the first segment start after
// above_threshold turns 1, lp_ctl[0] = 4); phase 1 (after k_lp_walk): a whole track the
// walker handed back (lp_ctl[0] = 2), frame by frame to the end
__global__ void __launch_bounds__(LN_NT) k_ln_dyn(LnArgs a0, int phase) {
    if (a0.lp_ctl && a0.lp_ctl[0] != (phase == 0 ? 1 : 2)) return;
    LnArgs a = a0;
    if (a0.lp_dctl) {
        a.offset = a0.lp_dctl[1];
        a.measured_i = a0.lp_dctl[2];
        a.measured_thresh = a0.lp_dctl[3];
    }
    __shared__ LnShared L;
    const int tid = threadIdx.x;
    for (int i = tid; i < 1000; i += LN_NT) { L.hist[i] = 0u; L.E[i] = a.energies[i]; }
    for (int i = tid; i < 1001; i += LN_NT) L.B[i] = a.bounds[i];
    if (tid < 30) L.oe[tid] = 0.0;
    __syncthreads();
    const int64_t n = a.n192;
    const float *u = a.u;
    double *ring = a.ring;
    const double ceiling = a.target_tp;
    LnProf P;
    if (n < LN_FIRST) {
        // the first frame is the whole input: af_loudnorm falls back to LINEAR_MODE with
        // an offset from r128_in's integrated loudness and sample peak
        for (int64_t k = 4; k * LN_FR <= n; k++) ln_add_block(L, a.hops, k);
        double global, rel;
        ln_global(L, global, rel);
        const double true_peak = a.peak[0] > a.peak[1] ? a.peak[0] : a.peak[1];
        const double offset = pow(10., (a.target_i - global) / 20.);
        const double offset_tp = true_peak * offset;
        const double off = offset_tp < a.target_tp ? offset : a.target_tp / true_peak;
        for (int64_t j = tid; j < n; j += LN_NT) {
            a.y[2 * j] = ln_s16((double)u[2 * j] * off);
            a.y[2 * j + 1] = ln_s16((double)u[2 * j + 1] * off);
        }
        if (tid == 0) {
            a.summary[0] = 1.0;
            a.summary[1] = off;
            for (int q = 10; q < 13; q++) a.summary[q] = 0.0;
            a.summary[13] = (a0.lp_ctl && a0.lp_ctl[0] == 2) ? 1.0 : 0.0;
        }
        return;
    }
    // ---- FIRST frame (3 s)
    for (int64_t k = 4; k <= LN_FIRST / LN_FR; k++) ln_add_block(L, a.hops, k);
    double delta[30];
    int index = 1, above;
    double prev_delta;
    {
        const double shortterm = ln_shortterm(a.hops, LN_FIRST / LN_FR, L.red);
        double env_shortterm;
        if (shortterm < a.measured_thresh) {
            above = 0;
            env_shortterm = shortterm <= -70. ? 0. : a.target_i - a.measured_i;
        } else {
            above = 1;
            env_shortterm = shortterm <= -70. ? 0. : a.target_i - shortterm;
        }
        const double d = pow(10., env_shortterm / 20.);
#pragma unroll
        for (int q = 0; q < 30; q++) delta[q] = d;
        prev_delta = delta[index];
    }
    for (int i = tid; i < LN_LIMF; i += LN_NT) {
        ring[2 * i] = (double)u[2 * i] * delta[1] * a.offset;
        ring[2 * i + 1] = (double)u[2 * i + 1] * delta[1] * a.offset;
    }
    __syncthreads();
    LnLim S{LIM_OUT_, 0, 0, 0, LN_ATT, 0.0, 0.0, {0.0, 0.0}};
    int lbi = 0;
    double kv[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    int oe_i = 0;
    auto out_feed = [&](int nb) {                        // r128_out, only while needed
        const uint64_t t0 = clock64();
        const double e = ln_out_energy(ring, lbi, nb, ceiling, a.kb, a.ka, kv, L.red);
        if (tid == 0) L.oe[oe_i] = e;
        oe_i = oe_i + 1 < 30 ? oe_i + 1 : 0;
        __syncthreads();
        P.feed += clock64() - t0;
    };
    int64_t out_pos = 0;
    ln_limiter(ring, S, lbi, LN_FR, true, ceiling, a.y, L, P);
    if (above == 0) out_feed(LN_FR);
    out_pos = LN_FR;
    int64_t R = LN_LIMF, Pin = LN_FIRST;
    auto gauss = [&](int idx) {
        double r = 0.;
        idx = idx - 10 > 0 ? idx - 10 : idx + 20;
#pragma unroll
        for (int i = 0; i < 21; i++) r += delta[((idx + i) < 30) ? (idx + i) : (idx + i - 30)] * a.weights[i];
        return r;
    };
    int ho_f = -1, ho_k = -1;                            // hand-over frame / segment (quiet start)
    // ---- INNER frames (100 ms)
    while (Pin < n) {
        const int t_in = (int)((Pin - LN_FIRST) / LN_FR);     // this INNER frame
        if (phase == 0 && t_in >= a0.lp_tstop) return;        // (a shard: past rank 0's frames)
        const int nb = (int)(n - Pin < LN_FR ? n - Pin : LN_FR);
        const uint64_t t_fill = clock64();
        const double gain = gauss(index + 10 < 30 ? index + 10 : index + 10 - 30);
        const double gain_next = gauss(index + 11 < 30 ? index + 11 : index + 11 - 30);
        {
            constexpr int U = 4;
            for (int i0 = 0; i0 < nb; i0 += LN_NT * U) {
                float v0[U], v1[U];
#pragma unroll
                for (int q = 0; q < U; q++) {
                    const int i = i0 + LN_NT * q + tid;
                    v0[q] = i < nb ? u[2 * (R + i)] : 0.0f;
                    v1[q] = i < nb ? u[2 * (R + i) + 1] : 0.0f;
                }
#pragma unroll
                for (int q = 0; q < U; q++) {
                    const int i = i0 + LN_NT * q + tid;
                    if (i < nb) {
                        const int slot = ln_wrap(lbi + 2 * i);
                        const double g = gain + (((double)i / nb) * (gain_next - gain));
                        ring[slot] = (double)v0[q] * g * a.offset;
                        ring[slot + 1] = (double)v1[q] * g * a.offset;
                    }
                }
            }
        }
        __syncthreads();
        lbi = ln_wrap(lbi + 2 * nb);
        {
            const int sub = (LN_FR - nb) * 2;
            lbi = lbi + sub < LN_RSZ ? lbi + sub : lbi + sub - LN_RSZ;
        }
        R += nb;
        Pin += nb;
        P.fill += clock64() - t_fill;
        ln_limiter(ring, S, lbi, nb, false, ceiling, a.y + 2 * out_pos, L, P);
        if (above == 0) out_feed(nb);
        const uint64_t t_stats = clock64();
        out_pos += nb;
        // r128_in after this frame: a full frame ends on hop Pin / 19200 (one new block)
        const int64_t hk = Pin / LN_FR;
        if (nb == LN_FR) ln_add_block(L, a.hops, hk);
        double global, relative_threshold;
        ln_global(L, global, relative_threshold);
        const double shortterm = ln_shortterm(a.hops, hk, L.red);
        if (above == 0) {
            if (shortterm > a.measured_thresh) prev_delta *= 1.0058;
            double so = 0.0;
            for (int q = 0; q < 30; q++) so += L.oe[q];
            const double shortterm_out = 10 * log10(so / (double)LN_FIRST) - 0.691;
            if (shortterm_out >= a.target_i) above = 1;
        }
        double dnew;
        if (shortterm < relative_threshold || shortterm <= -70. || above == 0) {
            dnew = prev_delta;
        } else {
            const double env_global = fabs(shortterm - global) < (a.target_lra / 2.)
                                          ? shortterm - global
                                          : (a.target_lra / 2.) * ((shortterm - global) < 0 ? -1 : 1);
            const double env_shortterm = a.target_i - shortterm;
            dnew = pow(10., (env_global + env_shortterm) / 20.);
        }
#pragma unroll
        for (int q = 0; q < 30; q++) delta[q] = q == index ? dnew : delta[q];
        prev_delta = dnew;
        index = index + 1 < 30 ? index + 1 : 0;
        P.stats += clock64() - t_stats;
        if (a0.lp_D && tid == 0) a0.lp_D[t_in] = dnew;
        if (phase == 0 && a0.lp_recG && above && ho_f < 0) {
            // from here the deltas follow r128_in alone: hand over at the next segment
            // start (frame 1 + k Fs, k <= J) -- after frame ho_f - 1, before ho_f's fill
            const int phi = t_in + 1;
            int k = (phi + a0.lp_Fs - 1) / a0.lp_Fs;
            if (k < 1) k = 1;
            if (k <= a0.lp_J) {
                ho_k = k;
                ho_f = 1 + k * a0.lp_Fs;
            } else {
                ho_f = 0;                                      // none left: run to the end
            }
        }
        if (ho_f > 0 && t_in + 1 == ho_f - 1) {
            // the state at frame ho_f's start, as k_lp_snapshot records it: the limiter
            // scalars (envelope slot in frames) and the 2048 ring slots from the frame's
            // first output position (19200 ho_f; INNER slot = position mod the ring)
            double *rec = a0.lp_recG + (int64_t)ho_k * AMX_LN_REC;
            if (tid == 0) {
                rec[0] = S.state;
                rec[1] = S.env_cnt;
                rec[2] = S.env_index / 2;
                rec[3] = S.attack_length;
                rec[4] = S.gr0;
                rec[5] = S.gr1;
                rec[6] = ho_f;
                rec[7] = 0.0;
                a0.lp_ctl[0] = 4;
                a0.lp_ctl[4] = ho_k;
                a0.lp_ctl[5] = ho_f;
            }
            const int s0 = (int)(((int64_t)LN_FR * ho_f) % LN_LIMF);
            for (int j = tid; j < AMX_LN_WIN; j += LN_NT) {
                const int sl = s0 + j < LN_LIMF ? s0 + j : s0 + j - LN_LIMF;
                rec[16 + 2 * j] = ring[2 * sl];
                rec[17 + 2 * j] = ring[2 * sl + 1];
            }
            return;
        }
    }
    // ---- FINAL frame (flush_frame: the last 3 s less one frame, re-read)
    {
        const int nbf = LN_FIRST - LN_FR;                // (buf_size - prev_nb) - (100 ms - prev_nb)
        const int64_t S0 = n - nbf;                      // its first frame in the stream
        const double gain = gauss(index + 10 < 30 ? index + 10 : index + 10 - 30);
        for (int i = tid; i < LN_LIMF; i += LN_NT) {
            ring[2 * i] = (double)u[2 * (S0 + i)] * gain * a.offset;
            ring[2 * i + 1] = (double)u[2 * (S0 + i) + 1] * gain * a.offset;
        }
        __syncthreads();
        lbi = 0;
        int64_t src = LN_LIMF;
        for (int it = 0; it < nbf / LN_FR; it++) {
            ln_limiter(ring, S, lbi, LN_FR, false, ceiling, a.y + 2 * out_pos, L, P);
            for (int i = tid; i < LN_FR; i += LN_NT) {
                const int slot = ln_wrap(lbi + 2 * i);
                const bool in = src + i < nbf;
                ring[slot] = in ? (double)u[2 * (S0 + src + i)] * gain * a.offset : 0.;
                ring[slot + 1] = in ? (double)u[2 * (S0 + src + i) + 1] * gain * a.offset : 0.;
            }
            __syncthreads();
            src += LN_FR;
            lbi = ln_wrap(lbi + 2 * LN_FR);
            out_pos += LN_FR;
        }
    }
    if (tid == 0) {
        a.summary[0] = 0.0;
        a.summary[1] = (double)above;
        a.summary[2] = (double)P.fill;
        a.summary[3] = (double)P.detect;
        a.summary[4] = (double)P.env;
        a.summary[5] = (double)P.out;
        a.summary[6] = (double)P.stats;
        a.summary[7] = (double)P.feed;
        a.summary[8] = (double)P.n_detect;
        a.summary[9] = (double)P.n_serial;
        for (int q = 10; q < 13; q++) a.summary[q] = 0.0;
        a.summary[13] = (a0.lp_ctl && a0.lp_ctl[0] == 2) ? 1.0 : 0.0;   // handed over by k_lp_walk
    }
}

// ======================================================================
// Dynamic mode in parallel form.  k_ln_dyn above runs af_loudnorm
// frame by frame on one workgroup; it stays the path for the < 3 s linear fallback
// and for a track whose first 3 s are below measured_thresh (above_threshold 0: the
// output's own short-term loudness then steers the gains).  Every other track -- the
// reference's pass 1 always, pass 2 unless the track starts quietly -- runs here:
//  1. With above_threshold 1 the AGC value an INNER frame t writes depends only on
//     r128_in after that frame (3 s short-term, gated integrated loudness, relative
//     gate), i.e. on pass 1's hop energies of this 192 kHz stream: k_lp_stats forms
//     every frame's value at once, k_lp_dscan the deltas (a held frame keeps the
//     previous delta: a last-valid scan), k_lp_gains the Gaussian gain of every frame
//     (frame t's fill uses the deltas of frames t-30 .. t-10).
//  2. The limiter ring then holds a known stream: every fill is u * gain ramp * offset.
//     A wave keeps only the slots the limiter has multiplied (one flag bit per slot in
//     LDS, the values in a per-wave ring in HBM); an unflagged slot's value is formed
//     from u when read.  The ring is literal -- slot indices, wrap reads and FINAL's
//     re-basing are af_loudnorm's own -- so a frame with the limiter idle costs a
//     64-wide peak scan and the output pass.
//  3. The limiter forgets: two runs that differ at some frame agree again after a
//     release completes or a new deepest reduction is attacked.  k_lp_seg runs every
//     segment of Fs frames at once, each from rest Wf frames early, and records its
//     guessed start state and its end state (the scalars and the 2048 ring slots from
//     the frame start: every slot multiplied and not yet output lies there; a record
//     with a flag outside is marked and never matches); the second of two neighbours
//     to finish compares them.  k_lp_walk walks the boundaries in order and re-runs,
//     with output, any segment whose start guess was wrong, from the true state.
// Every output sample is the reference's operation sequence applied from the true
// state, so the result equals k_ln_dyn's given the same gains.
#define LP_FR LN_FR
#define LP_FIRST LN_FIRST
#define LP_RS AMX_LN_RING
#define LP_ATT LN_ATT
#define LP_FW (LP_RS / 32)       // flag words per ring
#define LP_NFIN 29               // FINAL's 100 ms sub-frames: (576000 - 19200) / 19200
#define LP_REC AMX_LN_REC
#define LP_WIN AMX_LN_WIN
#define LP_STAT_NT 256
#define LP_STAT_F 4              // INNER frames per k_lp_stats workgroup (16: 135 us per run at C3)
#define LP_DIRTY 7               // record slot: 1 = a flagged slot lies outside the window

enum { LO_OUT = 0, LO_ATTACK, LO_SUSTAIN, LO_RELEASE };

__device__ __forceinline__ double lp_bsum(double v, double *red) {
    v = ln_wsum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = 0.0;
#pragma unroll
    for (int w = 0; w < LP_STAT_NT / 64; w++) r += red[w];
    return r;
}

// 3 s short-term loudness ending at hop k (hops k-30 .. k-1), every thread
__device__ __forceinline__ double lp_shortterm(const double *hops, int64_t k, double *red) {
    double c0 = 0.0, c1 = 0.0;
    if (threadIdx.x < 30 && k - 30 + (int)threadIdx.x >= 0) {
        c0 = hops[2 * (k - 30 + threadIdx.x)];
        c1 = hops[2 * (k - 30 + threadIdx.x) + 1];
    }
    return 10 * log10((lp_bsum(c0, red) + lp_bsum(c1, red)) / (double)LP_FIRST) - 0.691;
}

// frame statistics: block 0 the FIRST frame and the resolved options; block b > 0
// the INNER frames [16 (b - 1), 16 b): the histogram of the blocks before them, then
// frame by frame its block, the gated loudness, the short-term loudness, the value
__global__ void __launch_bounds__(LP_STAT_NT) k_lp_stats(LpArgs a) {
    __shared__ unsigned hist[1000];
    __shared__ double E[1000], B[1001], red[LP_STAT_NT / 64], sbuf[1001];
    __shared__ int scan[LP_STAT_NT / 64 + 1];
    const int tid = threadIdx.x;
    const double mi = a.measured_src ? a.measured_src[4] : a.measured_i;
    const double mt = a.measured_src ? a.measured_src[7] : a.measured_thresh;
    if (AMX_LN_GATED(a.gate)) {        // the track is not in dynamic mode: nothing runs
        if (blockIdx.x == 0 && tid == 0) a.ctl[0] = 3;
        return;
    }
    if (blockIdx.x == 0) {
        const bool full = a.n >= LP_FIRST;
        const double st = full ? lp_shortterm(a.hops, LP_FIRST / LP_FR, red) : 0.0;
        if (tid == 0) {
            const bool above = !(st < mt);
            const double env = st <= -70. ? 0. : a.target_i - (above ? st : mi);
            a.ctl[0] = (full && above) ? 0 : 1;
            a.ctl[1] = 0;
            a.ctl[2] = 0;
            a.ctl[3] = above ? 1 : 0;
            a.dctl[0] = pow(10., env / 20.);
            const double off_db = a.offset_src ? round2(a.target_i - a.offset_src[0]) : 20. * log10(a.offset);
            a.dctl[1] = a.offset_src ? pow(10., off_db / 20.) : a.offset;
            a.dctl[4] = off_db;
            a.dctl[2] = mi;
            a.dctl[3] = mt;
        }
        return;
    }
    const int t0 = (blockIdx.x - 1) * LP_STAT_F;
    if (a.n < LP_FIRST || t0 >= a.T) return;
    for (int i = tid; i < 1000; i += LP_STAT_NT) { hist[i] = 0u; E[i] = a.energies[i]; }
    for (int i = tid; i < 1001; i += LP_STAT_NT) B[i] = a.bounds[i];
    __syncthreads();
    // gating blocks ending at hops 4 .. 30 + t0 (the FIRST frame's and every full INNER
    // frame's before t0)
    for (int64_t k = 4 + tid; k <= 30 + t0; k += LP_STAT_NT) {
        const double en = ln_block_energy(a.hops, k);
        if (en >= B[0]) atomicAdd(&hist[ln_find_bin(B, en)], 1u);
    }
    __syncthreads();
    for (int j = 0; j < LP_STAT_F && t0 + j < a.T; j++) {
        const int t = t0 + j;
        const bool full = t < a.T - 1 || a.nb_last == LP_FR;
        const int64_t kt = full ? 31 + t : 30 + t;        // r128_in's hops after this frame
        if (full && tid == 0) {
            const double en = ln_block_energy(a.hops, kt);
            if (en >= B[0]) hist[ln_find_bin(B, en)] += 1u;
        }
        __syncthreads();
        // ebur128 gated loudness and relative threshold (ln_global's arithmetic: the energy
        // sums in libebur128's sequential bin order, ln_seq_sum)
        double c = 0.0;
        for (int q = tid; q < 1000; q += LP_STAT_NT) c += (double)hist[q];
        const double s = ln_seq_sum<LP_STAT_NT>(hist, E, 0, sbuf, scan);
        c = lp_bsum(c, red);
        double global = -HUGE_VAL, rel_thr = -70.0;
        if (c != 0.0) {
            double rel = s / c;
            rel *= 0.1;
            rel_thr = 10 * log10(rel) - 0.691;
            int start;
            if (rel < B[0]) start = 0;
            else {
                start = ln_find_bin(B, rel);
                if (rel > E[start]) ++start;
            }
            double ab = 0.0;
            for (int q = start + tid; q < 1000; q += LP_STAT_NT) ab += (double)hist[q];
            const double g = ln_seq_sum<LP_STAT_NT>(hist, E, start, sbuf, scan);
            ab = lp_bsum(ab, red);
            global = ab == 0.0 ? -HUGE_VAL : 10 * log10(g / ab) - 0.691;
        }
        const double st = lp_shortterm(a.hops, kt, red);
        if (tid == 0) {
            const bool hold = st < rel_thr || st <= -70.;
            a.hold[t] = hold ? 1 : 0;
            double v = 0.0;
            if (!hold) {
                const double env_global = fabs(st - global) < (a.target_lra / 2.)
                                              ? st - global
                                              : (a.target_lra / 2.) * ((st - global) < 0 ? -1 : 1);
                const double env_shortterm = a.target_i - st;
                v = pow(10., (env_global + env_shortterm) / 20.);
            }
            a.v[t] = v;
        }
    }
}

// the delta each INNER frame writes: its value, or (held) the previous frame's; the
// FIRST frame's d0 before any value.  One workgroup: last-valid index scan.
__global__ void __launch_bounds__(1024) k_lp_dscan(LpArgs a) {
    if (a.ctl[0] != 0 && a.ctl[0] != 4) return;
    __shared__ int s[1024];
    const int tid = threadIdx.x, T = a.T;
    // a quiet start: k_ln_dyn wrote the deltas of the INNER frames before the hand-over
    // frame; they stand (a fixed value each)
    const int t0 = a.ctl[0] == 4 ? a.ctl[5] - 1 : 0;
    const int per = (T + 1023) / 1024, lo = tid * per, hi = min(T, lo + per);
    int last = -1;
    for (int t = lo; t < hi; t++)
        if (t < t0 || !a.hold[t]) last = t;
    s[tid] = last;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int v = tid >= o ? s[tid - o] : -1;
        __syncthreads();
        s[tid] = max(s[tid], v);
        __syncthreads();
    }
    int cur = tid > 0 ? s[tid - 1] : -1;
    const double d0 = a.dctl[0];
    for (int t = lo; t < hi; t++) {
        if (t < t0) {
            cur = t;
            continue;
        }
        if (!a.hold[t]) cur = t;
        a.D[t] = cur < 0 ? d0 : (cur < t0 ? a.D[cur] : a.v[cur]);
    }
}

// G[t] = gaussian_filter at INNER frame t (t = T: the FINAL frame's gain): the 21
// weights over the deltas of frames t-30 .. t-10 (the FIRST frame's d0 before 0),
// summed in af_loudnorm's order; and the fill ramp i / 19200
__global__ void __launch_bounds__(256) k_lp_gains(LpArgs a) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (int64_t i = g; i < LP_FR; i += (int64_t)gridDim.x * 256) a.ramp[i] = (double)i / (double)LP_FR;
    if ((a.ctl[0] != 0 && a.ctl[0] != 4) || g > a.T) return;
    const int t = (int)g;
    const double d0 = a.dctl[0];
    double r = 0.;
#pragma unroll
    for (int i = 0; i < 21; i++) {
        const int f = t + i - 30;
        r += (f >= 0 ? a.D[f] : d0) * a.weights[i];
    }
    a.G[t] = r;
}

// ------------------------------------------------------------ one wave's limiter
// Frame phi: 0 = FIRST, 1 .. T = INNER frame phi - 1, T + 1 .. T + 29 = FINAL's
// 100 ms calls.  Positions are 192 kHz frame indices of the output stream.
struct LpFrame {
    int phi, nb, lbi, sF, fin;
    int64_t base, F;       // first output position; the fill frontier (positions < F)
};

__device__ __forceinline__ int lp_mod(int64_t v) { return (int)(v % LP_RS); }

__device__ __forceinline__ LpFrame lp_frame(const LpArgs &a, int phi) {
    LpFrame f;
    f.phi = phi;
    if (phi == 0) {
        f.base = 0;
        f.nb = LP_FR;
        f.F = LP_RS;
        f.fin = 0;
    } else if (phi <= a.T) {
        const int t = phi - 1;
        f.base = (int64_t)LP_FR * phi;
        f.nb = t < a.T - 1 ? LP_FR : a.nb_last;
        f.F = LP_RS + (int64_t)LP_FR * t + f.nb;
        f.fin = 0;
    } else {
        const int i = phi - a.T - 1;
        f.base = a.S0 + (int64_t)LP_FR * i;
        f.nb = LP_FR;
        f.F = a.S0 + LP_RS + (int64_t)LP_FR * i;
        f.fin = 1;
    }
    const int64_t o = f.fin ? a.S0 : 0;     // FINAL re-bases the ring at S0
    f.lbi = lp_mod(f.base - o);
    f.sF = lp_mod(f.F - o);
    return f;
}

// the segment starts: 0, 1 + k Fs (INNER, never the partial last frame), S0's frame
// T + 1 and every Fs FINAL frames after it
__device__ __forceinline__ int lp_seg_start(const LpArgs &a, int k) {
    if (k == 0) return 0;
    if (k <= a.J) return 1 + k * a.Fs;
    return a.T + 1 + (k - a.J - 1) * a.Fs;
}

// The limiter of one segment runs on a workgroup of LP_NT lanes (LP_NW waves): its
// slot loops (fills, envelopes, output) and its peak scans are LP_NT wide, so a release's
// 19 200 slots or a frame's scan take 1 / LP_NW of one wave's dependent memory round
// trips; the scalar state is workgroup-uniform (every lane holds it).
#ifndef AMX_LP_NT
#define AMX_LP_NT 256
#endif
#define LP_NT AMX_LP_NT
#define LP_NW (LP_NT / 64)
#define LP_STW (LP_NT + 16)      // one channel's scan row: a group and its 12-position look-ahead

struct LpWave {
    double2 *ring;         // [LP_RS] the multiplied slots' values (HBM)
    unsigned *flags;       // [LP_FW] LDS: slot multiplied since its last fill
    double *st;            // [2][LP_STW] LDS: |x| of a peak-scan group
    double *gl;            // [8] LDS: G[tb .. tb + 7] (clamped to T), the gain rows the frame's slots use
    unsigned long long *sv;   // [LP_NW] LDS: the waves' votes
    int tb;
    double gT;             // G[T] (FINAL's gain)
    LpFrame f;
    int mode, env_cnt, env_index, attack_length;
    double gr0, gr1;
    double d0, off;
};

// a barrier only a multi-wave workgroup needs (one wave's lanes run in lock step)
__device__ __forceinline__ void lp_wg_barrier() {
#if LP_NW > 1
    __syncthreads();
#endif
}

// the workgroup barrier after ring stores another wave reads next: every wave's stores
// have completed (vmcnt) before it arrives
__device__ __forceinline__ void lp_sync_ring() {
#if LP_NW > 1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    __syncthreads();
}

// workgroup votes (uniform control flow only): the waves' ballots through LDS
__device__ __forceinline__ void lp_vote(const LpWave &W, bool p, unsigned long long (&m)[LP_NW]) {
    const unsigned long long b = __ballot(p);
#if LP_NW == 1
    m[0] = b;
#else
    __syncthreads();                       // the previous vote's readers are done
    if ((threadIdx.x & 63) == 0) W.sv[threadIdx.x >> 6] = b;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < LP_NW; w++) m[w] = W.sv[w];
#endif
}
// the first set bit at index >= from of an LP_NT-bit vote, or -1
__device__ __forceinline__ int lp_next(const unsigned long long (&m)[LP_NW], int from) {
#pragma unroll
    for (int w = 0; w < LP_NW; w++) {
        if (from >= 64 * (w + 1)) continue;
        const int sh = from > 64 * w ? from - 64 * w : 0;
        const unsigned long long x = m[w] >> sh;
        if (x) return 64 * w + sh + __ffsll((long long)x) - 1;
    }
    return -1;
}
// the first lane whose p holds, or -1
__device__ __forceinline__ int lp_first(const LpWave &W, bool p) {
    unsigned long long m[LP_NW];
    lp_vote(W, p, m);
    return lp_next(m, 0);
}
// workgroup max / sum (the waves' reductions through the vote scratch)
__device__ __forceinline__ double lp_wg_max(const LpWave &W, double v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = fmax(v, __shfl_xor(v, o));
#if LP_NW > 1
    __syncthreads();
    if ((threadIdx.x & 63) == 0) W.sv[threadIdx.x >> 6] = (unsigned long long)__double_as_longlong(v);
    __syncthreads();
#pragma unroll
    for (int w = 0; w < LP_NW; w++) v = fmax(v, __longlong_as_double((long long)W.sv[w]));
#endif
    return v;
}
__device__ __forceinline__ int lp_wg_sum(const LpWave &W, int v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
#if LP_NW > 1
    __syncthreads();
    if ((threadIdx.x & 63) == 0) W.sv[threadIdx.x >> 6] = (unsigned long long)(unsigned)v;
    __syncthreads();
    v = 0;
#pragma unroll
    for (int w = 0; w < LP_NW; w++) v += (int)(unsigned)W.sv[w];
#endif
    return v;
}

// the position a slot holds: the latest filled one with that slot
__device__ __forceinline__ int64_t lp_pos(const LpFrame &f, int s) {
    int d = s - f.sF;
    if (d < 0) d += LP_RS;
    return f.F - LP_RS + d;
}

__device__ __forceinline__ bool lp_flag(const LpWave &W, int s) { return (W.flags[s >> 5] >> (s & 31)) & 1u; }

// the value a slot holds: the multiplied value if flagged, else its position's fill
// (af_loudnorm filter_frame: FIRST u d0 offset, INNER u (gain ramp) offset, FINAL
// u G_T offset, 0 past the track).  No control flow around the loads (a load inside a
// divergent branch made the compiler wait for every outstanding load at the join, which
// undid the scans' loads ahead): every operand is loaded -- an unflagged slot's ring
// value from slot 0 (one line for the whole wave), the gain rows clamped in range -- and
// the value selected
__device__ __forceinline__ double2 lp_val(const LpArgs &a, const LpWave &W, int s) {
    const bool fl = lp_flag(W, s);
    const double2 rv = W.ring[fl ? s : 0];
    const int64_t pos = lp_pos(W.f, s);
    const bool fin = W.f.fin != 0;
    const bool past = fin && pos >= a.n;
    // (a past position reads the track's last one, unused: inside every window that
    // holds FINAL, amx_ln_shard.windowed)
    const float2 x = reinterpret_cast<const float2 *>(a.u)[past ? a.n - 1 : pos];
    const int64_t q = pos - LP_RS > 0 ? pos - LP_RS : 0;
    int t, i;
    if (a.n < ((int64_t)1 << 31)) {             // wave-uniform: 32-bit quotient (tracks < 3.1 h)
        const uint32_t q32 = (uint32_t)q;
        t = (int)(q32 / (uint32_t)LP_FR);
        i = (int)(q32 - (uint32_t)t * (uint32_t)LP_FR);
    } else {
        t = (int)(q / LP_FR);
        i = (int)(q - (int64_t)t * LP_FR);
    }
    const int tc = t < a.T - 1 ? t : a.T - 1;
    // the gain rows from the frame's LDS copy (a slot of frame f holds a position of one of
    // the <= 4 INNER frames from tb, lp_gload): LDS reads instead of 3 vector loads
    int k = tc - W.tb;
    k = k < 0 ? 0 : (k > 6 ? 6 : k);
    const double r0 = a.ramp[i], g0 = W.gl[k], g1 = W.gl[k + 1], gT = W.gT;
    double r = r0;
    if (!(t < a.T - 1 || a.nb_last == LP_FR)) r = (double)i / (double)a.nb_last;
    const double gi = g0 + (r * (g1 - g0));
    const double g = fin ? gT : (pos < LP_RS ? W.d0 : gi);
    double2 v = make_double2(((double)x.x * g) * W.off, ((double)x.y * g) * W.off);
    if (past) v = make_double2(0.0, 0.0);
    return fl ? rv : v;
}

// the frame's gain rows into LDS: positions [F - LP_RS, F) fall in INNER frames
// t = (pos - LP_RS) / LP_FR >= tb; the caller synchronises before lp_val reads them
__device__ __forceinline__ void lp_gload(const LpArgs &a, LpWave &W) {
    const int64_t q = W.f.F - 2 * (int64_t)LP_RS;
    W.tb = q > 0 ? (int)(q / LP_FR) : 0;
    if (threadIdx.x < 8) {
        const int t = W.tb + (int)threadIdx.x;
        W.gl[threadIdx.x] = a.G[t < a.T ? t : a.T];
    }
}

__device__ __forceinline__ void lp_clear_range(LpWave &W, int lo, int hi) {   // slots [lo, hi)
    if (hi <= lo) return;
    for (int w = (lo >> 5) + (int)threadIdx.x; w <= ((hi - 1) >> 5); w += LP_NT) {
        const int b0 = w * 32;
        const int x0 = max(lo, b0) - b0, x1 = min(hi, b0 + 32) - b0;
        const unsigned m = (x1 - x0 == 32) ? 0xffffffffu : (((1u << (x1 - x0)) - 1u) << x0);
        W.flags[w] &= ~m;
    }
}

// the fill at the start of frame phi: the slots it refills lose their flags
__device__ __forceinline__ void lp_refill(const LpArgs &a, LpWave &W, int phi) {
    // every wave is done with the previous frame's flags and gain rows (its output pass
    // reads them) before they are rewritten
    lp_wg_barrier();
    int s0 = 0, cnt = LP_RS;
    if (phi != 0 && phi != a.T + 1) {
        if (phi <= a.T) {
            const int t = phi - 1;
            s0 = lp_mod((int64_t)LP_FR * t);
            cnt = t < a.T - 1 ? LP_FR : a.nb_last;
        } else {
            s0 = lp_mod((int64_t)LP_FR * (phi - a.T - 2));
            cnt = LP_FR;
        }
    }
    if (cnt >= LP_RS) {
        for (int w = threadIdx.x; w < LP_FW; w += LP_NT) W.flags[w] = 0u;
    } else {
        lp_clear_range(W, s0, min(s0 + cnt, LP_RS));
        if (s0 + cnt > LP_RS) lp_clear_range(W, 0, s0 + cnt - LP_RS);
    }
    lp_gload(a, W);
    __syncthreads();
}

// multiply k slots from e0 by env(i) (af_loudnorm's envelope loops).  The k slots are
// distinct, so the values of 4 groups of LP_NT are loaded before any of them is written
// (one memory round trip per 4 LP_NT slots), and no pass reads a slot another pass
// writes: the ring is synchronised once, after the last pass (AMX_LP_ENV_SYNC1; a sync
// per pass drained every pass's stores before the next one's loads -- a release's 19 200
// slots paid 19 store drains and barriers)
#ifndef AMX_LP_ENV_SYNC1
#define AMX_LP_ENV_SYNC1 1
#endif
#ifndef AMX_LP_EG
#define AMX_LP_EG 4              // groups of LP_NT slots per envelope pass (one memory round trip)
#endif
template <class F>
__device__ __forceinline__ void lp_env(const LpArgs &a, LpWave &W, int e0, int k, F env) {
    for (int i00 = 0; i00 < k; i00 += AMX_LP_EG * LP_NT) {
        double2 v[AMX_LP_EG];
        int s[AMX_LP_EG];
#pragma unroll
        for (int p = 0; p < AMX_LP_EG; p++) {
            const int i = i00 + LP_NT * p + (int)threadIdx.x;
            int ss = e0 + i;
            if (ss >= LP_RS) ss -= LP_RS;
            s[p] = ss;
            v[p] = lp_val(a, W, ss);                       // (i >= k: read, unused)
        }
#pragma unroll
        for (int p = 0; p < AMX_LP_EG; p++) {
            const int i = i00 + LP_NT * p + (int)threadIdx.x;
            if (i < k) {
                const double g = env(i);
                v[p].x = v[p].x * g;
                v[p].y = v[p].y * g;
                W.ring[s[p]] = v[p];
                atomicOr(&W.flags[s[p] >> 5], 1u << (s[p] & 31));
            }
        }
#if !AMX_LP_ENV_SYNC1
        lp_sync_ring();
#endif
    }
#if AMX_LP_ENV_SYNC1
    if (k > 0) lp_sync_ring();
#endif
}

__device__ __forceinline__ int lp_env_end(int e0, int k) {
    int e = e0 + (k > 0 ? k : 0);
    return e >= LP_RS ? e - LP_RS : e;
}

#ifndef AMX_LP_PD
#define AMX_LP_PD 4              // (measurement builds: scripts/build_var.py)
#endif
#define LP_PD AMX_LP_PD          // lp_detect: groups of LP_NT positions loaded together
// one group's values: LP_NT positions from slot s0
__device__ __forceinline__ double2 lp_grp(const LpArgs &a, const LpWave &W, int s0, int lane) {
    int s = s0 + lane;
    while (s >= LP_RS) s -= LP_RS;
    return lp_val(a, W, s);
}
// detect_peak from offset smp over count positions: peak_delta or -1; the peak's |x|
// and slot.  LP_NT positions per step: the first one that is a candidate with its
// previous sample as predecessor is found by a vote; only from there on is the scan
// serial (a candidate that fails the 10-sample look-ahead keeps the older predecessor).
// A candidate needs |x| > ceiling.  Outside FINAL, a slot's value is its position's
// fill (a function of the position alone, k_lp_fill) or that fill multiplied by the
// limiter's envelope gains, which are <= 1 (attack / release ramps between a gain
// reduction and 1, sustain at the reduction) up to their rounding: so a group whose
// positions' fill maxima (a.bm, 64-position blocks), raised by a relative 1e-9 margin
// for that rounding, are <= ceiling holds no candidate -- flagged or not -- and is
// skipped without loading a value, LP_NT groups per vote
__device__ __forceinline__ int lp_detect(const LpArgs &a, LpWave &W, int smp, int count, double &peak_value,
                         int &peak_slot) {
#ifdef AMX_LPV_NODETECT        // measurement variant: the limiter never engages (wrong output)
    return -1;
#endif
    const int lane = threadIdx.x;
    int slot0 = W.f.lbi + smp + LP_ATT;
    if (slot0 >= LP_RS) slot0 -= LP_RS;
    const double ceiling = a.ceiling;
    double pv0 = 0.0, pv1 = 0.0;               // n = 0 never qualifies (n > 0)
    double *st0 = W.st, *st1 = W.st + LP_STW;
    // the slots' bound: bm outside FINAL, bmF in FINAL (its frames hold u G_T offset fills,
    // multiplied by envelope gains <= 1, and 0 past the track: blocks from n on bound 0)
    const double *bmx = W.f.fin ? a.bmF : a.bm;
    const bool skip = bmx != nullptr;
    const int64_t nbx = W.f.fin ? (a.n + 63) >> 6 : INT64_MAX;
    // the positions of consecutive slots from slot0 are consecutive
    const int64_t pos0 = lp_pos(W.f, slot0);
    unsigned long long mask[LP_NW];
#pragma unroll
    for (int w = 0; w < LP_NW; w++) mask[w] = 0ull;
    int mask_base = -1;
    bool stale = false;
    int nb00 = 0;
    while (nb00 < count) {
        if (skip) {
            if (mask_base < 0 || nb00 >= mask_base + LP_NT * LP_NT) {
                // lane j: may group nb00 + LP_NT j hold a candidate?
                const int g0 = nb00 + LP_NT * lane;
                bool may = false;
                if (g0 < count) {
                    const int64_t p = pos0 + g0;
                    auto bnd = [&](int64_t bi) -> double { return bi < nbx ? bmx[bi] : 0.0; };
                    double mx = bnd(p >> 6);
#pragma unroll
                    for (int k = 1; k <= LP_NT / 64; k++) mx = fmax(mx, bnd((p + 64 * k - 1) >> 6));
                    may = mx * (1.0 + 1e-9) > ceiling;
                }
                lp_vote(W, may, mask);
                mask_base = nb00;
            }
            const int d = lp_next(mask, (nb00 - mask_base) / LP_NT) - (nb00 - mask_base) / LP_NT;
            if (d < 0) {
                nb00 = mask_base + LP_NT * LP_NT;
                mask_base = -1;
                stale = true;
                continue;
            }
            if (d > 0) {
                nb00 += LP_NT * d;
                stale = true;
                if (nb00 >= count) break;
            }
            if (stale) {
                // the predecessor: the value just before the group (skipped, so <= ceiling)
                int s = slot0 + nb00 - 1;
                while (s >= LP_RS) s -= LP_RS;
                const double2 v = lp_val(a, W, s);
                pv0 = fabs(v.x);
                pv1 = fabs(v.y);
                stale = false;
            }
        }
        // LP_PD groups from nb00 and the next one's first 12 positions (the look-ahead),
        // loaded together: one memory round trip per LP_PD groups.  Loads past count read
        // slots of the same ring window, in bounds, unused.
        double2 q[LP_PD + 1];
#pragma unroll
        for (int p = 0; p <= LP_PD; p++) q[p] = lp_grp(a, W, slot0 + nb00 + p * LP_NT, lane);
#pragma unroll
    for (int p = 0; p < LP_PD; p++) {
        const int nb0 = nb00 + LP_NT * p;
        if (nb0 >= count) break;
        {
            const double2 v = q[p], v2 = q[p + 1];
            __syncthreads();                   // the previous group's serial reads are done
            st0[lane] = fabs(v.x);
            st1[lane] = fabs(v.y);
            if (lane < 12) {
                st0[LP_NT + lane] = fabs(v2.x);
                st1[LP_NT + lane] = fabs(v2.y);
            }
            __syncthreads();
        }
        const int n = nb0 + lane;
        const int last = (count - nb0 < LP_NT ? count - nb0 : LP_NT) - 1;
        bool cand = false;
        if (n < count && n > 0) {
            const double t0 = st0[lane], t1 = st1[lane];
            const double p0 = lane == 0 ? pv0 : st0[lane - 1], p1 = lane == 0 ? pv1 : st1[lane - 1];
            cand = (p0 <= t0 && st0[lane + 1] <= t0 && t0 > ceiling) ||
                   (p1 <= t1 && st1[lane + 1] <= t1 && t1 > ceiling);
        }
        const int L0 = lp_first(W, cand);
        if (L0 < 0) {
            pv0 = st0[last];
            pv1 = st1[last];
            continue;
        }
        if (L0 > 0) {
            pv0 = st0[L0 - 1];
            pv1 = st1[L0 - 1];
        }
        for (int k = L0; k <= last; k++) {
            const int nn = nb0 + k;
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const double *sc = c ? st1 : st0;
                double &pv = c ? pv1 : pv0;
                const double t = sc[k];
                if (pv <= t && sc[k + 1] <= t && t > ceiling && nn > 0) {
                    bool detected = true;
                    for (int i = 2; i < 12; i++)
                        if (sc[k + i] > t) { detected = false; break; }
                    if (!detected) continue;
                    const double q0 = st0[k], q1 = st1[k];
                    peak_value = q1 > q0 ? q1 : q0;
                    int ps = slot0 + nn;
                    if (ps >= LP_RS) ps -= LP_RS;
                    peak_slot = ps;
                    return nn;
                }
                pv = t;
            }
        }
    }
        nb00 += LP_NT * LP_PD;
    }
    return -1;
}

// the output of the frame: the ring from its first slot, clamped to the ceiling, s16.
// Four groups' values are loaded before any output is stored (the stores could alias
// the loads for the compiler, which would otherwise wait out one load per group)
__device__ __forceinline__ void lp_emit(const LpArgs &a, const LpWave &W) {
    const double ceiling = a.ceiling;
    uint32_t *y = reinterpret_cast<uint32_t *>(a.y);
    const int nb = W.f.nb;
    for (int i00 = 0; i00 < nb; i00 += 4 * LP_NT) {
        double2 v[4];
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int i = i00 + LP_NT * p + (int)threadIdx.x;
            int s = W.f.lbi + i;
            while (s >= LP_RS) s -= LP_RS;
            v[p] = lp_val(a, W, s);                        // (i >= nb: read, unused)
        }
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int i = i00 + LP_NT * p + (int)threadIdx.x;
            if (i < nb) {
                double o0 = v[p].x, o1 = v[p].y;
                if (fabs(o0) > ceiling) o0 = ceiling * (o0 < 0 ? -1 : 1);
                if (fabs(o1) > ceiling) o1 = ceiling * (o1 < 0 ? -1 : 1);
                y[W.f.base + i] = pack2(ln_s16(o0), ln_s16(o1));
            }
        }
    }
}

#define LP_SPARSE_MAX 4096       // multiplied slots in a frame above which lp_emit_sparse emits densely
// the bits of flag word w inside slots [lo, lo + len) mod LP_RS
__device__ __forceinline__ unsigned lp_range_bits(int w, int lo, int len) {
    unsigned m = 0u;
#pragma unroll
    for (int part = 0; part < 2; part++) {
        const int a0 = part == 0 ? lo : 0;
        const int a1 = part == 0 ? min(lo + len, LP_RS) : max(lo + len - LP_RS, 0);
        const int b0 = w * 32;
        const int x0 = max(a0, b0) - b0, x1 = min(a1, b0 + 32) - b0;
        if (x1 > x0) m |= (x1 - x0 == 32) ? 0xffffffffu : (((1u << (x1 - x0)) - 1u) << x0);
    }
    return m;
}

// the output of the frame where k_lp_fill already wrote every position's unlimited
// value: only the slots the limiter multiplied differ -- their ring values, clamped, s16.
// AMX_LP_EMIT_RANGE (default): the frame positions from the first to the last flagged
// one, a lane per position and AMX_LP_EM groups of LP_NT per pass, each lane loading its
// ring slot unconditionally (slot 0 when unflagged) and storing only a flagged one -- one
// memory round trip per pass.  The per-word form below walked a word's set bits with a
// load each: a burst frame's thousands of flagged slots cost ~50 us of dependent loads
#ifndef AMX_LP_EMIT_RANGE
#define AMX_LP_EMIT_RANGE 1
#endif
#ifndef AMX_LP_EM
#define AMX_LP_EM 8
#endif
__device__ __forceinline__ void lp_emit_range(const LpArgs &a, const LpWave &W) {
    const int nb = W.f.nb, lbi = W.f.lbi;
    // the first and last flagged frame positions (i = slot - lbi mod LP_RS, i < nb).  The
    // frame's range (nb <= LP_FR, far below LP_RS - 32) never holds both ends of itself in
    // one word, so i rises with the slot inside a masked word: its lowest and highest set
    // bits give its extremes
    int lo = nb, hi = -1;
    for (int w = threadIdx.x; w < LP_FW; w += LP_NT) {
        const unsigned m = W.flags[w] & lp_range_bits(w, lbi, nb);
        if (m) {
            int i0 = 32 * w + __ffs(m) - 1 - lbi, i1 = 32 * w + 31 - __clz(m) - lbi;
            if (i0 < 0) i0 += LP_RS;
            if (i1 < 0) i1 += LP_RS;
            lo = min(lo, i0);
            hi = max(hi, i1);
        }
    }
    lo = -(int)lp_wg_max(W, -(double)lo);
    hi = (int)lp_wg_max(W, (double)hi);
    if (hi < lo) return;
    const double ceiling = a.ceiling;
    uint32_t *y = reinterpret_cast<uint32_t *>(a.y);
    for (int i00 = lo; i00 <= hi; i00 += AMX_LP_EM * LP_NT) {
        double2 v[AMX_LP_EM];
        bool fl[AMX_LP_EM];
#pragma unroll
        for (int p = 0; p < AMX_LP_EM; p++) {
            const int i = i00 + LP_NT * p + (int)threadIdx.x;
            int sl = lbi + i;
            if (sl >= LP_RS) sl -= LP_RS;
            fl[p] = i <= hi && lp_flag(W, sl < LP_RS ? sl : 0);
            v[p] = W.ring[fl[p] ? sl : 0];
        }
#pragma unroll
        for (int p = 0; p < AMX_LP_EM; p++) {
            if (fl[p]) {
                const int i = i00 + LP_NT * p + (int)threadIdx.x;
                double o0 = v[p].x, o1 = v[p].y;
                if (fabs(o0) > ceiling) o0 = ceiling * (o0 < 0 ? -1 : 1);
                if (fabs(o1) > ceiling) o1 = ceiling * (o1 < 0 ? -1 : 1);
                y[W.f.base + i] = pack2(ln_s16(o0), ln_s16(o1));
            }
        }
    }
}

__device__ __forceinline__ void lp_emit_sparse(const LpArgs &a, const LpWave &W) {
#if AMX_LP_EMIT_RANGE
    lp_emit_range(a, W);
    return;
#endif
    const int nb = W.f.nb, lbi = W.f.lbi;
    int cnt = 0;
    for (int w = threadIdx.x; w < LP_FW; w += LP_NT) cnt += __popc(W.flags[w] & lp_range_bits(w, lbi, nb));
    cnt = lp_wg_sum(W, cnt);
    if (cnt == 0) return;
    if (cnt > LP_SPARSE_MAX) {
        lp_emit(a, W);
        return;
    }
    const double ceiling = a.ceiling;
    uint32_t *y = reinterpret_cast<uint32_t *>(a.y);
    for (int w = threadIdx.x; w < LP_FW; w += LP_NT) {
        unsigned m = W.flags[w] & lp_range_bits(w, lbi, nb);
        while (m) {
            const int s = 32 * w + __ffs(m) - 1;
            m &= m - 1u;
            int i = s - lbi;
            if (i < 0) i += LP_RS;
            const double2 v = W.ring[s];
            double o0 = v.x, o1 = v.y;
            if (fabs(o0) > ceiling) o0 = ceiling * (o0 < 0 ? -1 : 1);
            if (fabs(o1) > ceiling) o1 = ceiling * (o1 < 0 ? -1 : 1);
            y[W.f.base + i] = pack2(ln_s16(o0), ln_s16(o1));
        }
    }
}

// true_peak_limiter on frame W.f (af_loudnorm), then its output: emit 0 none, 1 sparse
// (over k_lp_fill's output), 2 dense
__device__ __forceinline__ void lp_call(const LpArgs &a, LpWave &W, int emit) {
    const int nb = W.f.nb;
    const double ceiling = a.ceiling;
    if (W.f.phi == 0) {
        double mx = 0.0;
        for (int i = threadIdx.x; i < LP_ATT; i += LP_NT) {
            const double2 v = lp_val(a, W, i);
            mx = fmax(mx, fmax(fabs(v.x), fabs(v.y)));
        }
        mx = lp_wg_max(W, mx);
        if (mx > ceiling) {
            W.gr1 = ceiling / mx;
            W.mode = LO_SUSTAIN;
            const double g = W.gr1;
            lp_env(a, W, 0, LP_ATT, [&](int) { return g; });
        }
    }
    int smp = 0;
    double pv = 0.0;
    int pslot = 0;
    do {
        if (W.mode == LO_OUT) {
            const int pd = lp_detect(a, W, smp, nb - smp, pv, pslot);
            if (pd != -1) {
                W.env_cnt = 0;
                smp += (pd - W.attack_length);
                W.gr0 = 1.;
                W.gr1 = ceiling / pv;
                W.mode = LO_ATTACK;
                int e = pslot - W.attack_length;
                if (e < 0) e += LP_RS;
                e += W.env_cnt;
                if (e > LP_RS) e -= LP_RS;
                W.env_index = e;
            } else {
                smp = nb;
            }
        } else if (W.mode == LO_ATTACK) {
            int k = W.attack_length - W.env_cnt;
            if (k > nb - smp) k = nb - smp;
            if (k < 0) k = 0;
            const int c0 = W.env_cnt, al = W.attack_length;
            const double g0 = W.gr0, g1 = W.gr1;
            lp_env(a, W, W.env_index, k, [&](int i) { return g0 - ((double)(c0 + i) / (al - 1) * (g0 - g1)); });
            W.env_index = lp_env_end(W.env_index, k);
            W.env_cnt += k;
            smp += k;
            if (smp < nb) {
                W.env_cnt = 0;
                W.attack_length = LP_ATT;
                W.mode = LO_SUSTAIN;
            }
        } else if (W.mode == LO_SUSTAIN) {
            const int pd = lp_detect(a, W, smp, nb, pv, pslot);
            if (pd == -1) {
                W.mode = LO_RELEASE;
                W.gr0 = W.gr1;
                W.gr1 = 1.;
                W.env_cnt = 0;
            } else {
                const double gain_reduction = ceiling / pv;
                if (gain_reduction < W.gr1) {
                    W.mode = LO_ATTACK;
                    W.attack_length = pd <= 1 ? 2 : pd;
                    W.gr0 = W.gr1;
                    W.gr1 = gain_reduction;
                    W.env_cnt = 0;
                } else {
                    int k = pd;
                    if (k > nb - smp) k = nb - smp;
                    if (k < 0) k = 0;
                    const double g1 = W.gr1;
                    lp_env(a, W, W.env_index, k, [&](int) { return g1; });
                    W.env_index = lp_env_end(W.env_index, k);
                    W.env_cnt = k;
                    smp += k;
                }
            }
        } else {   // RELEASE
            const int rl = LP_FR;
            int k = rl - W.env_cnt;
            if (k > nb - smp) k = nb - smp;
            if (k < 0) k = 0;
            const int c0 = W.env_cnt;
            const double g0 = W.gr0, g1 = W.gr1;
            lp_env(a, W, W.env_index, k, [&](int i) { return g0 + (((double)(c0 + i) / (rl - 1)) * (g1 - g0)); });
            W.env_index = lp_env_end(W.env_index, k);
            W.env_cnt += k;
            smp += k;
            if (smp < nb) {
                W.env_cnt = 0;
                W.mode = LO_OUT;
            }
        }
    } while (smp < nb);
#ifdef AMX_LPV_NOEMIT          // measurement variant: no output (wrong output)
    emit = 0;
#endif
    if (emit == 1) lp_emit_sparse(a, W);
    else if (emit == 2) lp_emit(a, W);
}

__device__ __forceinline__ void lp_rest(LpWave &W) {        // af_loudnorm's initial limiter state
    lp_wg_barrier();                       // (the flags' previous readers are done)
    W.mode = LO_OUT;
    W.env_cnt = 0;
    W.env_index = 0;
    W.attack_length = LP_ATT;
    W.gr0 = 0.0;
    W.gr1 = 0.0;
    for (int w = threadIdx.x; w < LP_FW; w += LP_NT) W.flags[w] = 0u;
    __syncthreads();
}

// the state at the start of frame W.f (after its fill): scalars and the values of
// the 2048 slots from the frame's first; [LP_DIRTY] = a flag outside those slots
__device__ __forceinline__ void lp_snapshot(const LpArgs &a, const LpWave &W, double *rec) {
    const int lane = threadIdx.x;
    const int w0 = W.f.lbi;
    bool out = false;
    for (int w = lane; w < LP_FW; w += LP_NT) {
        unsigned m = W.flags[w];
        // clear the window's bits: slots [w0, w0 + LP_WIN) mod LP_RS
#pragma unroll
        for (int part = 0; part < 2; part++) {
            const int lo = part == 0 ? w0 : 0;
            const int hi = part == 0 ? min(w0 + LP_WIN, LP_RS) : max(w0 + LP_WIN - LP_RS, 0);
            const int b0 = w * 32;
            const int x0 = max(lo, b0) - b0, x1 = min(hi, b0 + 32) - b0;
            if (x1 > x0) m &= ~((x1 - x0 == 32) ? 0xffffffffu : (((1u << (x1 - x0)) - 1u) << x0));
        }
        out |= m != 0u;
    }
    const bool dirty = lp_first(W, out) >= 0;
#if AMX_LP_HANDOFF
    // the record goes out write-through (sc1, 16-B buffer stores): k_lp_seg's other
    // workgroups read it in this launch (lp_arrive), on any XCD, with no release fence.
    // The window's values are loaded half at a time before they are stored (two memory
    // round trips; all at once spilled).
    static_assert(LP_WIN % LP_NT == 0, "record window");
    constexpr int NS = LP_WIN / LP_NT;
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(rec, 0, LP_REC * (int)sizeof(double), 0x00020000);
    if (lane < 4) {                       // scalars 0..7, two per lane
        const double sc[8] = {(double)W.mode, (double)W.env_cnt, (double)W.env_index, (double)W.attack_length,
                              W.gr0, W.gr1, (double)W.f.phi, dirty ? 1.0 : 0.0};
        const double2 pr = make_double2(lane == 0 ? sc[0] : lane == 1 ? sc[2] : lane == 2 ? sc[4] : sc[6],
                                        lane == 0 ? sc[1] : lane == 1 ? sc[3] : lane == 2 ? sc[5] : sc[7]);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lp_u4, pr), rr, lane * 16, 0, 16);
    }
    constexpr int NH = NS / 2;
#pragma unroll 1
    for (int h = 0; h < 2; h++) {
        double2 v[NH];
#pragma unroll
        for (int q = 0; q < NH; q++) {
            int s = w0 + lane + (h * NH + q) * LP_NT;
            if (s >= LP_RS) s -= LP_RS;
#ifdef AMX_LPV_NOSNAP          // measurement variant: the window's values not loaded (wrong output)
            v[q] = make_double2(0.0, 0.0);
#else
            v[q] = lp_val(a, W, s);
#endif
        }
#pragma unroll
        for (int q = 0; q < NH; q++)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lp_u4, v[q]), rr,
                                                   (16 + 2 * (lane + (h * NH + q) * LP_NT)) * (int)sizeof(double), 0, 16);
    }
#else
    if (lane == 0) {
        rec[0] = W.mode;
        rec[1] = W.env_cnt;
        rec[2] = W.env_index;
        rec[3] = W.attack_length;
        rec[4] = W.gr0;
        rec[5] = W.gr1;
        rec[6] = W.f.phi;
        rec[LP_DIRTY] = dirty ? 1.0 : 0.0;
    }
    for (int j = lane; j < LP_WIN; j += LP_NT) {
        int s = w0 + j;
        if (s >= LP_RS) s -= LP_RS;
#ifdef AMX_LPV_NOSNAP          // measurement variant: the window's values not loaded (wrong output)
        const double2 v = make_double2(0.0, 0.0);
#else
        const double2 v = lp_val(a, W, s);
#endif
        rec[16 + 2 * j] = v.x;
        rec[17 + 2 * j] = v.y;
    }
#endif
}

// the same state back into a wave (every window slot flagged with its recorded value)
__device__ __forceinline__ void lp_restore(const LpArgs &a, LpWave &W, const double *rec, int phi) {
    lp_wg_barrier();                       // (the flags', gain rows' and ring's previous readers are done)
    W.f = lp_frame(a, phi);
    lp_gload(a, W);
    W.mode = (int)rec[0];
    W.env_cnt = (int)rec[1];
    W.env_index = (int)rec[2];
    W.attack_length = (int)rec[3];
    W.gr0 = rec[4];
    W.gr1 = rec[5];
    for (int w = threadIdx.x; w < LP_FW; w += LP_NT) W.flags[w] = 0u;
    __syncthreads();
    for (int j = threadIdx.x; j < LP_WIN; j += LP_NT) {
        int s = W.f.lbi + j;
        if (s >= LP_RS) s -= LP_RS;
        W.ring[s] = make_double2(rec[16 + 2 * j], rec[17 + 2 * j]);
        atomicOr(&W.flags[s >> 5], 1u << (s & 31));
    }
    lp_sync_ring();
}

__device__ __forceinline__ bool lp_bits_eq(double x, double y) {
    return __double_as_longlong(x) == __double_as_longlong(y);
}

// two states at the same frame lead to the same future: equal scalars (only the mode
// when both are at rest: OUT re-initialises the rest) and equal window values, and
// neither has a multiplied slot outside the window
__device__ __forceinline__ bool lp_same(const LpWave &W, const double *A, const double *B) {
    bool diff = A[LP_DIRTY] != 0.0 || B[LP_DIRTY] != 0.0 || (int)A[0] != (int)B[0];
    if ((int)A[0] != LO_OUT || (int)B[0] != LO_OUT)
        for (int q = 0; q < 6; q++) diff |= !lp_bits_eq(A[q], B[q]);
#if AMX_LP_HANDOFF
    // every load issued before any compare (one round trip, not one per pass)
    constexpr int NC = 2 * LP_WIN / LP_NT, NH = NC / 2;
#pragma unroll 1
    for (int h = 0; h < 2; h++) {
        double x[NH], y[NH];
#pragma unroll
        for (int q = 0; q < NH; q++) {
            x[q] = A[16 + threadIdx.x + (h * NH + q) * LP_NT];
            y[q] = B[16 + threadIdx.x + (h * NH + q) * LP_NT];
        }
#pragma unroll
        for (int q = 0; q < NH; q++) diff |= !lp_bits_eq(x[q], y[q]);
    }
#else
    for (int j = threadIdx.x; j < 2 * LP_WIN; j += LP_NT) diff |= !lp_bits_eq(A[16 + j], B[16 + j]);
#endif
    return lp_first(W, diff) < 0;
}

// boundary j: the later of segment j-1 (its end state) and segment j (its guess) to
// arrive compares them
// (every wave's record stores are released -- its own fence -- before lane 0 counts
// the arrival; the count is broadcast through LDS)
__device__ __forceinline__ void lp_arrive(const LpArgs &a, const LpWave &W, int j) {
#if AMX_LP_HANDOFF
    // the hand-off of DESIGN.md §3.7 / the guide's R1 form: the records were stored sc1
    // (lp_snapshot); every wave drains its stores, then one relaxed agent-scope count;
    // the second arriver acquires once (one lane's fence, its wait, the barrier) and reads
    // both records with plain loads.  __threadfence() here wrote back the whole L2 at
    // every arrival (2 per segment: the median segment spent ~180 us in snapshots and
    // arrivals, profiles/r06t_seg_times.txt)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        W.sv[0] = (unsigned long long)__hip_atomic_fetch_add(&a.cnt[j], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int old = (int)(unsigned)W.sv[0];
    if (old == 1) {
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const bool same = lp_same(W, a.recE + (int64_t)(j - 1) * LP_REC, a.recG + (int64_t)j * LP_REC);
        if (threadIdx.x == 0) a.match[j] = same ? 1 : 0;
    }
#else
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) W.sv[0] = (unsigned long long)(unsigned)atomicAdd(&a.cnt[j], 1);
    __syncthreads();
    const int old = (int)(unsigned)W.sv[0];
    if (old == 1) {
        __threadfence();
        const bool same = lp_same(W, a.recE + (int64_t)(j - 1) * LP_REC, a.recG + (int64_t)j * LP_REC);
        if (threadIdx.x == 0) a.match[j] = same ? 1 : 0;
    }
#endif
}

__device__ __forceinline__ void lp_wave_init(const LpArgs &a, LpWave &W, double2 *ring, unsigned *flags,
                                             double *st, unsigned long long *sv) {
    W.ring = ring;
    W.flags = flags;
    W.st = st;
    W.gl = st + 2 * LP_STW;
    W.sv = sv;
    W.tb = 0;
    W.gT = a.G[a.T];
    W.d0 = a.dctl[0];
    W.off = a.dctl[1];
}

// Every output position's unlimited value, before the limiter runs (the gains are known,
// fact 1 above): y = s16(clamp(fill)) over the positions [y_lo, y_hi) the segments emit,
// so k_lp_seg only writes the slots its limiter multiplied (lp_emit_sparse); and bm[b],
// the largest |fill| of positions [64 b, 64 b + 64) as a frame outside FINAL reads them
// (lp_val's unflagged value), for lp_detect's skip -- +inf for a block with a position
// outside [u_lo, u_hi) or past the track.  The fill is lp_val's expression term for
// term: u (gain ramp) offset for INNER positions, u d0 offset below the ring's first
// fill, u G_T offset for the positions FINAL emits.  One wave per 64-position block.
#ifndef AMX_LPF_GRID
#define AMX_LPF_GRID 65536
#endif
__global__ void __launch_bounds__(256) k_lp_fill(LpArgs a, int64_t y_lo, int64_t y_hi, int64_t u_lo, int64_t u_hi) {
    if ((a.ctl[0] != 0 && a.ctl[0] != 4) || a.T < 1) return;
    if (a.ctl[0] == 4) {
        // a quiet start: k_ln_dyn wrote the frames before the hand-over segment
        const int phi = lp_seg_start(a, a.ctl[4]);
        const int64_t b = phi <= a.T ? (int64_t)LP_FR * phi : a.S0 + (int64_t)LP_FR * (phi - a.T - 1);
        y_lo = y_lo > b ? y_lo : b;
    }
    const double d0 = a.dctl[0], off = a.dctl[1], gT = a.G[a.T], ceiling = a.ceiling;
    // four consecutive positions per thread (a 64-position block is 16 lanes): 32-B
    // loads of u, 16-B stores of y
    const int lane = threadIdx.x & 63;
    const int64_t b_lo = u_lo >> 6, b_hi = (u_hi + 63) >> 6;
    uint32_t *y = reinterpret_cast<uint32_t *>(a.y);
    const float4 *u4 = reinterpret_cast<const float4 *>(a.u);
    const double2 *ramp2 = reinterpret_cast<const double2 *>(a.ramp);      // (16-B aligned: lp_fill)
    const bool small = a.n < ((int64_t)1 << 31);          // wave-uniform: 32-bit quotients
    for (int64_t b = b_lo + (((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4); b < b_hi;
         b += ((int64_t)gridDim.x * 256) >> 4) {
        const int64_t p0 = 64 * b + 4 * (lane & 15);
        const bool whole = p0 >= u_lo && p0 + 4 <= u_hi && p0 + 4 <= a.n;
        double mx = 0.0, mxF = 0.0;
        if (whole) {
            const float4 xa = u4[p0 >> 1], xb = u4[(p0 >> 1) + 1];     // positions p0 .. p0 + 3
            const float xs[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
            // p0, LP_RS and LP_FR are multiples of 4, so the quad's positions lie in one
            // frame t at ramp indices i .. i + 3 (below LP_RS all four take d0): one pair of
            // gain rows and one 32-B ramp piece per quad, every load issued before any use
            const int64_t q = p0 - LP_RS > 0 ? p0 - LP_RS : 0;
            int t, i;
            if (small) {
                t = (int)((uint32_t)q / (uint32_t)LP_FR);
                i = (int)((uint32_t)q - (uint32_t)t * (uint32_t)LP_FR);
            } else {
                t = (int)(q / LP_FR);
                i = (int)(q - (int64_t)t * LP_FR);
            }
            const int tc = t < a.T - 1 ? t : a.T - 1;
            const double2 ra = ramp2[i >> 1], rb = ramp2[(i >> 1) + 1];
            const double g0 = a.G[tc], g1 = a.G[tc + 1];
            double rk[4] = {ra.x, ra.y, rb.x, rb.y};
            if (!(t < a.T - 1 || a.nb_last == LP_FR)) {            // the partial last frame's ramp
#pragma unroll
                for (int k = 0; k < 4; k++) rk[k] = (double)(i + k) / (double)a.nb_last;
            }
            // below LP_RS the gain is d0: as d0 + r * 0, which is d0 exactly (a positive gain)
            const bool below = p0 < LP_RS;
            const double gb = below ? d0 : g0, dg = below ? 0.0 : g1 - g0;
            double o[8];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const double g = gb + (rk[k] * dg);
                o[2 * k] = ((double)xs[2 * k] * g) * off;
                o[2 * k + 1] = ((double)xs[2 * k + 1] * g) * off;
                mx = fmax(mx, fmax(fabs(o[2 * k]), fabs(o[2 * k + 1])));
            }
            if (p0 + 3 >= a.S0) {                      // FINAL emits these: u G_T offset
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    if (p0 + k >= a.S0) {
                        o[2 * k] = ((double)xs[2 * k] * gT) * off;
                        o[2 * k + 1] = ((double)xs[2 * k + 1] * gT) * off;
                        mxF = fmax(mxF, fmax(fabs(o[2 * k]), fabs(o[2 * k + 1])));
                    }
                }
            }
            uint32_t ow[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                int16_t h[2];
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    // |v| > ceiling -> ceiling * sign (+-ceiling exactly) as one fmax / fmin
                    // pair (an in-range v, -0 included, passes unchanged)
                    const double v = fmin(fmax(o[2 * k + c], -ceiling), ceiling);
                    h[c] = ln_s16_lim(v);
                }
                ow[k] = pack2(h[0], h[1]);
            }
            if (p0 >= y_lo && p0 + 4 <= y_hi) {
                *reinterpret_cast<uint4 *>(y + p0) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (p0 + k >= y_lo && p0 + k < y_hi) y[p0 + k] = ow[k];
            }
        } else {
            // a block edge of the window or the track: any position outside holds no fill
            // (+inf: the scan never skips such a block); inside ones one at a time
            mx = HUGE_VAL;
            mxF = HUGE_VAL;
            const float2 *u = reinterpret_cast<const float2 *>(a.u);
            for (int k = 0; k < 4; k++) {
                const int64_t pos = p0 + k;
                if (!(pos >= u_lo && pos < u_hi && pos < a.n)) continue;
                const float2 x = u[pos];
                const int64_t q = pos - LP_RS > 0 ? pos - LP_RS : 0;
                const int t = (int)(q / LP_FR), i = (int)(q - (int64_t)t * LP_FR);
                const int tc = t < a.T - 1 ? t : a.T - 1;
                double r = a.ramp[i];
                if (!(t < a.T - 1 || a.nb_last == LP_FR)) r = (double)i / (double)a.nb_last;
                const double g0 = a.G[tc], g1 = a.G[tc + 1];
                const double gi = g0 + (r * (g1 - g0));
                const double g = pos < LP_RS ? d0 : gi;
                double o0 = ((double)x.x * g) * off, o1 = ((double)x.y * g) * off;
                if (pos >= a.S0) {
                    o0 = ((double)x.x * gT) * off;
                    o1 = ((double)x.y * gT) * off;
                }
                if (fabs(o0) > ceiling) o0 = ceiling * (o0 < 0 ? -1 : 1);
                if (fabs(o1) > ceiling) o1 = ceiling * (o1 < 0 ? -1 : 1);
                if (pos >= y_lo && pos < y_hi) y[pos] = pack2(ln_s16(o0), ln_s16(o1));
            }
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            mx = fmax(mx, __shfl_xor(mx, o));
            mxF = fmax(mxF, __shfl_xor(mxF, o));
        }
        if ((lane & 15) == 0) {
            a.bm[b] = mx;
            if (a.bmF) a.bmF[b] = mxF;
        }
    }
}

// every segment at once (persistent waves): from rest Wf frames before its start
#ifndef AMX_LP_WPE
#define AMX_LP_WPE 3             // k_lp_seg waves per SIMD the register budget allows (168
                                 // VGPRs, a 300-B spill; 2: C5 dynamic 43.0 vs 40.9 ms)
#endif
__global__ void __launch_bounds__(LP_NT) __attribute__((amdgpu_waves_per_eu(AMX_LP_WPE))) k_lp_seg(LpArgs a) {
    if (a.ctl[0] != 0 && a.ctl[0] != 4) return;
    const int kh = a.ctl[0] == 4 ? a.ctl[4] : 0;     // a quiet start: k_ln_dyn ran segments < kh
    __shared__ unsigned flags[LP_FW];
    __shared__ double st[2 * LP_STW + 8];
    __shared__ unsigned long long sv[LP_NW];
    LpWave W;
    lp_wave_init(a, W, reinterpret_cast<double2 *>(a.rings) + (int64_t)blockIdx.x * LP_RS, flags, st, sv);
    const int NF = a.T + 1 + LP_NFIN;
    for (int k = a.kb + blockIdx.x; k < a.ke; k += gridDim.x) {
        if (k < kh) continue;
        const int ak = lp_seg_start(a, k), bk = k + 1 < a.K ? lp_seg_start(a, k + 1) : NF;
        if (k == kh && kh > 0) {
            // the hand-over segment starts from k_ln_dyn's true state (recG[kh])
            lp_restore(a, W, a.recG + (int64_t)k * LP_REC, ak);
            for (int phi = ak; phi < bk; phi++) {
                if (phi > ak) {
                    W.f = lp_frame(a, phi);
                    lp_refill(a, W, phi);
                }
                lp_call(a, W, a.bm ? 1 : 2);
            }
        } else {
            const int w = ak - a.Wf > 0 ? ak - a.Wf : 0;
            lp_rest(W);
            for (int phi = w; phi < bk; phi++) {
                W.f = lp_frame(a, phi);
                lp_refill(a, W, phi);
                if (phi == ak) {
                    lp_snapshot(a, W, a.recG + (int64_t)k * LP_REC);
                    if (k > kh) lp_arrive(a, W, k);
                }
                lp_call(a, W, phi >= ak ? (a.bm ? 1 : 2) : 0);
            }
        }
        if (k + 1 < a.K) {
            W.f = lp_frame(a, bk);
            lp_refill(a, W, bk);
            lp_snapshot(a, W, a.recE + (int64_t)k * LP_REC);
            lp_arrive(a, W, k + 1);
        }
    }
}

// in order over the boundaries: skip the matched ones, re-run a segment whose start
// guess was wrong from the true state (rewriting its output).  If the limiter is
// active where FINAL re-bases the ring, FINAL runs here from that state.  A true state
// with a multiplied slot outside its window (never expected) hands the whole track
// to k_ln_dyn (ctl[0] = 2).
// A shard (a.rec_in, chunk-sharded tracks): the walk covers the boundaries [kb, ke) from
// the true state at kb that the previous rank's walker made, and leaves the true state at
// ke in a.rec_out for the next rank (marked dirty when this walk fell back).
__global__ void __launch_bounds__(LP_NT) k_lp_walk(LpArgs a) {
    if (a.ctl[0] != 0 && a.ctl[0] != 4) return;
    const int kh = a.ctl[0] == 4 ? a.ctl[4] : 0;
    __shared__ unsigned flags[LP_FW];
    __shared__ double st[2 * LP_STW + 8];
    __shared__ unsigned long long sv[LP_NW];
    LpWave W;
    lp_wave_init(a, W, reinterpret_cast<double2 *>(a.wring), flags, st, sv);
    const int lane = threadIdx.x;
    const int NF = a.T + 1 + LP_NFIN, kS0 = a.J + 1, ke = a.ke;
    const double *cur = a.rec_in ? a.rec_in : a.recE + (int64_t)kh * LP_REC;
    bool k4 = a.rec_in == nullptr;
    int toggle = 0, reruns = 0, fin = 0, fallback = 0;
    int k = a.rec_in ? a.kb : kh + 1;
    while (k < ke) {
        if (k4) {
            while (k < ke) {
                const int j = k + lane;
                const bool stop = j >= ke || j == kS0 || a.match[j] == 0;
                const int f = lp_first(W, stop);
                if (f >= 0) {
                    k += f;
                    break;
                }
                k += LP_NT;
            }
            cur = a.recE + (int64_t)(k - 1) * LP_REC;
            if (k >= ke) break;
        }
        if (cur[LP_DIRTY] != 0.0) {
            fallback = 1;
            break;
        }
        if (k == kS0 && (int)cur[0] != LO_OUT) {
            lp_restore(a, W, cur, a.T + 1);
            for (int phi = a.T + 1; phi < NF; phi++) {
                if (phi > a.T + 1) {
                    W.f = lp_frame(a, phi);
                    lp_refill(a, W, phi);
                }
                lp_call(a, W, 2);
            }
            fin = 1;
            break;
        }
        const bool ok = k4 ? (a.match[k] != 0) : lp_same(W, cur, a.recG + (int64_t)k * LP_REC);
        if (ok) {
            cur = a.recE + (int64_t)k * LP_REC;
            k4 = true;
            k++;
            continue;
        }
        const int ak = lp_seg_start(a, k), bk = k + 1 < a.K ? lp_seg_start(a, k + 1) : NF;
        lp_restore(a, W, cur, ak);
        for (int phi = ak; phi < bk; phi++) {
            if (phi > ak) {
                W.f = lp_frame(a, phi);
                lp_refill(a, W, phi);
            }
            lp_call(a, W, 2);
        }
        reruns++;
        if (k + 1 < a.K) {
            W.f = lp_frame(a, bk);
            lp_refill(a, W, bk);
            double *r = a.wrec + (int64_t)toggle * LP_REC;
            toggle ^= 1;
            lp_snapshot(a, W, r);
            lp_sync_ring();                // (the record's stores, read by every wave next)
            cur = r;
            k4 = false;
        }
        k++;
    }
    if (a.rec_out && ke < a.K) {
        // the true state at boundary ke for the next rank's walk
        for (int q = lane; q < LP_REC; q += LP_NT) a.rec_out[q] = cur[q];
        __syncthreads();
        if (lane == 0 && fallback) a.rec_out[LP_DIRTY] = 1.0;
    }
    if (lane == 0) {
        if (fallback) a.ctl[0] = 2;
        a.ctl[1] = reruns;
        a.ctl[2] = fin;
        a.summary[0] = 0.0;
        a.summary[1] = 1.0;
        for (int q = 2; q < 10; q++) a.summary[q] = 0.0;
        a.summary[10] = (double)reruns;
        a.summary[11] = (double)fin;
        a.summary[12] = (double)a.K;
        a.summary[13] = (double)fallback;
        a.summary[14] = a.ctl[0] == 4 ? (double)a.ctl[5] : 0.0;    // quiet start: hand-over frame
    }
}

static_assert(LP_RS % 4 == 0 && LP_FR % 4 == 0, "k_lp_fill: a quad of positions lies in one frame");
static hipError_t lp_fill(const LpArgs &lp, int64_t y_lo, int64_t y_hi, int64_t u_lo, int64_t u_hi,
                          hipStream_t st) {
    // (the ramp's 32-B pieces: the plan's scratch is 256-B aligned)
    if (reinterpret_cast<uintptr_t>(lp.ramp) % 16 != 0) return hipErrorInvalidValue;
    const int64_t blocks = ((u_hi + 63) >> 6) - (u_lo >> 6);
    if (blocks <= 0) return hipSuccess;
    // grid-stride over at most AMX_LPF_GRID workgroups (a gated track's launch returns at
    // once); a workgroup covers 16 blocks.  65 536 rather than 4 096: 5 us less per launch
    // at C3 (profiles/r06ac_lp_fill_ab.txt)
    const int64_t g = (blocks + 15) / 16;
    hipLaunchKernelGGL(k_lp_fill, dim3((unsigned)(g < AMX_LPF_GRID ? g : AMX_LPF_GRID)), dim3(256), 0, st, lp, y_lo, y_hi, u_lo,
                       u_hi);
    return hipSuccess;
}

static void ln_upsample(const uint32_t *x, int64_t n_in, const SwrDev &r, int64_t j0, int64_t j1, float *u,
                        const int32_t *gate, hipStream_t st) {
    if (j1 <= j0) return;
    // grid-stride over at most 8192 workgroups: a gated (linear) track's launch then
    // dispatches a bounded number of workgroups that return at once
    auto grid = [](int64_t n) {
        const int64_t nb = (n + AMX_BLOCK - 1) / AMX_BLOCK;
        return dim3((unsigned)(nb < 8192 ? nb : 8192));
    };
    if (r.taps != LN_TAPS) {
        hipLaunchKernelGGL(k_ln_upsample_wide, grid(j1 - j0), dim3(AMX_BLOCK), 0, st, x, n_in, r, j0, j1, u, gate);
        return;
    }
    if (!r.lin && r.src == r.dst) {
        const int64_t nf = ((j1 + r.pc - 1) / r.pc - j0 / r.pc + LN_UPF - 1) / LN_UPF;   // frame blocks
        switch (r.pc) {
#define LN_UPS(LL) \
        case LL: hipLaunchKernelGGL(k_ln_up_static<LL>, grid(nf), dim3(AMX_BLOCK), 0, st, x, n_in, r.bank, j0, j1, u, gate); return;
        LN_UPS(1) LN_UPS(2) LN_UPS(3) LN_UPS(4) LN_UPS(6)
#undef LN_UPS
        default: break;
        }
    }
    hipLaunchKernelGGL(k_ln_upsample, grid(j1 - j0), dim3(AMX_BLOCK), 0, st, x, n_in, r, j0, j1, u, gate);
}

hipError_t launch_loudnorm(const LnArgs &ln, const LpArgs &lp, const uint32_t *x, int64_t n_in,
                           const SwrDev &r, bool resample, hipStream_t st) {
    if (ln.n192 <= 0) return hipSuccess;
    if (resample) ln_upsample(x, n_in, r, 0, ln.n192, ln.u, lp.gate, st);
    // reuse (pass 2 on pass 1's scratch): the frames' statistics depend on the input's hop
    // energies alone and stand -- only block 0, the resolved options, runs
    hipLaunchKernelGGL(k_lp_stats, dim3(resample ? 1 + (lp.T + LP_STAT_F - 1) / LP_STAT_F : 1), dim3(LP_STAT_NT), 0,
                       st, lp);
    hipLaunchKernelGGL(k_ln_dyn, dim3(1), dim3(LN_NT), 0, st, ln, 0);
    hipLaunchKernelGGL(k_lp_dscan, dim3(1), dim3(1024), 0, st, lp);
    const int gb = max((lp.T + 1 + 255) / 256, (LP_FR + 255) / 256);
    hipLaunchKernelGGL(k_lp_gains, dim3(gb), dim3(256), 0, st, lp);
    hipError_t e = lp.bm ? lp_fill(lp, 0, ln.n192, 0, ln.n192, st) : hipSuccess;
    if (e != hipSuccess) return e;
    e = launch_zero(lp.cnt, sizeof(int) * (size_t)(lp.K + 1), st);
    if (e != hipSuccess) return e;
    e = launch_zero(lp.match, sizeof(int) * (size_t)(lp.K + 1), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lp_seg, dim3(lp.P), dim3(LP_NT), 0, st, lp);
    hipLaunchKernelGGL(k_lp_walk, dim3(1), dim3(LP_NT), 0, st, lp);
    hipLaunchKernelGGL(k_ln_dyn, dim3(1), dim3(LN_NT), 0, st, ln, 1);
    return hipGetLastError();
}

// a chunk-sharded track's share of one filter run (amx_loudnorm_192k_shard), in three
// parts the host puts the rank-to-rank hand-off between: 0 -- the 192 kHz stream over
// [u_lo, u_hi) and every frame's statistics (the host then reads lp.ctl[0]: 0 = the
// parallel form runs, else the whole track must run frame by frame); 1 -- deltas, gains
// and the segments [kb, ke); 2 -- the walk over their boundaries from lp.rec_in
hipError_t launch_loudnorm_shard(const LnArgs &ln, const LpArgs &lp, const uint32_t *x, int64_t n_in,
                                 const SwrDev &r, int64_t u_lo, int64_t u_hi, int64_t y_lo, int64_t y_hi, int part,
                                 bool resample, hipStream_t st) {
    if (ln.n192 <= 0) return hipSuccess;
    if (part == 0) {
        if (resample) ln_upsample(x, n_in, r, u_lo, u_hi, ln.u, lp.gate, st);
        hipLaunchKernelGGL(k_lp_stats, dim3(resample ? 1 + (lp.T + LP_STAT_F - 1) / LP_STAT_F : 1), dim3(LP_STAT_NT),
                           0, st, lp);
    } else if (part == 1) {
        hipLaunchKernelGGL(k_lp_dscan, dim3(1), dim3(1024), 0, st, lp);
        const int gb = max((lp.T + 1 + 255) / 256, (LP_FR + 255) / 256);
        hipLaunchKernelGGL(k_lp_gains, dim3(gb), dim3(256), 0, st, lp);
        hipError_t e = lp.bm ? lp_fill(lp, y_lo, y_hi, u_lo, u_hi, st) : hipSuccess;
        if (e != hipSuccess) return e;
        e = launch_zero(lp.cnt, sizeof(int) * (size_t)(lp.K + 1), st);
        if (e != hipSuccess) return e;
        e = launch_zero(lp.match, sizeof(int) * (size_t)(lp.K + 1), st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_lp_seg, dim3(lp.P), dim3(LP_NT), 0, st, lp);
    } else if (part == 2) {
        hipLaunchKernelGGL(k_lp_walk, dim3(1), dim3(LP_NT), 0, st, lp);
    } else {
        // part 3 (rank 0 of a quiet start): the frames in order from the track start until
        // the hand-over segment (k_ln_dyn phase 0, bounded by ln.lp_tstop)
        hipLaunchKernelGGL(k_ln_dyn, dim3(1), dim3(LN_NT), 0, st, ln, 0);
    }
    return hipGetLastError();
}

}  // namespace amx
