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

// one thread per 192 kHz frame: both channels
__global__ void __launch_bounds__(AMX_BLOCK) k_ln_upsample(const uint32_t *__restrict__ x, int64_t n_in,
                                                           int L, int M, const float *__restrict__ bank,
                                                           int64_t n192, float *__restrict__ u) {
    const int64_t j = (int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x;
    if (j >= n192) return;
    const int64_t idx = j * M, base = idx / L;
    const int ph = (int)(idx % L);
    float w0[LN_TAPS], w1[LN_TAPS];
#pragma unroll
    for (int i = 0; i < LN_TAPS; i++) {
        const uint32_t v = x[ln_reflect(base - LN_C + i, n_in)];
        w0[i] = (float)lo16(v) * (1.0f / 32768.0f);
        w1[i] = (float)hi16(v) * (1.0f / 32768.0f);
    }
    const float *h = bank + (int64_t)ph * LN_TAPS;
    u[2 * j] = ln_dot(w0, h);
    u[2 * j + 1] = ln_dot(w1, h);
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
};

__device__ __forceinline__ int ln_find_bin(const double *B, double e) {
    int lo = 0, hi = 1000;
    do {
        const int mid = (lo + hi) / 2;
        if (e >= B[mid]) lo = mid; else hi = mid;
    } while (hi - lo != 1);
    return lo;
}

// ebur128 gated loudness + relative threshold of the histogram (every thread)
__device__ void ln_global(LnShared &L, double &global, double &rel_thr) {
    const int tid = threadIdx.x;
    double s = 0.0, c = 0.0;
    for (int j = tid; j < 1000; j += LN_NT) { s += (double)L.hist[j] * L.E[j]; c += (double)L.hist[j]; }
    s = ln_bsum(s, L.red);
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
    double g = 0.0, a = 0.0;
    for (int j = start + tid; j < 1000; j += LN_NT) { g += (double)L.hist[j] * L.E[j]; a += (double)L.hist[j]; }
    g = ln_bsum(g, L.red);
    a = ln_bsum(a, L.red);
    global = a == 0.0 ? -HUGE_VAL : 10 * log10(g / a) - 0.691;
}

// gating block ending at hop k (k >= 4): the mean square of hops k-4 .. k-1
__device__ __forceinline__ void ln_add_block(LnShared &L, const double *hops, int64_t k) {
    const double c0 = ((hops[2 * (k - 4)] + hops[2 * (k - 3)]) + hops[2 * (k - 2)]) + hops[2 * (k - 1)];
    const double c1 = ((hops[2 * (k - 4) + 1] + hops[2 * (k - 3) + 1]) + hops[2 * (k - 2) + 1]) + hops[2 * (k - 1) + 1];
    const double en = (c0 + c1) / (double)(4 * LN_FR);
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

__global__ void __launch_bounds__(LN_NT) k_ln_dyn(LnArgs a) {
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
        if (tid == 0) { a.summary[0] = 1.0; a.summary[1] = off; }
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
    // ---- INNER frames (100 ms)
    while (Pin < n) {
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
    }
}

hipError_t launch_loudnorm(const LnArgs &a, const uint32_t *x, int64_t n_in, int L, int M,
                           const float *bank, hipStream_t st) {
    if (a.n192 <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_ln_upsample, dim3((unsigned)((a.n192 + AMX_BLOCK - 1) / AMX_BLOCK)), dim3(AMX_BLOCK),
                       0, st, x, n_in, L, M, bank, a.n192, a.u);
    hipLaunchKernelGGL(k_ln_dyn, dim3(1), dim3(LN_NT), 0, st, a);
    return hipGetLastError();
}

}  // namespace amx
