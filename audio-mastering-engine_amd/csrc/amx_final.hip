// amx_final.hip -- loudnorm linear gain (:240) + alimiter (:223).
#include "amx_dev.hpp"

namespace amx {

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

// limiter never engages (proved from the sample peak: max|gained x| <= limit):
// att == 1, delta == 0 for every frame, so out[n] = level-scaled input[n - (B-1)]
// (B = ring frames).  A workgroup covers AMX_BLOCK * FPT frames of one track span;
// thread k handles frames k, k + AMX_BLOCK, ... so every load and store instruction
// of a wave is one contiguous 256-B run, with FPT independent loads in flight.
// ctl (nullable): per-track decision word of k_decide; this kernel only runs the
// tracks whose AMX_CTL_FAST bit is set.
// UNIT (level_in == level_out == 1, limit*32768 <= 32767 -- the reference's
// alimiter settings, :223): the same values with fewer fp64 operations.  Scaling by
// 2^15 commutes with rounding and x*1 is exact, so
//   gain16(x)        = clip(rint(x * g))                    (one rounding in x*g)
//   limiter(v) * 2^15 = rint(clamp(v, +-limit*2^15) * level) (one rounding in *level)
// and the gain stage's own clip is subsumed by the +-limit*2^15 clamp.
#define AMX_FINAL_FPT 8
typedef uint32_t fu4v __attribute__((ext_vector_type(4)));

// one stereo frame through the gain stage and the idle limiter
template <bool UNIT>
__device__ __forceinline__ uint32_t final_frame(uint32_t p, double g, double level_in,
                                                double level, double level_out, double limit) {
    int16_t o[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        if constexpr (UNIT) {
            double v = (double)(c ? hi16(p) : lo16(p));
            if (g > 0.0) v = rint(v * g);
            const double l32 = limit * 32768.0;
            v = v < -l32 ? -l32 : (v > l32 ? l32 : v);
            o[c] = clip_llrint(v * level);
        } else {
            int16_t v = gain16(c ? hi16(p) : lo16(p), g);
            double smp = ((double)v * (1.0 / 32768.0)) * level_in;
            double d = smp * 1.0;
            d = d < -limit ? -limit : (d > limit ? limit : d);
            d = d * level * level_out;
            o[c] = clip_llrint(d * 32768.0);
        }
    }
    return pack2(o[0], o[1]);
}

template <bool UNIT>
__device__ __forceinline__ void final_fast_block(const SpanDev *__restrict__ spans,
                                                 const uint32_t *__restrict__ x,
                                                 const uint32_t *__restrict__ halo,
                                                 int halo_frames,
                                                 const double *__restrict__ gains,
                                                 double level_in, double level,
                                                 double level_out, double limit,
                                                 uint32_t *__restrict__ y) {
    const int t = blockIdx.y;
    const SpanDev sp = spans[t];
    const int64_t blk0 = (int64_t)blockIdx.x * (AMX_BLOCK * AMX_FINAL_FPT);
    if (blk0 >= sp.out_n) return;                    // block-uniform
    const double g = gains[t];
    const int h = halo_frames;
    // Interior blocks (every source frame inside the span, whole block in range, the
    // span 16-B aligned): thread t owns 4 consecutive frames per group, so every load
    // and store instruction of a wave moves one contiguous KiB in 16-B pieces.  The
    // delay h makes the source run start at word r = (-h) mod 4 of an aligned 4-frame
    // vector: two aligned vectors are loaded and r selects the window (the neighbour
    // lane loads the same lines, so HBM sees each byte once).
    if (blk0 >= h + 3 && blk0 + AMX_BLOCK * AMX_FINAL_FPT <= sp.out_n && (sp.out_off & 3) == 0 &&
        h >= 4) {
        const int r = (4 - (h & 3)) & 3;
        const uint32_t *xs = x + sp.out_off;
        fu4v v0[AMX_FINAL_FPT / 4], v1[AMX_FINAL_FPT / 4];
#pragma unroll
        for (int m = 0; m < AMX_FINAL_FPT / 4; m++) {
            const int64_t i = blk0 + 4 * threadIdx.x + (int64_t)m * 4 * AMX_BLOCK;
            const int64_t base = i - h - r;          // aligned: i % 4 == 0, (h + r) % 4 == 0
            v0[m] = *reinterpret_cast<const fu4v *>(xs + base);
            v1[m] = *reinterpret_cast<const fu4v *>(xs + base + 4);
        }
#pragma unroll
        for (int m = 0; m < AMX_FINAL_FPT / 4; m++) {
            const int64_t i = blk0 + 4 * threadIdx.x + (int64_t)m * 4 * AMX_BLOCK;
            uint32_t w[8] = {v0[m].x, v0[m].y, v0[m].z, v0[m].w, v1[m].x, v1[m].y, v1[m].z, v1[m].w};
            fu4v o;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t p = r == 0 ? w[q] : (r == 1 ? w[q + 1] : (r == 2 ? w[q + 2] : w[q + 3]));
                o[q] = final_frame<UNIT>(p, g, level_in, level, level_out, limit);
            }
            *reinterpret_cast<fu4v *>(y + sp.out_off + i) = o;
        }
        return;
    }
    // edge blocks: one frame per load, frames before the span from the halo
    const int64_t i0 = blk0 + threadIdx.x;
    uint32_t p[AMX_FINAL_FPT];
#pragma unroll
    for (int m = 0; m < AMX_FINAL_FPT; m++) {
        const int64_t i = i0 + (int64_t)m * AMX_BLOCK;
        const int64_t src = i - halo_frames;      // span-local source frame (delay B-1)
        const int64_t cs = src < 0 ? 0 : (src >= sp.out_n ? sp.out_n - 1 : src);
        // one unconditional load from a selected address (see tile_load): frames
        // before the span come from the halo, frames before the track are silence
        const uint32_t *a = src < 0 ? halo + (int64_t)t * halo_frames + (halo_frames + src)
                                    : x + sp.out_off + cs;
        const uint32_t v = *a;
        p[m] = (sp.tframe0 + src < 0) ? 0u : v;
    }
#pragma unroll
    for (int m = 0; m < AMX_FINAL_FPT; m++) {
        const int64_t i = i0 + (int64_t)m * AMX_BLOCK;
        const uint32_t o = final_frame<UNIT>(p[m], g, level_in, level, level_out, limit);
        if (i < sp.out_n) y[sp.out_off + i] = o;
    }
}

// General alimiter (af_alimiter.c filter_frame, asc off), one wave per track span.
// The recurrence is sequential and runs on lane 0 with the ring buffer, nextdelta
// and nextpos in LDS (dynamic shared memory, 3 bs doubles); the wave loads, gains
// and converts 64 frames at a time in parallel around it (coalesced loads and
// stores, the per-sample gain stage off the sequential chain).  The operation
// sequence per frame is the reference's.  State layout in `state` (doubles), for
// the rank-to-rank hand-off: [0] att [1] delta [2] pos [3] nextiter [4] nextlen
// [5] valid  [8 .. 8+bs) buffer  [8+bs .. 8+2bs) nextdelta  [8+2bs .. 8+3bs) nextpos.
#define AMX_LIM_BATCH 64
__device__ void final_general_wave(int t, const SpanDev *__restrict__ spans,
                                   const uint32_t *__restrict__ x,
                                   const uint32_t *__restrict__ halo, int halo_frames,
                                   const double *__restrict__ gains, int fs, double level_in,
                                   double level, double level_out, double limit, double release,
                                   int bs, double *__restrict__ state, int64_t state_doubles,
                                   uint32_t *__restrict__ y, double *lds) {
    const int lane = threadIdx.x & 63;
    const SpanDev sp = spans[t];
    const int channels = 2;
    double *S = state + (int64_t)t * state_doubles;
    double *buffer = lds, *nextdelta = lds + bs, *nextposd = lds + 2 * bs;
    double *inb = lds + 3 * bs, *outb = inb + 2 * AMX_LIM_BATCH;
    const double g = gains[t];
    const bool fresh = sp.tframe0 == 0 || S[5] == 0.0;
    for (int k = lane; k < bs; k += 64) {
        buffer[k] = fresh ? 0.0 : S[8 + k];
        nextdelta[k] = fresh ? 0.0 : S[8 + bs + k];
        nextposd[k] = fresh ? -1.0 : S[8 + 2 * bs + k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    double att = 1.0, delta = 0.0;
    int pos = 0, nextiter = 0, nextlen = 0;
    if (lane == 0) {
        if (fresh) {
            if (sp.tframe0 != 0) {
                // no carried state: prime the ring with the halo (limiter assumed idle)
                for (int h = 0; h < halo_frames; h++) {
                    uint32_t p = halo[(int64_t)t * halo_frames + h];
                    for (int c = 0; c < channels; c++)
                        buffer[pos + c] = ((double)gain16(c ? hi16(p) : lo16(p), g) * (1.0 / 32768.0)) * level_in;
                    pos = (pos + channels) % bs;
                }
            }
        } else {
            att = S[0]; delta = S[1]; pos = (int)S[2]; nextiter = (int)S[3]; nextlen = (int)S[4];
        }
    }
#define NEXTPOS(k) ((int)nextposd[(k)])
    for (int64_t base = 0; base < sp.out_n; base += AMX_LIM_BATCH) {
        const int nb = (int)(sp.out_n - base < AMX_LIM_BATCH ? sp.out_n - base : AMX_LIM_BATCH);
        if (lane < nb) {
            const uint32_t p = x[sp.out_off + base + lane];
            for (int c = 0; c < channels; c++)
                inb[2 * lane + c] = ((double)gain16(c ? hi16(p) : lo16(p), g) * (1.0 / 32768.0)) * level_in;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            for (int k = 0; k < nb; k++) {
                double dst[2];
                double peak = 0;
                for (int c = 0; c < channels; c++) {
                    const double sample = inb[2 * k + c];
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
                for (int c = 0; c < channels; c++) outb[2 * k + c] = dst[c];
                pos = (pos + channels) % bs;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (lane < nb) {
            int16_t o[2];
            for (int c = 0; c < channels; c++) {
                double v = outb[2 * lane + c];
                v = v < -limit ? -limit : (v > limit ? limit : v);
                v = v * level * level_out;
                o[c] = clip_llrint(v * 32768.0);
            }
            y[sp.out_off + base + lane] = pack2(o[0], o[1]);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
#undef NEXTPOS
    if (lane == 0) {
        S[0] = att; S[1] = delta; S[2] = pos; S[3] = nextiter; S[4] = nextlen; S[5] = 1.0;
    }
    for (int k = lane; k < bs; k += 64) {
        S[8 + k] = buffer[k];
        S[8 + bs + k] = nextdelta[k];
        S[8 + 2 * bs + k] = nextposd[k];
    }
}

// One launch for both limiter paths.  Columns blockIdx.x < gridDim.x - 1 are the
// parallel idle-limiter pass of track blockIdx.y; the last column runs the
// sequential general limiter for that track (thread 0).  With ctl (k_decide's
// word) each track takes exactly one of them; without it `fast` picks for all.
struct FinalArgs {
    const SpanDev *spans;
    const uint32_t *x, *halo;
    int halo_frames, fs, bs, fast;
    const double *gains;
    const int32_t *ctl;
    double level_in, level, level_out, limit, release;
    double *state;
    int64_t state_doubles;
    uint32_t *y;
};

template <bool UNIT>
__global__ void __launch_bounds__(AMX_BLOCK) k_final(FinalArgs a) {
    extern __shared__ double lim_lds[];                 // general path: 3 bs + 4 x 64 doubles
    const int t = blockIdx.y;
    const bool fast = a.ctl ? (a.ctl[t] & AMX_CTL_FAST) != 0 : a.fast != 0;
    if (blockIdx.x + 1 < gridDim.x) {
        if (fast)
            final_fast_block<UNIT>(a.spans, a.x, a.halo, a.halo_frames, a.gains, a.level_in,
                                   a.level, a.level_out, a.limit, a.y);
    } else if (!fast && threadIdx.x < 64) {
        final_general_wave(t, a.spans, a.x, a.halo, a.halo_frames, a.gains, a.fs, a.level_in,
                           a.level, a.level_out, a.limit, a.release, a.bs, a.state,
                           a.state_doubles, a.y, lim_lds);
    }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_final(const SpanDev *spans, int n_tracks, int64_t max_span, const int16_t *x,
                        const int16_t *halo, int halo_frames, const double *gains,
                        const int32_t *ctl, int fast, int fs, double level_in, double level,
                        double level_out, double limit, double release, int buffer_size,
                        double *state, int64_t state_doubles, int16_t *y, hipStream_t st) {
    const int64_t per = (int64_t)AMX_BLOCK * AMX_FINAL_FPT;
    dim3 g((unsigned)((max_span + per - 1) / per) + 1, (unsigned)n_tracks);
    if (n_tracks <= 0) return hipSuccess;
    FinalArgs a{spans, reinterpret_cast<const uint32_t *>(x), reinterpret_cast<const uint32_t *>(halo),
                halo_frames, fs, buffer_size, fast, gains, ctl, level_in, level, level_out, limit,
                release, state, state_doubles, reinterpret_cast<uint32_t *>(y)};
    const bool unit = level_in == 1.0 && level_out == 1.0 && limit * 32768.0 <= 32767.0;
    const size_t lds = ((size_t)3 * buffer_size + 4 * AMX_LIM_BATCH) * sizeof(double);
    if (lds > 64 * 1024) return hipErrorInvalidValue;   // bs <= 2645: attack <= 13.7 ms at 96 kHz
    if (unit) hipLaunchKernelGGL(k_final<true>, g, dim3(AMX_BLOCK), lds, st, a);
    else hipLaunchKernelGGL(k_final<false>, g, dim3(AMX_BLOCK), lds, st, a);
    return hipGetLastError();
}

}  // namespace amx
