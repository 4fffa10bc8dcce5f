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

// ------------------------------------------------------------ general alimiter
// af_alimiter.c filter_frame (asc off) for a track span where the limiter can
// engage.  The recurrence is sequential; it is parallelised exactly:
//  * Rest state.  After a release completes (the att > 1 reset) the state is
//    att = 1, delta = 0, nextlen = nextiter = 0, nextpos[0] = -1 (entries past the
//    list terminator are never read before they are rewritten), and the ring holds
//    only the last B/2 input frames, which the input alone determines.  Call it
//    IDLE.  From IDLE, frames whose peak is <= limit keep it IDLE and output the
//    delayed input at att = 1: such stretches are skipped 64 frames per step (a
//    wave ballot finds the next frame over the limit, lanes write the delayed
//    outputs); only active stretches run frame by frame, the whole wave in step
//    (the pending-peak list search 64 entries at a time), with the ring,
//    nextdelta and nextpos in LDS.
//  * Segments (parallel, one wave each).  The span is cut into segments of LS
//    frames.  Segment 0 runs from the exact span start state.  Segment k > 0
//    starts from IDLE W frames early (or from the exact span start when that is
//    before the span), runs the warm-up without output, records its guess G_k of
//    the state at its first frame, then runs the segment with output and records
//    its end state E_k.  A release takes ~ release·fs frames, so the guess is
//    exact unless the limiter stays active through the whole warm-up.
//  * Walk (the last wave of the track to finish).  State equality is exact
//    equality of the scalars and the live list (nextpos / nextdelta from nextiter
//    to the terminator) at the same canonical ring positions.  If E_{k-1} == G_k,
//    segment k ran from its true start and E_k is its true end; the walker checks
//    64 boundaries per step.  At the first mismatch it re-runs segment k from the
//    true state, rewriting its output, and compares the new end with G_{k+1}.
// Output is bit-identical to the sequential filter (tests/test_gpu_parity.py).
// State layout (doubles) of the hand-off `state` and of each G / E slot:
// [0] att [1] delta [2] pos [3] nextiter [4] nextlen [5] valid, [8 .. 8+B) ring,
// [8+B .. 8+2B) nextdelta, [8+2B .. 8+3B) nextpos.  Ring positions are canonical:
// span frame f sits at (P0 + 2 f) mod B, so states of different waves compare.
#define AMX_LIM_BATCH 64

struct LimArgs {
    const SpanDev *spans;
    const uint32_t *x, *halo;
    int halo_frames, fs, bs, seg_frames, warm_frames, max_segs, fast;
    int from_rest;          // amx_final_desc.from_rest: every span starts fresh, `state` is out only
    double *att;            // [out frames] each output frame's att (amx_plan_set_limiter_trace), or NULL
    int64_t warm_cap;
    const double *gains;
    const int32_t *ctl;
    double level_in, level, level_out, limit, release;
    double *state;          // [tracks][state_doubles] hand-off state in / out
    int64_t state_doubles;
    double *seg_state;      // [tracks][max_segs][2][state_doubles]: G_k, E_k
    unsigned *cnt;          // [tracks] finished-block counters (re-armed by the walker)
    uint32_t *y;
};

struct Lim {
    const uint32_t *xs, *hl;    // span input (x + out_off), the track's halo row
    uint32_t *ys;
    double *as;                 // the span's att trace (LimArgs.att), or NULL
    int64_t n, tframe0;
    double g, level_in, level, level_out, limit, release;
    int fs, bs, halo, P0;
    bool from_rest;             // the carried state is not read (LimArgs.from_rest)
    double *buffer, *nextdelta, *nextposd, *inb, *outb;   // LDS
    double att, delta;          // scalar state, identical in every lane between batches
    int nextiter, nextlen;
};

__device__ __forceinline__ double lim_sample(const Lim &L, uint32_t p, int c) {
    return ((double)gain16(c ? hi16(p) : lo16(p), L.g) * (1.0 / 32768.0)) * L.level_in;
}
// ring position of span frame f (f >= -halo)
__device__ __forceinline__ int lim_pos(const Lim &L, int64_t f) {
    const int64_t q = ((int64_t)L.P0 + 2 * f) % L.bs;
    return (int)(q < 0 ? q + L.bs : q);
}
__device__ __forceinline__ int16_t lim_out(const Lim &L, double v) {
    v = v < -L.limit ? -L.limit : (v > L.limit ? L.limit : v);
    v = v * L.level * L.level_out;
    return clip_llrint(v * 32768.0);
}
__device__ __forceinline__ bool lim_is_idle(const Lim &L) {
    return L.att == 1.0 && L.delta == 0.0 && L.nextlen == 0 && L.nextiter == 0 && L.nextposd[0] == -1.0;
}
// ring slots of span frames [max(lo, 0), hi) from the input, lanes in parallel
__device__ void lim_reload(Lim &L, int64_t lo, int64_t hi) {
    const int lane = threadIdx.x & 63;
    if (lo < 0) lo = 0;
    for (int64_t f = lo + lane; f < hi; f += 64) {
        const uint32_t p = L.xs[f];
        const int q = lim_pos(L, f);
        L.buffer[q] = lim_sample(L, p, 0);
        L.buffer[q + 1] = lim_sample(L, p, 1);
    }
    amx_wave_sync();
}
__device__ void lim_set_idle(Lim &L) {
    for (int k = threadIdx.x & 63; k < L.bs; k += 64) {
        L.nextdelta[k] = 0.0;
        L.nextposd[k] = -1.0;
    }
    L.att = 1.0;
    L.delta = 0.0;
    L.nextiter = 0;
    L.nextlen = 0;
    amx_wave_sync();
}
// The span's start state, exactly as the sequential filter has it: carried in
// `S` (valid), or fresh -- silence before the track, or the halo frames before a
// span that starts inside it (limiter assumed idle there).
__device__ void lim_init_span(Lim &L, const double *S) {
    const int lane = threadIdx.x & 63;
    const bool fresh = L.tframe0 == 0 || L.from_rest || S[5] == 0.0;
    for (int k = lane; k < L.bs; k += 64) {
        L.buffer[k] = fresh ? 0.0 : S[8 + k];
        L.nextdelta[k] = fresh ? 0.0 : S[8 + L.bs + k];
        L.nextposd[k] = fresh ? -1.0 : S[8 + 2 * L.bs + k];
    }
    amx_wave_sync();
    if (fresh) {
        L.att = 1.0; L.delta = 0.0; L.nextiter = 0; L.nextlen = 0;
        if (L.tframe0 != 0) {
            for (int h = lane; h < L.halo; h += 64) {
                const uint32_t p = L.hl[h];
                L.buffer[2 * h] = lim_sample(L, p, 0);
                L.buffer[2 * h + 1] = lim_sample(L, p, 1);
            }
        }
    } else {
        L.att = S[0]; L.delta = S[1]; L.nextiter = (int)S[3]; L.nextlen = (int)S[4];
    }
    amx_wave_sync();
}
__device__ __forceinline__ int lim_p0(const SpanDev &sp, const double *S, int halo, int bs, bool from_rest) {
    const bool fresh = sp.tframe0 == 0 || from_rest || S[5] == 0.0;
    return fresh ? (sp.tframe0 != 0 ? (2 * halo) % bs : 0) : (int)S[2];
}
__device__ __forceinline__ int lim_wrap(int v, int bs) { return v >= bs ? v - bs : v; }

__device__ __forceinline__ double lim_readlane(double v, int k) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, k);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The whole wave, frames f .. f+nb-1 (first frame at ring position pos): the
// reference's operation sequence per frame, every lane holding the same scalars.
// Lane k holds frame f+k's samples (s0, s1) and the delayed samples the ring
// returns for it (d0, d1: frame f+k-halo -- the ring only ever holds input
// samples), read by the wave with readlane, so a frame without list work makes no
// LDS round trip; `head` caches nextpos[nextiter].  The ring is still written
// (the list search reads it).  The pending-peak search evaluates 64 entries per
// step, one per lane, each with the reference's own expression.  Lane k keeps
// frame k's dst in o0, o1.  Stops after the first frame that leaves the state
// IDLE (nowidle).  Returns the frames done.
__device__ int lim_seq(Lim &L, int nb, int pos, double s0v, double s1v, double d0v, double d1v,
                       double &o0, double &o1, double &oa, bool &nowidle) {
    const int lane = threadIdx.x & 63;
    const int bs = L.bs, channels = 2;
    const double limit = L.limit;
    double att = L.att, delta = L.delta;
    int nextiter = L.nextiter, nextlen = L.nextlen;
    double *buffer = L.buffer, *nextdelta = L.nextdelta, *nextposd = L.nextposd;
#define NEXTPOS(k) ((int)nextposd[(k)])
    int head = NEXTPOS(nextiter);
    int k = 0;
    nowidle = false;
    while (k < nb) {
        const double x0 = lim_readlane(s0v, k), x1 = lim_readlane(s1v, k);
        if (lane == 0) {
            buffer[pos] = x0;
            buffer[pos + 1] = x1;
        }
        double peak = fmax(fmax(0.0, fabs(x0)), fabs(x1));
        if (peak > limit) {
            amx_wave_sync();
            double patt = fmin(limit / peak, 1.);
            double rdelta = (1.0 - patt) / (L.fs * L.release);
            double d = (limit / peak - att) / bs * channels;
            if (d < delta) {
                delta = d;
                if (lane == 0) {
                    nextposd[0] = pos;
                    nextposd[1] = -1;
                    nextdelta[0] = rdelta;
                }
                nextlen = 1;
                nextiter = 0;
            } else {
                int i = -1;                          // the first entry found
                double pfound = 0.0;
                for (int b0 = 0; b0 < nextlen; b0 += 64) {
                    const int e = b0 + lane;
                    bool hit = false;
                    double pdelta = 0.0;
                    if (e < nextlen) {
                        const int jx = (nextiter + e) % bs;
                        const int np = NEXTPOS(jx);
                        double ppeak = 0;
                        for (int c = 0; c < channels; c++) ppeak = fmax(ppeak, fabs(buffer[np + c]));
                        const int dist = ((bs - np + pos) % bs) / channels;
                        // equal peaks: the reference's (A - A) / dist is exactly +0 (dist >
                        // 0), so a steady over-limit stretch needs no division here
                        pdelta = (ppeak == peak && dist > 0) ? 0.0 : (limit / peak - limit / ppeak) / dist;
                        hit = pdelta < nextdelta[jx];
                    }
                    const unsigned long long bal = __ballot(hit);
                    if (bal) {
                        const int l = __ffsll(bal) - 1;
                        i = nextiter + b0 + l;
                        pfound = __shfl(pdelta, l);
                        break;
                    }
                }
                if (i >= 0) {
                    amx_wave_sync();
                    if (lane == 0) nextdelta[i % bs] = pfound;
                    nextlen = i - nextiter + 1;
                    if (lane == 0) {
                        nextposd[(nextiter + nextlen) % bs] = pos;
                        nextdelta[(nextiter + nextlen) % bs] = rdelta;
                        nextposd[(nextiter + nextlen + 1) % bs] = -1;
                    }
                    nextlen++;
                }
            }
            amx_wave_sync();
            head = NEXTPOS(nextiter);
        }
        const int bp = lim_wrap(pos + channels, bs);
        const double b0 = lim_readlane(d0v, k), b1 = lim_readlane(d1v, k);
        peak = fmax(fmax(0.0, fabs(b0)), fabs(b1));
        att += delta;
        const double dst0 = b0 * att, dst1 = b1 * att;
        const double att_used = att;
        if (bp == head) {
            amx_wave_sync();
            delta = nextdelta[nextiter];
            att = limit / peak;
            nextlen -= 1;
            amx_wave_sync();
            if (lane == 0) nextposd[nextiter] = -1;
            nextiter = lim_wrap(nextiter + 1, bs);
            amx_wave_sync();
            head = NEXTPOS(nextiter);
        }
        if (att > 1.) {
            att = 1.; delta = 0.; nextiter = 0; nextlen = 0;
            amx_wave_sync();
            if (lane == 0) nextposd[0] = -1;
            head = -1;
        }
        if (att <= 0.) { att = 0.0000000000001; delta = (1.0 - att) / (L.fs * L.release); }
        if (att != 1. && (1. - att) < 0.0000000000001) att = 1.;
        if (delta != 0. && fabs(delta) < 0.00000000000001) delta = 0.;
        if (lane == k) {
            o0 = dst0;
            o1 = dst1;
            oa = att_used;
        }
        pos = bp;
        k++;
        if (att == 1.0 && delta == 0.0 && nextlen == 0 && nextiter == 0 && head == -1) {
            nowidle = true;
            break;
        }
    }
#undef NEXTPOS
    amx_wave_sync();
    L.att = att; L.delta = delta; L.nextiter = nextiter; L.nextlen = nextlen;
    return k;
}

// Warm-up start for the segment at seg0: the latest frame w0 <= seg0 whose R
// frames before it are all at or under the limit (then the limiter has almost
// surely come to rest by w0), found by scanning back 64 frames per ballot; at
// most `cap` frames back.  Returns <= 0 when the scan reaches the span start.
__device__ int64_t lim_warm_start(const Lim &L, int64_t seg0, int64_t R, int64_t cap) {
    const int lane = threadIdx.x & 63;
    int64_t w0 = seg0;
    const int64_t floor_ = seg0 - cap;
    int64_t b = w0;                                   // scan [.., b) downwards
    while (true) {
        if (w0 <= 0) return 0;
        if (w0 <= floor_) return w0;
        if (b <= w0 - R || b <= 0) return w0;          // [w0 - R, w0) is clean
        const int64_t i = b - 64 + lane;
        bool over = false;
        if (i >= 0 && i >= w0 - R) {
            const uint32_t q = L.xs[i];
            over = fmax(fabs(lim_sample(L, q, 0)), fabs(lim_sample(L, q, 1))) > L.limit;
        }
        const unsigned long long bal = __ballot(over);
        if (bal) {
            w0 = b - 64 + (63 - __clzll(bal));          // the latest frame over the limit
            b = w0;
        } else {
            b -= 64;
        }
    }
}

// Runs span frames [f, fend) from the state in L (idle: it is IDLE), writing the
// output when OUT.
template <bool OUT>
__device__ void lim_run(Lim &L, int64_t f, int64_t fend, bool idle) {
    const int lane = threadIdx.x & 63;
    while (f < fend) {
        if (idle) {
            int64_t tgt = fend;
            for (int64_t b = f; b < fend; b += 64) {
                const int64_t i = b + lane;
                bool over = false;
                if (i < fend) {
                    const uint32_t q = L.xs[i];
                    over = fmax(fabs(lim_sample(L, q, 0)), fabs(lim_sample(L, q, 1))) > L.limit;
                }
                const unsigned long long bal = __ballot(over);
                const int64_t stop = bal ? b + (__ffsll(bal) - 1) : min(b + 64, fend);
                if (OUT && i < stop) {                // delayed input at att = 1
                    const int64_t src = i - L.halo;
                    double v0, v1;
                    if (src >= 0) {
                        const uint32_t q = L.xs[src];
                        v0 = lim_sample(L, q, 0);
                        v1 = lim_sample(L, q, 1);
                    } else {
                        const int r = lim_pos(L, src);
                        v0 = L.buffer[r];
                        v1 = L.buffer[r + 1];
                    }
                    L.ys[i] = pack2(lim_out(L, v0 * 1.0), lim_out(L, v1 * 1.0));
                    if (L.as) L.as[i] = 1.0;
                }
                if (bal) { tgt = stop; break; }
            }
            f = tgt;
            if (tgt == fend) break;
            lim_reload(L, f - L.halo, f);
            idle = false;
        } else {
            const int nb = (int)min((int64_t)AMX_LIM_BATCH, fend - f);
            double s0 = 0.0, s1 = 0.0, d0 = 0.0, d1 = 0.0;
            if (lane < nb) {
                const uint32_t q = L.xs[f + lane];
                s0 = lim_sample(L, q, 0);
                s1 = lim_sample(L, q, 1);
                const int64_t src = f + lane - L.halo;
                if (src >= 0) {
                    const uint32_t qd = L.xs[src];
                    d0 = lim_sample(L, qd, 0);
                    d1 = lim_sample(L, qd, 1);
                } else {                             // before the span: the initial ring
                    const int r = lim_pos(L, src);
                    d0 = L.buffer[r];
                    d1 = L.buffer[r + 1];
                }
            }
            bool nowidle = false;
            double o0 = 0.0, o1 = 0.0, oa = 1.0;
            const int kd = lim_seq(L, nb, lim_pos(L, f), s0, s1, d0, d1, o0, o1, oa, nowidle);
            if (OUT && lane < kd) {
                L.ys[f + lane] = pack2(lim_out(L, o0), lim_out(L, o1));
                if (L.as) L.as[f + lane] = oa;
            }
            f += kd;
            idle = nowidle;
        }
    }
}

// The segment records are read by the walker, another workgroup of this launch on any
// XCD: stored write-through (agent-scope atomic stores, sc1) so the hand-off needs no
// release fence (limiter_block: drain, relaxed count, one acquire in the walker)
__device__ __forceinline__ void lim_st(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ void lim_store(const Lim &L, double *E, int64_t f_end, bool with_ring) {
    const int lane = threadIdx.x & 63;
    if (lane == 0) {
        lim_st(E + 0, L.att); lim_st(E + 1, L.delta); lim_st(E + 2, (double)lim_pos(L, f_end));
        lim_st(E + 3, (double)L.nextiter); lim_st(E + 4, (double)L.nextlen);
        lim_st(E + 5, 1.0);
    }
    for (int k = lane; k < L.bs; k += 64) {
        if (with_ring) lim_st(E + 8 + k, L.buffer[k]);
        lim_st(E + 8 + L.bs + k, L.nextdelta[k]);
        lim_st(E + 8 + 2 * L.bs + k, L.nextposd[k]);
    }
}
__device__ void lim_load(Lim &L, const double *E) {
    for (int k = threadIdx.x & 63; k < L.bs; k += 64) {
        L.nextdelta[k] = E[8 + L.bs + k];
        L.nextposd[k] = E[8 + 2 * L.bs + k];
    }
    L.att = E[0]; L.delta = E[1]; L.nextiter = (int)E[3]; L.nextlen = (int)E[4];
    amx_wave_sync();
}
// state equality: scalars, then the live list from nextiter to its terminator
// (A, B: slot layout; either may be LDS-backed through the nd / np pointers)
__device__ bool lim_equal(double a_att, double a_delta, int a_it, int a_len, const double *a_nd,
                          const double *a_np, const double *B, int bs) {
    if (!(a_att == B[0] && a_delta == B[1] && a_it == (int)B[3] && a_len == (int)B[4])) return false;
    const double *b_nd = B + 8 + bs, *b_np = B + 8 + 2 * bs;
    bool ok = true;
    for (int i = threadIdx.x & 63; i <= a_len; i += 64) {
        const int j = (a_it + i) % bs;
        ok = ok && a_np[j] == b_np[j] && (i == a_len || a_nd[j] == b_nd[j]);
    }
    return __ballot(!ok) == 0ull;
}

// Wave 0 of general block bx of nbx (columns of k_final): runs segments bx,
// bx + nbx, ... of track blockIdx.y; the last block to finish walks them.
__device__ void limiter_block(const LimArgs &a, int bx, int nbx, double *lim_lds) {
    const int t = blockIdx.y;
    const int lane = threadIdx.x;
    const SpanDev sp = a.spans[t];
    Lim L;
    L.xs = a.x + sp.out_off;
    L.hl = a.halo + (int64_t)t * a.halo_frames;
    L.ys = a.y + sp.out_off;
    L.as = a.att ? a.att + sp.out_off : nullptr;
    L.n = sp.out_n;
    L.tframe0 = sp.tframe0;
    L.g = a.gains[t];
    L.level_in = a.level_in; L.level = a.level; L.level_out = a.level_out;
    L.limit = a.limit; L.release = a.release;
    L.fs = a.fs; L.bs = a.bs; L.halo = a.halo_frames;
    L.from_rest = a.from_rest != 0;
    L.buffer = lim_lds; L.nextdelta = lim_lds + a.bs; L.nextposd = lim_lds + 2 * a.bs;
    L.inb = lim_lds + 3 * a.bs; L.outb = L.inb + 2 * AMX_LIM_BATCH;
    double *S = a.state + (int64_t)t * a.state_doubles;
    L.P0 = lim_p0(sp, S, a.halo_frames, a.bs, L.from_rest);
    const int LS = a.seg_frames;
    const int nseg = (int)((sp.out_n + LS - 1) / LS);
    const int64_t sd = a.state_doubles;
    double *slots = a.seg_state + (int64_t)t * a.max_segs * 2 * sd;
#define GSLOT(k) (slots + (int64_t)(k) * 2 * sd)
#define ESLOT(k) (slots + (int64_t)(k) * 2 * sd + sd)

    // 1. segments: warm-up (no output) -> G_k, segment (output) -> E_k
    for (int s = bx; s < nseg; s += nbx) {
        const int64_t seg0 = (int64_t)s * LS;
        const int64_t fend = min(sp.out_n, seg0 + LS);
        if (s > 0) {
            const int64_t w0 = lim_warm_start(L, seg0, a.warm_frames, a.warm_cap);
            if (w0 <= 0) {
                lim_init_span(L, S);
                lim_run<false>(L, 0, seg0, lim_is_idle(L));
            } else {
                lim_set_idle(L);
                lim_reload(L, w0 - L.halo, w0);
                lim_run<false>(L, w0, seg0, true);
            }
            lim_store(L, GSLOT(s), seg0, false);
        } else {
            lim_init_span(L, S);
        }
        lim_run<true>(L, seg0, fend, lim_is_idle(L));
        lim_store(L, ESLOT(s), fend, false);
        amx_wave_sync();
    }

    // 2. the last block of the track walks (one wave per block: its drain, then the count;
    // the walker acquires once before it reads the other blocks' records)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned old = 0;
    if (lane == 0) old = __hip_atomic_fetch_add(a.cnt + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = __shfl(old, 0);
    if (old != (unsigned)nbx - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) a.cnt[t] = 0u;
    lim_init_span(L, S);                               // ring content before the span
    bool in_lds = false;                               // true end of segment k-1 is in L
    int k = 1;
    while (k < nseg) {
        if (!in_lds) {
            // first boundary k' >= k with E_{k'-1} != G_{k'}
            int kk = nseg;
            for (int b = k; b < nseg && kk == nseg; b += 64) {
                const int j = b + lane;
                int st = 0;                            // 0 equal, 1 differs, 2 compare lists
                if (j < nseg) {
                    const double *E = ESLOT(j - 1), *G = GSLOT(j);
                    if (!(E[0] == G[0] && E[1] == G[1] && E[3] == G[3] && E[4] == G[4])) st = 1;
                    else if (E[4] != 0.0) st = 2;
                    else {
                        const int it = (int)E[3];
                        st = E[8 + 2 * a.bs + it] == G[8 + 2 * a.bs + it] ? 0 : 1;
                    }
                }
                unsigned long long m = __ballot(st == 2);
                while (m) {
                    const int l = __ffsll(m) - 1;
                    const double *E = ESLOT(b + l - 1);
                    const bool eq = lim_equal(E[0], E[1], (int)E[3], (int)E[4], E + 8 + a.bs,
                                              E + 8 + 2 * a.bs, GSLOT(b + l), a.bs);
                    if (lane == l) st = eq ? 0 : 1;
                    m &= m - 1;
                }
                const unsigned long long d = __ballot(st == 1);
                if (d) kk = b + __ffsll(d) - 1;
            }
            if (kk >= nseg) break;
            k = kk;
            lim_load(L, ESLOT(k - 1));
        } else if (lim_equal(L.att, L.delta, L.nextiter, L.nextlen, L.nextdelta, L.nextposd,
                             GSLOT(k), a.bs)) {
            in_lds = false;                            // segment k ran from its true start
            k++;
            continue;
        }
        // re-run segment k from the true state in L
        const int64_t seg0 = (int64_t)k * LS;
        lim_reload(L, seg0 - L.halo, seg0);
        lim_run<true>(L, seg0, min(sp.out_n, seg0 + LS), lim_is_idle(L));
        in_lds = true;
        k++;
    }
    // hand-off state at the span end: the walker's own run, else the last segment's
    if (!in_lds && nseg > 0) lim_load(L, ESLOT(nseg - 1));
    lim_reload(L, sp.out_n - a.bs / 2, sp.out_n);
    lim_store(L, S, sp.out_n, true);
#undef GSLOT
#undef ESLOT
}

// One launch for both limiter paths of every track: columns x < fast_cols are
// the idle-limiter pass, the gen_cols after them the general limiter (wave 0 of
// each, limiter_block).  With ctl (k_decide's word) each track takes exactly one
// of them; without it `fast` picks for all.
struct FinalArgs {
    LimArgs lim;
    int fast_cols, gen_cols;
    const int32_t *gate;      // amx_plan_set_gate (a 192 kHz side plan in a captured step)
};

template <bool UNIT>
__global__ void __launch_bounds__(AMX_BLOCK, 8) k_final(FinalArgs fa) {
    extern __shared__ double lim_lds[];               // general columns: 3 B + 4 x 64 doubles
    if (AMX_LN_GATED(fa.gate)) return;
    const LimArgs &a = fa.lim;
    const int t = blockIdx.y;
    const bool fast = a.ctl ? (a.ctl[t] & AMX_CTL_FAST) != 0 : a.fast != 0;
    if ((int)blockIdx.x < fa.fast_cols) {
        if (fast)
            final_fast_block<UNIT>(a.spans, a.x, a.halo, a.halo_frames, a.gains, a.level_in,
                                   a.level, a.level_out, a.limit, a.y);
    } else if (!fast && threadIdx.x < 64) {
        limiter_block(a, (int)blockIdx.x - fa.fast_cols, fa.gen_cols, lim_lds);
    }
}

// ---------------------------------------------------------------- launchers
size_t limiter_lds_bytes(int buffer_size) {
    return ((size_t)3 * buffer_size + 4 * AMX_LIM_BATCH) * sizeof(double);
}

// a workgroup may declare all of a CU's 160 KiB of LDS on gfx950: the general columns'
// ring (3 B doubles) then fits a 5 ms attack up to ~670 kHz (B <= 6741; 384 kHz: 3 840)
hipError_t limiter_allow_lds(size_t bytes) {
    if (bytes > AMX_LIM_LDS_MAX) return hipErrorInvalidValue;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_final<true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)AMX_LIM_LDS_MAX);
    if (e == hipSuccess)
        e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_final<false>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)AMX_LIM_LDS_MAX);
    return e;
}

// ------------------------------------------------ more than two channels (round 6)
// af_alimiter's state (att, delta, the pending-peak list) evolves from each frame's
// largest |gained sample| alone: the peak over the channels when a frame enters, and
// that of the delayed frame (the ring only ever holds input samples; its list entries
// are compared through their frames' peaks).  So a stereo run over a "peak signal" --
// per frame the sample of the loudest channel in both channels -- goes through the same
// states, and its att trace (amx_plan_set_limiter_trace) gives every channel's output.
__global__ void __launch_bounds__(AMX_BLOCK) k_mc_peak_pick(const int16_t *__restrict__ y, int64_t frames,
                                                           int C, const double *__restrict__ gain,
                                                           uint32_t *__restrict__ syn) {
    const int64_t f = (int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x;
    if (f >= frames) return;
    const double g = gain[0];
    const int16_t *row = y + f * C;
    int16_t best = row[0];
    int bv = abs((int)gain16(best, g));
    for (int k = 1; k < C; k++) {
        const int16_t v = row[k];
        const int a = abs((int)gain16(v, g));
        if (a > bv) { bv = a; best = v; }
    }
    syn[f] = pack2(best, best);
}

// out[f][c] = the limiter output of channel c's gained sample B - 1 frames earlier (0
// before the track) x att[f] -- the operations of lim_run / af_alimiter per channel
__global__ void __launch_bounds__(AMX_BLOCK) k_mc_limiter_out(const int16_t *__restrict__ y, int64_t frames,
                                                             int C, int halo, const double *__restrict__ gains,
                                                             const int32_t *__restrict__ ctl,
                                                             const double *__restrict__ att, double level_in,
                                                             double level, double level_out, double limit,
                                                             int16_t *__restrict__ out) {
    const int64_t f = (int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x;
    if (f >= frames) return;
    const double g = gains[0];
    const bool fast = (ctl[0] & AMX_CTL_FAST) != 0;
    const double a = fast ? 1.0 : att[f];
    const int64_t src = f - halo;
    for (int k = 0; k < C; k++) {
        const double b = src >= 0 ? ((double)gain16(y[src * C + k], g) * (1.0 / 32768.0)) * level_in : 0.0;
        double v = b * a;
        v = v < -limit ? -limit : (v > limit ? limit : v);
        v = v * level * level_out;
        out[f * C + k] = clip_llrint(v * 32768.0);
    }
}

hipError_t launch_mc_peak_pick(const int16_t *y, int64_t frames, int C, const double *gain, int16_t *syn,
                               hipStream_t st) {
    if (frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mc_peak_pick, dim3((unsigned)((frames + AMX_BLOCK - 1) / AMX_BLOCK)), dim3(AMX_BLOCK), 0,
                       st, y, frames, C, gain, reinterpret_cast<uint32_t *>(syn));
    return hipGetLastError();
}

hipError_t launch_mc_limiter_out(const int16_t *y, int64_t frames, int C, int halo_frames, const double *gains,
                                 const int32_t *ctl, const double *att, double level_in, double level,
                                 double level_out, double limit, int16_t *out, hipStream_t st) {
    if (frames <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_mc_limiter_out, dim3((unsigned)((frames + AMX_BLOCK - 1) / AMX_BLOCK)), dim3(AMX_BLOCK),
                       0, st, y, frames, C, halo_frames, gains, ctl, att, level_in, level, level_out, limit, out);
    return hipGetLastError();
}

hipError_t launch_final(const SpanDev *spans, int n_tracks, int64_t max_span, const int16_t *x,
                        const int16_t *halo, int halo_frames, const double *gains,
                        const int32_t *ctl, int fast, int fs, double level_in, double level,
                        double level_out, double limit, double release, int buffer_size,
                        double *state, int64_t state_doubles, int from_rest, const LimScratch &ls,
                        int16_t *y, hipStream_t st) {
    if (n_tracks <= 0) return hipSuccess;
    const int64_t per = (int64_t)AMX_BLOCK * AMX_FINAL_FPT;
    const bool unit = level_in == 1.0 && level_out == 1.0 && limit * 32768.0 <= 32767.0;
    const bool general = ctl != nullptr || !fast;
    FinalArgs fa{};
    LimArgs &a = fa.lim;
    a.spans = spans;
    a.x = reinterpret_cast<const uint32_t *>(x);
    a.halo = reinterpret_cast<const uint32_t *>(halo);
    a.halo_frames = halo_frames; a.fs = fs; a.bs = buffer_size; a.fast = fast;
    a.gains = gains; a.ctl = ctl;
    a.level_in = level_in; a.level = level; a.level_out = level_out; a.limit = limit;
    a.release = release;
    a.state = state; a.state_doubles = state_doubles; a.from_rest = from_rest;
    a.y = reinterpret_cast<uint32_t *>(y);
    fa.fast_cols = (ctl != nullptr || fast) ? (int)((max_span + per - 1) / per) : 0;
    fa.gate = ls.gate;
    a.att = ls.att;
    size_t lds = 0;
    if (general) {
        lds = limiter_lds_bytes(buffer_size);
        if (lds > AMX_LIM_LDS_MAX) return hipErrorInvalidValue;   // B <= 6741: 5 ms up to ~670 kHz
        if (!ls.seg_state || !ls.cnt || ls.buffer_size != buffer_size || ls.max_segs < 1)
            return hipErrorInvalidValue;
        a.seg_frames = ls.seg_frames; a.warm_frames = ls.warm_frames; a.max_segs = ls.max_segs;
        a.warm_cap = ls.warm_cap;
        a.seg_state = ls.seg_state; a.cnt = ls.cnt;
        fa.gen_cols = ls.max_segs < AMX_LIM_MAX_BLOCKS ? ls.max_segs : AMX_LIM_MAX_BLOCKS;
    }
    dim3 g((unsigned)(fa.fast_cols + fa.gen_cols), (unsigned)n_tracks);
    if (g.x == 0) return hipSuccess;
    if (unit) hipLaunchKernelGGL(k_final<true>, g, dim3(AMX_BLOCK), lds, st, fa);
    else hipLaunchKernelGGL(k_final<false>, g, dim3(AMX_BLOCK), lds, st, fa);
    return hipGetLastError();
}

}  // namespace amx
