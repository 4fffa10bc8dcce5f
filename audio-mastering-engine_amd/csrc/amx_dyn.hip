// amx_dyn.hip -- multiband compressor dynamics (pydub compress_dynamic_range,
// audio_mastering_engine.py:306-308) and the overlay (:309).
//
// Per band b and frame i:
//   r_i   = audioop.rms of frames [max(i-look, 0), i)          (exact integer sums)
//   m_i   = (1 - 1/ratio) * max(20 log10(r_i / thr), 0)        (host tables, C libm)
//   att  <- (r_i > thr and att <= m_i) ? min(att + m_i/A, m_i) : max(att - m_i/R, 0)
//   out_i = audioop.mul(frame_i, 10^(-att/20))   if att != 0
//
// r is embarrassingly parallel (k_rms: block prefix sums).  It is stored as the u16
// table index r (m = mt[r] is a host table of C-libm values: 2 B per frame instead of
// the 8 B of m, read ~5 times per step); the readers gather m from the table, with
// lanes laid over consecutive frames so a gather touches few table lines.  The envelope is a
// sequential nonlinear recurrence; it is parallelised by exact speculation:
//   k_env0: every envelope segment of Le frames runs from att = 0 started W frames
//     earlier (the trajectories of this recurrence coincide after clamp events, so
//     the warm-up usually lands exactly on the true state) and writes its start guess
//     s_j, end state e_j, an over-threshold flag and a checkpoint every 16 frames;
//   k_envheads / k_envchain: segment j's true start is the end of segment j - 1 (0 at
//     a chunk's start).  A segment whose stored start differs while its predecessor's
//     holds heads a chain; one wave per chain re-runs the head from the true start,
//     rewriting checkpoints until the new state meets a stored one (the trajectories
//     have coincided), and walks on while the next segment's start is now wrong;
//   k_envseq: a final in-order walk per (chunk, band) fixes whatever is still
//     inconsistent, so the result is exact whatever the signal;
//   k_gain_overlay: every frame's attenuation from the checkpoint before it, the
//     gain, and the 3-band overlay.
// Every value is produced by the reference's own operation sequence from the true
// start state, so the envelope is bit-exact, not approximate.
#include "amx_dev.hpp"

namespace amx {

// clang vector types (HIP's double2 / uint4 structs defeat register promotion of arrays)
typedef double d2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

#define AMX_TAB 32769

// ----------------------------------------- compressor RMS detector (exact)
// One workgroup = AMX_RMS_N - LP frames of one (chunk, band); squares of the window
// [base - LP, base + AMX_RMS_N - LP) are prefix-summed in LDS (exact int64), so
// S_i = P(i) - P(i - look) with no sequential sliding window; LP is the smallest of
// 256 / 512 / 1024 frames >= look (5 ms: 220 / 240 / 480 at 44.1 / 48 / 96 kHz), so the
// halo re-read is 6-14 % and the 33 KB of prefix sums leave room for 4 workgroups per CU.
// Frames before the chunk count as 0 (audioop.rms over the shorter window divides by
// the frames present).  Loads are 16-B vectors (the LDS origin is 16-frame aligned);
// the output is r_i itself (u16, clamped to 32768 = |sample| max), m is not formed here.
#define AMX_RMS_N 4096
#define AMX_RMS_MAXLOOK 1024

// LDS index of prefix slot k: one spare slot per 16 keeps the scan's stores (lane
// stride 17 slots, odd) on distinct bank pairs
__device__ __forceinline__ int rms_slot(int k) { return k + (k >> 4); }

// audioop.rms's (unsigned) sqrt((double) S / cnt), S = the window's exact sum of
// squares (< 2^53, so the reference's double sum is exact), cnt the samples present.
// That value is max{k : k^2 cnt <= S}: with S, cnt integers, S/cnt just below k^2 is
// at least 1/cnt >= 2^-11 below it, far more than the double ulp at k^2 <= 2^30
// (2^-22), so the division cannot round up onto k^2, and then sqrt stays below k
// (by >= 1/(2 k cnt) >> ulp(k)); S/cnt >= k^2 gives sqrt >= k by monotone rounding.
// So a float estimate (within 0.01 of sqrt(S/cnt)) corrected by one exact integer test
// gives the same r without the double division and square root.  rc ~ 1/cnt.
__device__ __forceinline__ uint32_t rms_floor(uint64_t S, uint32_t cnt, double rc) {
    // S < 2^44 and k^2 cnt < 2^53: the double forms below are exact integers
    const double sd = fma((double)(uint32_t)(S >> 32), 4294967296.0, (double)(uint32_t)S);
    const double cd = (double)cnt;
    const uint32_t k = (uint32_t)__builtin_amdgcn_sqrtf((float)(sd * rc));
    const uint32_t k1 = k + 1;
    const bool up = (double)__umul24(k1, k1) * cd <= sd;
    const bool down = (double)__umul24(k, k) * cd > sd;
    const uint32_t r = k + (uint32_t)up - (uint32_t)(down & !up);
    return cnt ? (r > 32768u ? 32768u : r) : 0u;
}

// AMX_RMS_N256: the tile of the LP = 256 form (48 / 44.1 kHz).  Measured (round 6,
// profiles/r06m_rms_analog_ab.txt): 2048 frames (17 KB of prefix sums, 8 workgroups per
// CU, 12.5 % halo) 1-2 us slower at C3 than 4096 (4 per CU, 6 % halo)
#ifndef AMX_RMS_N256
#define AMX_RMS_N256 4096
#endif
template <int LP, int N>
__global__ void __launch_bounds__(AMX_BLOCK) k_rms(const ChainDev *__restrict__ cdp,
                                                   const ChunkDev *__restrict__ chunks,
                                                   const uint32_t *__restrict__ bands,
                                                   uint16_t *__restrict__ mi, int64_t nloc,
                                                   int *bact) {
    constexpr int F = N - LP;                          // frames out per workgroup
    constexpr int PER = N / AMX_BLOCK;                 // 16 slots per thread
    constexpr int VEC = PER / 4;                       // as 4 16-B loads
    static_assert(F % AMX_BLOCK == 0 && PER % 4 == 0, "tile shape");
    __shared__ unsigned long long P[N + N / 16];
    __shared__ unsigned long long wsum[AMX_BLOCK / 64];
    const int look = cdp->look;
    const int c = blockIdx.y, b = blockIdx.z;
    const ChunkDev ch = chunks[c];
    const int64_t base = (int64_t)blockIdx.x * F;
    if (base >= ch.n) return;                          // block-uniform
    const uint32_t *x = bands + b * nloc + ch.loc_off;
    uint16_t *mo = mi + b * nloc + ch.loc_off;
    const int64_t rowlen = (ch.n + 15) / 16 * 16;     // the chunk row (16-frame aligned)
    // LDS slot k holds frame base - LP + k
    const int64_t f0 = base - LP;
    const int t = threadIdx.x;
    // a0^2 + a1^2 <= 2^31: one frame's squares fit a u32
    uint32_t v[PER];
    if (f0 >= 0 && f0 + N <= ch.n) {                   // block-uniform: no frame masks
#pragma unroll
        for (int q = 0; q < VEC; q++) {
            const u4v u = *reinterpret_cast<const u4v *>(x + f0 + t * PER + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int32_t a0 = lo16(u[e]), a1 = hi16(u[e]);
                v[4 * q + e] = (uint32_t)(a0 * a0) + (uint32_t)(a1 * a1);
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < VEC; q++) {
            const int64_t f = f0 + t * PER + 4 * q;
            const bool ok = f >= 0 && f < rowlen;
            const u4v u = *reinterpret_cast<const u4v *>(x + (ok ? f : 0));
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int32_t a0 = lo16(u[e]), a1 = hi16(u[e]);
                v[4 * q + e] = (ok && f + e < ch.n) ? (uint32_t)(a0 * a0) + (uint32_t)(a1 * a1) : 0u;
            }
        }
    }
    // block inclusive scan: per-thread total, wave scan of totals, cross-wave
    unsigned long long run = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) run += v[q];
    unsigned long long incl = run;
    const int lane = t & 63, w = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long up = __shfl_up(incl, o);
        if (lane >= o) incl += up;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    unsigned long long p = incl - run;
    for (int q = 0; q < w; q++) p += wsum[q];
    const int s0 = rms_slot(t * PER);                  // the thread's 16 slots share one pad
#pragma unroll
    for (int q = 0; q < PER; q++) { p += v[q]; P[s0 + q] = p; }
    __syncthreads();
    // frame i = base + nn uses slots [nn + LP - look, nn + LP)
    constexpr int OUT = F / AMX_BLOCK;
    const uint32_t cfull = 2u * (uint32_t)look;
    const double rfull = 1.0 / (double)cfull;
    const bool whole = base >= look && base + F <= ch.n;   // block-uniform
    auto rms_at = [&](int k) -> uint32_t {
        const uint32_t nn = (uint32_t)t + (uint32_t)k * AMX_BLOCK;
        const uint32_t e1 = nn + (LP - 1), e0 = e1 - (uint32_t)look;
        const uint64_t S = P[e1 + (e1 >> 4)] - P[e0 + (e0 >> 4)];
        if (whole) return rms_floor(S, cfull, rfull);
        const int64_t i = base + nn;
        const bool head = i < look;                    // a chunk's first look frames
        const uint32_t cnt = head ? 2u * (uint32_t)i : cfull;
        return rms_floor(S, cnt, head ? 1.0 / (double)cnt : rfull);
    };
    // band activity: a frame whose m may be nonzero (r >= rq; every r below rq has m = 0)
    const uint32_t rq = (uint32_t)cdp->rq[b];
    bool hot = false;
    if (whole) {
#pragma unroll
        for (int k = 0; k < OUT; k++) {
            const uint32_t rms = rms_at(k);
            hot |= rms >= rq;
            mo[base + t + k * AMX_BLOCK] = (uint16_t)rms;
        }
    } else {
#pragma unroll
        for (int k = 0; k < OUT; k++) {
            const int64_t i = base + t + k * AMX_BLOCK;
            const uint32_t rms = rms_at(k);
            hot |= i < ch.n && rms >= rq;
            // the row's tail past the chunk (to the 16-frame boundary) gets r = 0, m = 0:
            // k_env0 feeds a chunk's partial last tile without masking
            if (i < rowlen) mo[i] = i < ch.n ? (uint16_t)rms : (uint16_t)0;
        }
    }
    // one word per band, cleared by k_xover2; set once (read first, so the later
    // workgroups of an active band do not all store to the one line)
    if (__syncthreads_or(hot) && t == 0 && bact[b] == 0) bact[b] = 1;
}

// m of table index r.  Rows hold r only where a chunk has frames: the padding and a
// row's tail past the chunk hold anything, and are clamped into the table (their m is
// never used)
__device__ __forceinline__ double m_of(const double *__restrict__ mt, uint32_t r) {
    return mt[r < 32768u ? r : 32768u];
}

// --------------------------------------------------------- envelope helpers
// The step needs only m: over-threshold <=> m != 0 for the reference's arithmetic
// (m != 0 needs 20 log10(r/thr) > 0, i.e. r > thr; and when m == 0 both branches
// return att unchanged: min(att + 0, 0) = 0 = att when att <= 0, max(att - 0, 0)
// = att otherwise), so frames below the threshold -- and frames outside a chunk,
// fed as m = 0 -- hold the state.

// inc = m / A, dec = m / R exactly as IEEE division (pydub): with RCP the quotient
// is formed as q = m (1/A) corrected by one FMA residual step -- the same correctly
// rounded value (Markstein), checked on the host for every table m (ChainDev::env_rcp)
template <bool RCP>
__device__ __forceinline__ double env_div(double m, double a, double ra) {
    if constexpr (RCP) {
        const double q = m * ra;
        return fma(fma(-q, a, m), ra, q);
    } else {
        return m / a;
    }
}

// v_min_f64 without the operand canonicalisation the compiler adds for fmin (IEEE
// mode quiets signalling NaNs; m is a table value, never a NaN): the instruction fmin
// compiles to, one fp64 operation per frame fewer
__device__ __forceinline__ double min_f64_raw(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// pydub envelope step, exact, branch-free (both candidates, then select): attenuation
// += inc, min(., max_att) or attenuation -= dec, max(., 0).  The reference's condition
// is (over and att <= m); over can be dropped: when m == 0 (not over) and att == 0 the
// attack branch gives min(0 + 0, 0) = 0 = att, and att > 0 takes the release branch
// anyway.  Every envelope kernel uses it (k_env0, the re-runs, k_gain_overlay).
__device__ __forceinline__ double env_step3(double att, double m, double inc, double dec) {
    const double up = min_f64_raw(att + inc, m);
    const double dn = fmax(att - dec, 0.0);
    return att <= m ? up : dn;
}

template <bool RCP>
__device__ __forceinline__ double env_step(const ChainDev &cd, double att, double m) {
    return env_step3(att, m, env_div<RCP>(m, cd.env_A, cd.env_rA), env_div<RCP>(m, cd.env_R, cd.env_rR));
}

// audioop.mul: floor(fbound(v * f)) (CPython Modules/audioop.c), the clamp to
// [-32768, 32767] included.  The compressor's factor is 0 <= f <= 1 (10^(-att/20), att
// >= 0; exp10_gain gives exactly 1 at 0 and never rounds above it), so for an int16 v the
// product already lies in [-32768, 32767] and the clamp never acts: floor alone.
__device__ __forceinline__ int mul16(int v, double f) {
    return (int)floor((double)v * f);
}

// 10^x for the gain: ROCm device-libs' exp10 (ocml) operation for operation --
// k = rint(x log2 10), r = x - k log10 2 (two-part), u = r ln 10 (two-part),
// e^u by a degree-11 polynomial, scaled by 2^k -- so the values are those the
// library gives; written out here so the constants are scalar operands of the
// FMAs.  The library's overflow / underflow selects are left out: x = -att/20 is
// finite and <= 0, and 2^k underflows to 0 by itself for very negative x.
__device__ __forceinline__ double exp10_gain(const double *__restrict__ E, double x) {
    const double k = rint(x * E[0]);
    double r = fma(E[1], k, x);
    r = fma(E[2], k, r);
    double u = r * E[3];
    u = fma(E[4], r, u);
    double p = fma(E[5], u, E[6]);
#pragma unroll
    for (int i = 7; i < 15; i++) p = fma(u, p, E[i]);
    p = fma(u, p, 1.0);
    p = fma(u, p, 1.0);
    return ldexp(p, (int)k);
}

// the gained frame for attenuation att (:306-308 output, audioop.mul).
// att == 0 is the reference's "no change"; exp10(-0/20) == 1 and mul16(v, 1) == v,
// so the branch-free form gives the same frame and keeps lanes converged.
// -att / 20 is the IEEE quotient, formed by reciprocal multiply + one FMA residual
// step (Markstein: exact for a correctly rounded 1/20; tests/test_host.py checks it
// against division on random attenuations).
__device__ __forceinline__ double gain_factor(const ChainDev &cd, double att) {
    const double q = -att * cd.exc[15];
    return exp10_gain(cd.exc, fma(fma(-q, 20.0, -att), cd.exc[15], q));
}

__device__ __forceinline__ uint32_t gain_apply(uint32_t v, double f) {
    return pack2((int16_t)mul16(lo16(v), f), (int16_t)mul16(hi16(v), f));
}

__device__ __forceinline__ uint32_t gain_frame(const ChainDev &cd, uint32_t v, double att) {
    return gain_apply(v, gain_factor(cd, att));
}

#define AMX_ENV_TF_ 16   // checkpoint spacing (frames)

// lane i's value of a double, as a wave-uniform (scalar) operand
__device__ __forceinline__ double lane_val(double v, int i) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)x, i);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), i);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Wave-cooperative re-run of one segment's frames [f0, f1) (chunk-local; f0 a
// multiple of 16) from the new start ns: every lane of the wave calls it with the
// same arguments.  Per 64-frame window each lane loads one frame's m and forms its
// inc = m / A and dec = m / R (coalesced; the next window's loads are in flight
// meanwhile) and stores the three into LDS; the recurrence -- a chain of dependent
// steps, the same on every lane -- then reads them 16 frames at a time as broadcast
// LDS loads issued ahead of the chain, so a step is just its dependent min / max /
// select (C5 made this chain the fix-up's critical path: runs of ~60 consecutive
// mis-speculated segments in one wave, each re-run after the previous one).  Lanes
// 0, 16, 32, 48 keep the new state before their frame and rewrite that checkpoint.
// The stored checkpoints are the trajectory from the old start, so at every 16-frame
// boundary the new state is compared with the stored one: once they are equal the two
// trajectories are identical from there on, the remaining checkpoints stand and the
// old end is the end.  Returns the segment's end state.
template <bool RCP>
__device__ double env_rerun_wave(const ChainDev &cd, const uint16_t *m, const double *mt, double *ckr,
                                 int64_t f0, int64_t f1, double ns, double old_end) {
    __shared__ __attribute__((aligned(16))) double s_m[64], s_i[64], s_d[64];
    const int lane = threadIdx.x & 63;
    const bool ckl = (lane & (AMX_ENV_TF_ - 1)) == 0;
    double c = ns;
    // the loads run ahead of the chain: r indices three windows ahead, their table
    // gathers (and the stored checkpoints) two, so a window's dependent index -> table
    // load pair is never waited for (one window ahead left ~2 load latencies per
    // window exposed against ~0.5 us of steps)
    auto ridx = [&](int64_t f) -> uint32_t { return f < f1 ? (uint32_t)m[f] : 0xffffffffu; };
    auto gath = [&](uint32_t r) -> double { return r == 0xffffffffu ? 0.0 : m_of(mt, r); };
    auto ckld = [&](int64_t f) -> double { return ckl && f < f1 ? ckr[f / AMX_ENV_TF_] : 0.0; };
    double ml = gath(ridx(f0 + lane));
    uint32_t ib = ridx(f0 + 128 + lane);
    double m1 = gath(ridx(f0 + 64 + lane));
    double ol = ckld(f0 + lane), o1 = ckld(f0 + 64 + lane);
    for (int64_t base = f0; base < f1; base += 64) {
        const uint32_t ic = ridx(base + 192 + lane);
        const double m2 = gath(ib);
        const double o2 = ckld(base + 128 + lane);
        s_m[lane] = ml;
        s_i[lane] = env_div<RCP>(ml, cd.env_A, cd.env_rA);
        s_d[lane] = env_div<RCP>(ml, cd.env_R, cd.env_rR);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        double mine = c;
        int stop = 4;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            double mv[16], iv[16], dv[16];
#pragma unroll
            for (int q = 0; q < 16; q += 2) {
                const d2v a = *reinterpret_cast<const d2v *>(s_m + 16 * t + q);
                const d2v b = *reinterpret_cast<const d2v *>(s_i + 16 * t + q);
                const d2v d = *reinterpret_cast<const d2v *>(s_d + 16 * t + q);
                mv[q] = a.x; mv[q + 1] = a.y;
                iv[q] = b.x; iv[q + 1] = b.y;
                dv[q] = d.x; dv[q + 1] = d.y;
            }
            const bool same = base + 16 * t < f1 && c == lane_val(ol, 16 * t);
            if (__builtin_amdgcn_readfirstlane((int)same)) { stop = t; break; }
            mine = lane == 16 * t ? c : mine;            // state before frame base + 16 t
#pragma unroll
            for (int q = 0; q < 16; q++) c = env_step3(c, mv[q], iv[q], dv[q]);
        }
        __builtin_amdgcn_wave_barrier();                  // LDS reads done before the next writes
        if (ckl && (lane >> 4) < stop && base + lane < f1) ckr[(base + lane) / AMX_ENV_TF_] = mine;
        if (stop < 4) return old_end;
        ml = m1;
        m1 = m2;
        ib = ic;
        ol = o1;
        o1 = o2;
    }
    return c;
}

// ------------------------------------------------------- round 0: speculation
// One lane per (envelope segment, band), a wave (= workgroup) per 64 consecutive
// segments.  Each lane runs the attenuation recurrence over its segment from
// att = 0 started W frames earlier (the warm-up: after a clamp event the trajectory
// no longer depends on the start) and records its start guess s_j
// (the state when its first frame begins), end state e_j, whether it has an
// over-threshold frame, and a checkpoint -- the state before every 16th frame of
// the chunk -- from which k_gain_overlay re-derives every frame's attenuation in
// parallel.  No gains are computed here: this is the latency-bound sequential
// part, kept to ~16 fp64 operations per frame.
// Frames move in 16-frame tiles.  A lane's tile is one 32-B row of r (64 rows per
// wave); the wave loads the 64 rows cooperatively -- lane l moves 8-B piece l % 4 of
// rows 16 i + l / 4 -- gathers m = mt[r] for the four frames of each piece (the four
// lanes of a row gather neighbouring entries: slowly varying r, few table lines per
// gather) and stages m in LDS (padded rows, conflict-free b128 reads).  The r loads
// run AMX_ENV_PF tiles ahead and the gathers 2 tiles ahead of the tile being computed
// (one tile is ~16 dependent steps, shorter than a miss to HBM).  Per tile the 16
// quotient pairs and the recurrence are one scheduling region.  (The recurrence's
// dependences do not set the time: with them removed the kernel took the same time;
// DESIGN.md §3.4.)  Frames before the chunk or
// after the segment are fed as m = 0 (state held); the buffer is padded so those rows
// read in bounds.  W and Le are multiples of 16 AMX_ENV_PF and chunk rows start
// 16-frame aligned, so the warm-up / main boundary is tile-uniform, every vector is
// aligned and checkpoints fall on tile starts.
// The bands k_rms found active (a frame over the threshold) and the segment table of
// their count (ChainDev::etab).  An inactive band has m = 0 on every frame, so its
// attenuation stays at the chunk start's 0 throughout: the envelope kernels skip it
// and k_gain_overlay passes it through unread.  Slot s (k_env0's blockIdx.y) runs the
// s-th active band, so t active bands share the CUs.
struct EnvBands {
    int mask;                    // bit b: band b active (wave-uniform)
    int nb;
    __device__ __forceinline__ bool act(int b) const { return (mask >> b) & 1; }
};
__device__ __forceinline__ EnvBands env_bands(const int *bact) {
    EnvBands e;
    e.mask = 0;
#pragma unroll
    for (int b = 0; b < 3; b++) e.mask |= (__builtin_amdgcn_readfirstlane(bact[b]) != 0) << b;
    e.nb = __builtin_popcount(e.mask);
    return e;
}
// the band of slot s: the position of the (s + 1)-th set bit of the mask
__device__ __forceinline__ int env_slot_band(const EnvBands &e, int s) {
    int m = e.mask;
    for (int k = 0; k < s; k++) m &= m - 1;
    return __builtin_ctz(m | 8);
}

#define AMX_ENV_TF 16
#define AMX_ENV_MP 18      // m tile pitch in doubles (144 B)
#define AMX_ENV_PF 8       // r tiles in flight

typedef uint32_t u2v __attribute__((ext_vector_type(2)));

// m of one staged piece (4 frames: r in the 4 u16 of v).  No clamp: an index is a u16
// (<= 65535) and a band's three tables (m, m/A, m/R: 3 x 32769 entries) lie behind mt,
// so every index reads in bounds; indices above 32768 occur only in rows k_rms did not
// write (padding before a chunk, past a segment), whose tiles k_env0 skips
__device__ __forceinline__ void env_gather(const double *__restrict__ mt, const u2v (&I)[4],
                                           double (&G)[16]) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const uint32_t r = (I[i][e >> 1] >> (16 * (e & 1))) & 0xffffu;
            G[4 * i + e] = mt[r];
        }
    }
}

template <bool RCP>
__device__ __forceinline__ void env0_tile(const ChainDev &cd, double *sm, double (&G)[16],
                                          u2v (&Islot)[4], const u2v (&Inext)[4],
                                          const uint16_t *const (&irow)[4], const double *mt, int q,
                                          int ntile, int nwarm, int64_t start, int64_t end,
                                          double *ckr, double &att, double &s_spec, bool &any) {
    const int lane = threadIdx.x & 63;
    // stage tile q's m (gathered two tiles ago)
#pragma unroll
    for (int i = 0; i < 4; i++) {
        double *d = sm + ((lane >> 2) + 16 * i) * AMX_ENV_MP + 4 * (lane & 3);
        *reinterpret_cast<d2v *>(d) = d2v{G[4 * i], G[4 * i + 1]};
        *reinterpret_cast<d2v *>(d + 2) = d2v{G[4 * i + 2], G[4 * i + 3]};
    }
    __builtin_amdgcn_wave_barrier();
    {
        // this ring slot (tile q's r, gathered already) takes tile q + PF (past the
        // end: re-read, unused); then the gathers of tile q + 2
        const int qn = (q + AMX_ENV_PF < ntile ? q + AMX_ENV_PF : q) * AMX_ENV_TF;
#pragma unroll
        for (int i = 0; i < 4; i++) Islot[i] = *reinterpret_cast<const u2v *>(irow[i] + qn);
        env_gather(mt, Inext, G);
    }
    const int64_t f0 = start + (int64_t)q * AMX_ENV_TF;
    const bool in = f0 >= 0 && f0 < end;           // whole tile in (else held)
    double mv[AMX_ENV_TF];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const d2v v = *reinterpret_cast<const d2v *>(sm + lane * AMX_ENV_MP + 2 * i);
        mv[2 * i] = v.x;
        mv[2 * i + 1] = v.y;
    }
    __builtin_amdgcn_wave_barrier();
    if (q == nwarm) s_spec = att;
    // a tile outside the chunk / segment holds the state: it is skipped rather than
    // fed zeros (the same state; no per-frame selects on the common path)
    if (in) {
        // (the partial last tile of a chunk-final segment reads r = 0 past the chunk:
        // the state is held there without masking, k_rms)
        if (q >= nwarm) {
            ckr[f0 / AMX_ENV_TF] = att;
            // any m != 0 in the tile: the OR of the 16 values' bits, sign masked (-0.0 is
            // a zero m); integer ORs instead of a fp64 compare per frame
            uint32_t h = 0, l = 0;
#pragma unroll
            for (int f = 0; f < AMX_ENV_TF; f++) {
                const unsigned long long x = (unsigned long long)__double_as_longlong(mv[f]);
                h |= (uint32_t)(x >> 32);
                l |= (uint32_t)x;
            }
            any |= ((h & 0x7fffffffu) | l) != 0u;
        }
        double iv[AMX_ENV_TF], dv[AMX_ENV_TF];
#pragma unroll
        for (int f = 0; f < AMX_ENV_TF; f++) {
            iv[f] = env_div<RCP>(mv[f], cd.env_A, cd.env_rA);
            dv[f] = env_div<RCP>(mv[f], cd.env_R, cd.env_rR);
        }
        // (no scheduling barrier: the scheduler may start the recurrence while later
        // quotients are still being formed; measured 206 -> 201 us at C3)
#pragma unroll
        for (int f = 0; f < AMX_ENV_TF; f++) att = env_step3(att, mv[f], iv[f], dv[f]);
    }
}

// Launch: W = 1, 2 or 4 waves per workgroup (a workgroup's waves go to
// distinct SIMDs) of one band, with enough dynamic LDS that a CU holds one workgroup,
// and no more workgroups than CUs.  The plan picks Le so that all segments fit one
// resident wave set.  What caps a CU is its memory pipeline, not the step's fp64
// arithmetic (scripts/env_mb.hip, profiles/r04_env_mb.txt): each wave-frame's m gather
// refills L1 lines of the 256 KB table from L2 (~55 CU cycles) beside the LDS staging
// (~45), while the step costs ~62 cycles of its own SIMD; a CU holding more waves, or
// band-interleaved waves, does not step more frames.
#define AMX_ENV_WG 4
#define AMX_ENV_LDS_PIN (48 * 1024)      // + 36 KB static: > 80 KB, one workgroup per CU
template <bool RCP>
__global__ void __launch_bounds__(64 * AMX_ENV_WG) k_env0(const ChainDev *__restrict__ cdp,
                                             const ChunkDev *__restrict__ chunks,
                                             const SegDev *__restrict__ es, int n_es,
                                             const uint16_t *__restrict__ mi,
                                             const double *__restrict__ tabs,
                                             double *__restrict__ ck,
                                             double *__restrict__ sv, double *__restrict__ ev,
                                             int *__restrict__ act, int64_t nloc, int warm,
                                             int *__restrict__ flags) {
    __shared__ __attribute__((aligned(16))) double sm_all[AMX_ENV_WG][64 * AMX_ENV_MP];
    const ChainDev &cd = *cdp;
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    double *sm = sm_all[wv];
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < AMX_ENV_MAX_ROUNDS) flags[threadIdx.x] = 0;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) {
        for (int k = lane; k < AMX_ENV_MAX_ROUNDS * AMX_ENV_NCTR; k += 64) flags[AMX_ENV_MAX_ROUNDS + k] = 0;
        if (lane < 3) flags[AMX_ENV_LIST + lane] = 0;   // the two lists' lengths, k_envseq's flag
    }
    const EnvBands eb = env_bands(flags + AMX_ENV_BACT);
    if ((int)blockIdx.y >= eb.nb) return;                 // workgroup-uniform
    const int b = env_slot_band(eb, blockIdx.y);
    es += cd.etab[eb.nb].es_off;
    n_es = cd.etab[eb.nb].n_es;
    const int Le = cd.etab[eb.nb].Le, ld = cd.es_ld;
    if ((int)(blockIdx.x * (blockDim.x >> 6)) * 64 >= n_es) return;
    const int j = (blockIdx.x * (blockDim.x >> 6) + wv) * 64 + lane;
    const bool valid = j < n_es;
    const SegDev sg = es[valid ? j : n_es - 1];
    const ChunkDev ch = chunks[sg.chunk];
    const int64_t rowoff = b * nloc + ch.loc_off;       // this lane's chunk row
    const int64_t start = sg.pos - warm;                // frame of step 0 (may be < 0)
    const int64_t end = valid ? sg.pos + sg.len : sg.pos;
    double *ckr = ck + rowoff / AMX_ENV_TF;             // checkpoint k: before frame 16 k
    const double *mt = tabs + (int64_t)b * 3 * AMX_TAB;
    const int ntile = (warm + Le) / AMX_ENV_TF, nwarm = warm / AMX_ENV_TF;
    const uint16_t *irow[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int r = 16 * i + (lane >> 2);
        irow[i] = mi + __shfl(rowoff + start, r) + 4 * (lane & 3);
    }
    u2v I[AMX_ENV_PF][4];
#pragma unroll
    for (int u = 0; u < AMX_ENV_PF; u++)
#pragma unroll
        for (int i = 0; i < 4; i++) I[u][i] = *reinterpret_cast<const u2v *>(irow[i] + u * AMX_ENV_TF);
    double G[2][16];
    env_gather(mt, I[0], G[0]);
    env_gather(mt, I[1], G[1]);
    // the warm-up's start guess: a chunk's first frames start from 0 (exact: the
    // reference starts every chunk there); elsewhere m of the warm-up's first frame --
    // inside a compressed stretch the state sits at or near m, and trajectories meet
    // sooner from there than from 0 (scripts/env_warm_sim.py)
    double att = 0.0, s_spec = 0.0;
    if (cd.env_guess && start >= 0) att = mt[mi[rowoff + start]];
    bool any = false;
    for (int q0 = 0; q0 < ntile; q0 += AMX_ENV_PF) {
#pragma unroll
        for (int u = 0; u < AMX_ENV_PF; u++)
            env0_tile<RCP>(cd, sm, G[u & 1], I[u], I[(u + 2) % AMX_ENV_PF], irow, mt,
                           q0 + u, ntile, nwarm, start, end, ckr, att, s_spec, any);
    }
    if (valid) {
        sv[(int64_t)b * ld + j] = s_spec;
        ev[(int64_t)b * ld + j] = att;
        act[(int64_t)b * ld + j] = any ? 1 : 0;
    }
}

// the wave fixes segment [pos, pos + len) of a chunk row from the new start ns (all
// lanes, uniform arguments); returns the segment's end state
template <bool RCP>
__device__ __forceinline__ double env_fix_segment(const ChainDev &cd, const uint16_t *mrow,
                                                  const double *mt, double *ckr, int64_t pos, int len,
                                                  bool active, double ns, double old_end) {
    if (!active) {
        // identity transfer: the held state is every checkpoint of the segment
        const int64_t k0 = pos / AMX_ENV_TF_, k1 = (pos + len + AMX_ENV_TF_ - 1) / AMX_ENV_TF_;
        for (int64_t k = k0 + (threadIdx.x & 63); k < k1; k += 64) ckr[k] = ns;
        return ns;
    }
    return env_rerun_wave<RCP>(cd, mrow, mt, ckr, pos, pos + len, ns, old_end);
}

// ------------------------------------------------ parallel fix-up: chains
// The link j - 1 -> j holds when segment j's stored start equals segment j - 1's stored
// end (a chunk's first segment: 0, where every chunk starts).  k_env0's speculation
// breaks few links.  A segment whose link is broken while its predecessor's link holds
// is a chain head: its predecessor is exact, so its true start is known.  k_envheads
// marks the heads and lists them (one atomicAdd per wave); k_envchain gives each head
// its own wave (a fixed grid looping over the list).  The wave re-runs the head from
// the true start (env_fix_segment: an inactive segment only takes the held state) and
// walks on to the next segment while that one's stored start differs from the new
// end (runs of inactive segments, which hold the state, 64 at a time).  It stops at
// the chunk's end, at a link that holds, or at another head, which has its own wave.  A head's wave may have read its predecessor's end before another
// chain rewrote it; the walker that reaches such a head with a changed end sets a flag,
// and k_envseq then checks every link in order.  Independent chains run in parallel
// (round 4's k_envfix re-ran all of a 64-segment wave's segments in turn).
// Before the chains, one optimistic parallel pass (k_envneed + k_envwide): every
// segment whose start differs from the end of its nearest earlier active segment
// (below-threshold segments hold the state, so that end is its true start) is listed
// and re-run at once by its own wave from that end as it stands.  Most such re-runs are
// independent (C4: 254 in a step, at most 2 in a row), and a re-run whose trajectory
// meets the old one keeps the old end exact; the chains then fix only the links that
// are still broken.
template <bool RCP>
__global__ void __launch_bounds__(64) k_envneed(const ChainDev *__restrict__ cdp,
                                                const SegDev *__restrict__ es, int n_es,
                                                const double *__restrict__ sv,
                                                const double *__restrict__ ev,
                                                const int *__restrict__ act, int *flags,
                                                int *__restrict__ prev, int *__restrict__ list) {
    const ChainDev &cd = *cdp;
    const int b = blockIdx.y, lane = threadIdx.x;
    const EnvBands eb = env_bands(flags + AMX_ENV_BACT);
    if (!eb.act(b)) return;
    es += cd.etab[eb.nb].es_off;
    n_es = cd.etab[eb.nb].n_es;
    const int w0 = blockIdx.x * 64;
    if (w0 >= n_es) return;
    const int j = w0 + lane;
    const bool valid = j < n_es;
    const int64_t bo = (int64_t)b * cd.es_ld;
    const SegDev sg = es[valid ? j : n_es - 1];
    const bool a = valid && act[bo + j] != 0;
    // p: the nearest earlier active segment of the chunk (a ballot in the wave, then a
    // wave-uniform look-back over earlier segments for the lanes that have none here)
    const unsigned long long am = __ballot(a);
    const unsigned long long below = lane ? am & (~0ull >> (64 - lane)) : 0ull;
    int p = below ? w0 + 63 - __clzll((long long)below) : -1;
    if (p < sg.first) p = -1;
    const bool lb = valid && p < 0 && sg.first < w0;
    if (__ballot(lb)) {
        const int first0 = __shfl(sg.first, 0);
        int last = -1;
        for (int base = w0 - 64; base + 63 >= first0; base -= 64) {
            const int jj = base + lane;
            const unsigned long long mk = __ballot(jj >= first0 && act[bo + jj] != 0);
            if (mk) { last = base + 63 - __clzll((long long)mk); break; }
        }
        if (lb) p = last;
    }
    bool need = false;
    if (valid) {
        prev[bo + j] = p;
        need = !((p >= 0 ? ev[bo + p] : 0.0) == sv[bo + j]);
    }
    const unsigned long long nm = __ballot(need);
    if (nm) {
        int base = 0;
        if (lane == 0) base = atomicAdd(flags + AMX_ENV_LIST, __popcll(nm));
        base = __shfl(base, 0);
        const unsigned long long lt = lane ? ~0ull >> (64 - lane) : 0ull;
        if (need) list[base + __popcll(nm & lt)] = (int)(bo + j);
    }
}

template <bool RCP>
__global__ void __launch_bounds__(64) k_envwide(const ChainDev *__restrict__ cdp,
                                                const ChunkDev *__restrict__ chunks,
                                                const SegDev *__restrict__ es,
                                                const uint16_t *__restrict__ mm,
                                                const double *__restrict__ tabs,
                                                double *__restrict__ ck, double *sv, double *ev,
                                                const int *__restrict__ act, int *flags,
                                                const int *__restrict__ prev,
                                                const int *__restrict__ list, int64_t nloc) {
    const int count = __builtin_amdgcn_readfirstlane(flags[AMX_ENV_LIST]);
    if (blockIdx.x == 0 && threadIdx.x == 0) flags[AMX_ENV_MAX_ROUNDS + 3] = count;   // (amx_env_counters)
    if ((int)blockIdx.x >= count) return;
    const ChainDev &cd = *cdp;
    const int lane = threadIdx.x;
    const EnvBands eb = env_bands(flags + AMX_ENV_BACT);
    const SegDev *et = es + cd.etab[eb.nb].es_off;
    const int ld = cd.es_ld;
    for (int i = blockIdx.x; i < count; i += gridDim.x) {
        const int k = __builtin_amdgcn_readfirstlane(list[i]);
        const int b = k / ld, j = k - b * ld;
        const int64_t bo = (int64_t)b * ld;
        const SegDev sg = et[j];
        const int p = prev[bo + j];
        const double ns = p >= 0 ? ev[bo + p] : 0.0;
        const int64_t ro = b * nloc + chunks[sg.chunk].loc_off;
        const double r = env_fix_segment<RCP>(cd, mm + ro, tabs + (int64_t)b * 3 * AMX_TAB, ck + ro / AMX_ENV_TF_,
                                              sg.pos, sg.len, act[bo + j] != 0, ns, ev[bo + j]);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            sv[bo + j] = ns;
            ev[bo + j] = r;
        }
    }
}

#ifndef AMX_ENV_CHAIN_WAVES
#define AMX_ENV_CHAIN_WAVES 2048    // k_envchain grid (waves loop over the head list)
#endif
template <bool RCP>
__global__ void __launch_bounds__(64) k_envheads(const ChainDev *__restrict__ cdp,
                                                 const SegDev *__restrict__ es, int n_es,
                                                 const double *__restrict__ sv,
                                                 const double *__restrict__ ev,
                                                 int *flags, int *__restrict__ list,
                                                 int *__restrict__ hmark) {
    const ChainDev &cd = *cdp;
    const int b = blockIdx.y, lane = threadIdx.x;
    const EnvBands eb = env_bands(flags + AMX_ENV_BACT);
    if (!eb.act(b)) return;
    es += cd.etab[eb.nb].es_off;
    n_es = cd.etab[eb.nb].n_es;
    if ((int)blockIdx.x * 64 >= n_es) return;
    const int j = blockIdx.x * 64 + lane;
    const int64_t bo = (int64_t)b * cd.es_ld;
    bool head = false;
    if (j < n_es) {
        const int first = es[j].first;
        const bool need = !(sv[bo + j] == (j == first ? 0.0 : ev[bo + j - 1]));
        bool needp = false;
        if (j > first) needp = !(sv[bo + j - 1] == (j - 1 == first ? 0.0 : ev[bo + j - 2]));
        head = need && !needp;
        hmark[bo + j] = head ? 1 : 0;
    }
    const unsigned long long hm = __ballot(head);
    if (hm) {
        int base = 0;
        if (lane == 0) base = atomicAdd(flags + AMX_ENV_LIST + 1, __popcll(hm));
        base = __shfl(base, 0);
        const unsigned long long below = lane ? hm & (~0ull >> (64 - lane)) : 0ull;
        if (head) list[base + __popcll(below)] = (int)(bo + j);
    }
}

template <bool RCP>
__global__ void __launch_bounds__(64) k_envchain(const ChainDev *__restrict__ cdp,
                                                 const ChunkDev *__restrict__ chunks,
                                                 const SegDev *__restrict__ es,
                                                 const uint16_t *__restrict__ mm,
                                                 const double *__restrict__ tabs,
                                                 double *__restrict__ ck, double *sv, double *ev,
                                                 const int *__restrict__ act, int *flags,
                                                 const int *__restrict__ list,
                                                 const int *__restrict__ hmark, int64_t nloc) {
    const int count = __builtin_amdgcn_readfirstlane(flags[AMX_ENV_LIST + 1]);
    if ((int)blockIdx.x >= count) return;
    const ChainDev &cd = *cdp;
    const int lane = threadIdx.x;
    const EnvBands eb = env_bands(flags + AMX_ENV_BACT);
    const SegDev *et = es + cd.etab[eb.nb].es_off;
    const int ld = cd.es_ld;
    // per-round counters after the round flags (amx_env_counters): segments re-run,
    // the longest walk, chains, 0
    int *ctr = flags + AMX_ENV_MAX_ROUNDS;
    int runs = 0, longest = 0, chains = 0;
    bool stale = false;
    const int n_es = cd.etab[eb.nb].n_es;
    for (int i = blockIdx.x; i < count; i += gridDim.x) {
        const int k = __builtin_amdgcn_readfirstlane(list[i]);
        const int b = k / ld, j = k - b * ld;
        const int64_t bo = (int64_t)b * ld;
        const double *mt = tabs + (int64_t)b * 3 * AMX_TAB;
        SegDev sg = et[j];
        const int64_t ro = b * nloc + chunks[sg.chunk].loc_off;
        double *ckr = ck + ro / AMX_ENV_TF_;
        double state = j == sg.first ? 0.0 : ev[bo + j - 1];
        int cur = j, walked = 0;
        bool done = false;
        while (!done) {
            const bool a = act[bo + cur] != 0;
            double old_end = ev[bo + cur];
            const double r = env_fix_segment<RCP>(cd, mm + ro, mt, ckr, sg.pos, sg.len, a, state, old_end);
            walked++;
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                sv[bo + cur] = state;
                ev[bo + cur] = r;
            }
            if (sg.last) break;                              // the chunk's end
            // the segments after it, 64 at a time: inactive ones whose start is wrong
            // take the held state r in bulk (their checkpoints too); the walk goes on at
            // the first segment that is active, another chain's head, past the chunk,
            // or already starts at r
            int nx = cur + 1;
            while (true) {
                const int kk = nx + lane;
                const bool inch = kk < n_es && et[kk < n_es ? kk : n_es - 1].first == sg.first;
                bool hk = false, ak = false, st = true;
                double svk = 0.0, evk = 0.0;
                if (inch) {
                    hk = hmark[bo + kk] != 0;
                    ak = act[bo + kk] != 0;
                    svk = sv[bo + kk];
                    evk = ev[bo + kk];
                    st = hk || ak || svk == r;
                }
                const unsigned long long mk = __ballot(st);
                const int f = mk ? __ffsll((long long)mk) - 1 : 64;
                if (f > 0) {
                    const SegDev s0 = et[nx], s1 = et[nx + f - 1];
                    const int64_t k0 = s0.pos / AMX_ENV_TF_, k1 = (s1.pos + s1.len + AMX_ENV_TF_ - 1) / AMX_ENV_TF_;
                    for (int64_t q = k0 + lane; q < k1; q += 64) ckr[q] = r;
                    if (lane < f) {
                        sv[bo + kk] = r;
                        ev[bo + kk] = r;
                    }
                    old_end = __shfl(evk, f - 1);            // the old end before the stop
                    walked += f;
                }
                if (f == 64) {
                    nx += 64;
                    continue;
                }
                const bool ins = __shfl((int)inch, f) != 0, hs = __shfl((int)hk, f) != 0;
                const double ss = __shfl(svk, f);
                if (!ins) { done = true; break; }            // past the chunk
                if (hs) {                                    // another chain's head
                    stale = stale || !(r == old_end);
                    done = true;
                    break;
                }
                if (ss == r) { done = true; break; }         // the link holds: the rest stands
                state = r;                                   // an active segment to re-run
                cur = nx + f;
                sg = et[cur];
                break;
            }
        }
        runs += walked;
        longest = walked > longest ? walked : longest;
        chains++;
    }
    if (lane == 0) {
        if (stale) flags[AMX_ENV_LIST + 2] = 1;          // k_envseq must check the links
        atomicAdd(ctr + 0, runs);
        atomicMax(ctr + 1, longest);
        atomicAdd(ctr + 2, chains);
    }
}

// --------------------------------------- final in-order walk (exactness net)
// One wave per (chunk, band): find the first segment whose start disagrees with
// its predecessor's end (64 at a time) and fix it with the whole wave, continue
// after it.  Nothing to do when no chain walker reported a head it may have raced
// (flags[fl] == 0; fl < 0: no fix-up ran, always walk).
template <bool RCP>
__global__ void __launch_bounds__(64) k_envseq(const ChainDev *__restrict__ cdp,
                                               const ChunkDev *__restrict__ chunks,
                                               const SegDev *__restrict__ es, int n_es,
                                               const int *__restrict__ eseg0,
                                               const int *__restrict__ neseg,
                                               const uint16_t *__restrict__ mm,
                                               const double *__restrict__ tabs,
                                               double *__restrict__ ck,
                                               double *__restrict__ sv, double *__restrict__ ev,
                                               const int *__restrict__ act, int64_t nloc,
                                               const int *__restrict__ flags, int fl) {
    if (fl >= 0 && __builtin_amdgcn_readfirstlane(flags[fl]) == 0) return;
    const ChainDev &cd = *cdp;
    const int c = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    const EnvBands eb = env_bands(flags + AMX_ENV_BACT);
    if (!eb.act(b)) return;
    const int tb = eb.nb;
    es += cd.etab[tb].es_off;
    const int s0 = eseg0[cd.etab[tb].ch_off + c], s1 = s0 + neseg[cd.etab[tb].ch_off + c];
    const ChunkDev ch = chunks[c];
    const int64_t ld = cd.es_ld;
    double *S = sv + (int64_t)b * ld, *E = ev + (int64_t)b * ld;
    const int *A = act + (int64_t)b * ld;
    const int64_t ro = b * nloc + ch.loc_off;
    int cur = s0;
    while (cur < s1) {
        int found = s1;
        for (int base = cur; base < s1; base += 64) {
            const int j = base + lane;
            bool bad = false;
            if (j < s1) bad = !((j == s0 ? 0.0 : E[j - 1]) == S[j]);
            const unsigned long long mk = __ballot(bad);
            if (mk) { found = base + __ffsll((long long)mk) - 1; break; }
        }
        if (found >= s1) break;
        const SegDev sg = es[found];
        const double ns = found == s0 ? 0.0 : E[found - 1];
        const double r = env_fix_segment<RCP>(cd, mm + ro, tabs + (int64_t)b * 3 * AMX_TAB,
                                              ck + ro / AMX_ENV_TF_, sg.pos, sg.len, A[found] != 0,
                                              ns, E[found]);
        __syncthreads();                    // every lane has read E/S of `found`
        if (lane == 0) {
            E[found] = r;
            S[found] = ns;
        }
        __threadfence_block();
        __syncthreads();
        cur = found + 1;
    }
}

// ------------------------------------------------------- gains + overlay
// The compressor output (audioop.mul of each frame by 10^(-att/20), :306-308) of
// all three bands and low.overlay(mid).overlay(high) (:309) with pydub's
// ms-rounded lengths (n1 after the first overlay, n2 = out_n after the second).
// A thread owns 16 consecutive frames of a chunk: per band it re-runs the
// recurrence from the checkpoint before its first frame (exact: the same operation
// sequence from the same state) and applies the gain; the three gained samples are
// summed with int16 saturation, band by band.
// Memory: a wave owns 1024 consecutive frames.  Per band its samples (4 KB) are read
// by 16-B pieces over consecutive lanes (every load instruction one contiguous KiB)
// into LDS rows of 16 frames, the next band's pieces already in flight (thread-owned
// 16-frame runs read directly touch 64 lines per instruction and left the loads
// TA-bound); the output goes back the same way.  A thread reads its own 16 r (32 B:
// the wave's loads still cover one contiguous 2 KB) and gathers m = mt[r] --
// neighbouring threads hold neighbouring frames, so a gather touches few table lines.
#define AMX_GO_XP 20       // sample / output row pitch in dwords (80 B)
#define AMX_GO_WAVES (AMX_BLOCK / 64)
template <bool RCP>
__global__ void __launch_bounds__(AMX_BLOCK) k_gain_overlay(const ChainDev *__restrict__ cdp,
                                                            const ChunkDev *__restrict__ chunks,
                                                            const uint16_t *__restrict__ mm,
                                                            const double *__restrict__ tabs,
                                                            const double *__restrict__ ck,
                                                            const uint32_t *__restrict__ bands,
                                                            uint32_t *__restrict__ out,
                                                            int64_t nloc,
                                                            const int64_t *__restrict__ n1tab,
                                                            const int *__restrict__ act,
                                                            const int *__restrict__ eseg0,
                                                            const int *__restrict__ neseg,
                                                            int use_act, const int *__restrict__ bact) {
    __shared__ __attribute__((aligned(16))) uint32_t sx_all[AMX_GO_WAVES][64 * AMX_GO_XP];
    const ChainDev &cd = *cdp;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = blockIdx.y;
    const ChunkDev ch = chunks[c];
    const int64_t wbase = ((int64_t)blockIdx.x * AMX_GO_WAVES + wv) * (64 * AMX_ENV_TF_);
    const int64_t n = ch.n, n2 = ch.out_n;
    if (wbase >= n2) return;                            // wave-uniform; no block barriers below
    const int64_t n1 = n1tab[c];
    uint32_t *sxw = sx_all[wv];
    const int64_t i0 = wbase + lane * AMX_ENV_TF_;      // this thread's first frame
    // the chunk row holds (n + 15) / 16 * 16 frames; pieces past it re-read its start
    const int64_t rowlen = (n + AMX_ENV_TF_ - 1) / AMX_ENV_TF_ * AMX_ENV_TF_;
    // r: this thread's 16 frames; sample piece p = 64 i + lane (i < 4) = frames 4p .. 4p+3
    const int64_t mo = ch.loc_off + (i0 < rowlen ? i0 : 0);
    int64_t xo[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int64_t f = wbase + 4 * (64 * i + lane);
        xo[i] = ch.loc_off + (f < rowlen ? f : 0);
    }
    // an inactive band (k_rms) has m = 0 and att = 0 everywhere: neither its r nor its
    // checkpoints are read.  With Le (the table's) a multiple of this wave's 1024 frames,
    // a band whose envelope segment has no over-threshold frame (act == 0) has m = 0 on
    // the whole tile -- its r is not read
    const EnvBands eb = env_bands(bact);
    bool mzero[3];
#pragma unroll
    for (int b = 0; b < 3; b++) mzero[b] = !eb.act(b);
    const int seg_tiles = use_act && cd.etab[eb.nb].Le % (64 * AMX_ENV_TF_) == 0 ? cd.etab[eb.nb].Le : 0;
    const int jt = seg_tiles ? (int)(wbase / seg_tiles) : 0;   // the envelope segment holding the wave
    if (seg_tiles && jt < neseg[cd.etab[eb.nb].ch_off + c]) {
        const int js = eseg0[cd.etab[eb.nb].ch_off + c] + jt;
#pragma unroll
        for (int b = 0; b < 3; b++) mzero[b] = mzero[b] || act[(int64_t)b * cd.es_ld + js] == 0;
    }
    u4v Mp[2];
    u4v Xp[4];
#pragma unroll
    for (int i = 0; i < 2; i++)
        Mp[i] = mzero[0] ? u4v{0u, 0u, 0u, 0u} : *reinterpret_cast<const u4v *>(mm + mo + 8 * i);
#pragma unroll
    for (int i = 0; i < 4; i++) Xp[i] = *reinterpret_cast<const u4v *>(bands + xo[i]);
    uint32_t acc[AMX_ENV_TF_];
#pragma unroll
    for (int f = 0; f < AMX_ENV_TF_; f++) acc[f] = 0u;
#pragma unroll
    for (int b = 0; b < 3; b++) {
        // this band's m for the thread's frames (frames past the chunk: r = 0, m = 0)
        const double *mt = tabs + (int64_t)b * 3 * AMX_TAB;
        double mv[AMX_ENV_TF_];
#pragma unroll
        for (int f = 0; f < AMX_ENV_TF_; f++) {
            const uint32_t r = (Mp[f >> 3][(f & 7) >> 1] >> (16 * (f & 1))) & 0xffffu;
            mv[f] = m_of(mt, i0 + f < n ? r : 0u);
        }
        // sample piece p -> row p / 4, dwords 4 (p % 4)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int p = 64 * i + lane;
            *reinterpret_cast<u4v *>(sxw + (p >> 2) * AMX_GO_XP + 4 * (p & 3)) = Xp[i];
        }
        __builtin_amdgcn_wave_barrier();
        if (b < 2) {                                    // next band in flight
            const int64_t bo = (int64_t)(b + 1) * nloc;
#pragma unroll
            for (int i = 0; i < 2; i++)
                Mp[i] = mzero[b + 1] ? u4v{0u, 0u, 0u, 0u} : *reinterpret_cast<const u4v *>(mm + bo + mo + 8 * i);
#pragma unroll
            for (int i = 0; i < 4; i++) Xp[i] = *reinterpret_cast<const u4v *>(bands + bo + xo[i]);
        }
        uint32_t xv[AMX_ENV_TF_];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const u4v v = *reinterpret_cast<const u4v *>(sxw + lane * AMX_GO_XP + 4 * k);
            xv[4 * k] = v.x; xv[4 * k + 1] = v.y; xv[4 * k + 2] = v.z; xv[4 * k + 3] = v.w;
        }
        __builtin_amdgcn_wave_barrier();
        double att = i0 < n && eb.act(b) ? ck[(b * nloc + ch.loc_off + i0) / AMX_ENV_TF_] : 0.0;
        // m = 0 on every frame of the wave (below the threshold) holds each lane's att,
        // so its gain is one value: formed once instead of per frame.  With att = 0 as
        // well every frame passes unchanged (the reference's "att != 0" test)
        bool loud = false;
#pragma unroll
        for (int f = 0; f < AMX_ENV_TF_; f++) loud = loud || mv[f] != 0.0;
        uint32_t gv[AMX_ENV_TF_];
        if (__ballot(loud) == 0) {
            if (__ballot(att != 0.0) == 0) {
#pragma unroll
                for (int f = 0; f < AMX_ENV_TF_; f++) gv[f] = xv[f];
            } else {
                const double g = gain_factor(cd, att);
#pragma unroll
                for (int f = 0; f < AMX_ENV_TF_; f++) gv[f] = gain_apply(xv[f], g);
            }
        } else {
#pragma unroll
            for (int f = 0; f < AMX_ENV_TF_; f++) {
                att = env_step<RCP>(cd, att, mv[f]);
                gv[f] = gain_frame(cd, xv[f], att);
            }
        }
#pragma unroll
        for (int f = 0; f < AMX_ENV_TF_; f++) {
            const int64_t i = i0 + f;
            const int g0 = lo16(gv[f]), g1 = hi16(gv[f]);
            if (b == 0) {
                acc[f] = gv[f];
            } else if (b == 1) {
                const bool in1 = i < n1;                // first overlay's length
                acc[f] = in1 ? pack2(sat16(lo16(acc[f]) + g0), sat16(hi16(acc[f]) + g1)) : 0u;
            } else {
                acc[f] = i < n ? pack2(sat16(lo16(acc[f]) + g0), sat16(hi16(acc[f]) + g1)) : 0u;
            }
        }
    }
    // output through LDS: row lane = frames i0 .. i0+15, stored as 16-B pieces
#pragma unroll
    for (int k = 0; k < 4; k++)
        *reinterpret_cast<u4v *>(sxw + lane * AMX_GO_XP + 4 * k) =
            u4v{acc[4 * k], acc[4 * k + 1], acc[4 * k + 2], acc[4 * k + 3]};
    __builtin_amdgcn_wave_barrier();
    uint32_t *ob = out + ch.out_off + wbase;
    const bool al = ((ch.out_off + wbase) & 3) == 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int p = 64 * i + lane;
        const u4v v = *reinterpret_cast<const u4v *>(sxw + (p >> 2) * AMX_GO_XP + 4 * (p & 3));
        const int64_t f = wbase + 4 * p;
        if (al && f + 4 <= n2) {
            *reinterpret_cast<u4v *>(ob + 4 * p) = v;
        } else {
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (f + q < n2) ob[4 * p + q] = v[q];
        }
    }
}

// ------------------------------------------ more than two channels (round 6)
// pydub's compressor on frames of C samples (a C > 2 file, :306-308).  The bands come
// from a stream sub-plan (pseudo-stereo int16 pairs: the stream in lo16, R = 0), whose
// chunk k holds chunk k's frames as n * C stream samples (frame i, channel c = stream
// sample i C + c); r, the checkpoints and the envelope segments belong to a stereo plan
// over the chunks' real frames (its k_env0 / fix-up kernels run on them unchanged).
// k_mc_rms: audioop.rms over the window's C (i - lo) samples, exactly as k_rms does for
// C = 2 (the same block prefix sums, S < 2^44 for C <= 8).
template <int LP>
__global__ void __launch_bounds__(AMX_BLOCK) k_mc_rms(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const ChunkDev *__restrict__ schunks,
                                                      const uint32_t *__restrict__ bands, int64_t snloc,
                                                      int C, uint16_t *__restrict__ mi, int64_t nloc,
                                                      int *bact) {
    constexpr int N = AMX_RMS_N;
    constexpr int F = N - LP;
    constexpr int PER = N / AMX_BLOCK;
    __shared__ unsigned long long P[N + N / 16];
    __shared__ unsigned long long wsum[AMX_BLOCK / 64];
    const int look = cdp->look;
    const int c = blockIdx.y, b = blockIdx.z;
    const ChunkDev ch = chunks[c];
    const int64_t base = (int64_t)blockIdx.x * F;
    if (base >= ch.n) return;                          // block-uniform
    const uint32_t *x = bands + b * snloc + schunks[c].loc_off;
    uint16_t *mo = mi + b * nloc + ch.loc_off;
    const int64_t rowlen = (ch.n + 15) / 16 * 16;
    const int64_t f0 = base - LP;
    const int t = threadIdx.x;
    unsigned long long v[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int64_t f = f0 + t * PER + q;
        unsigned long long e = 0;
        if (f >= 0 && f < ch.n) {
            const uint32_t *row = x + f * C;
            for (int k = 0; k < C; k++) {
                const int32_t a = lo16(row[k]);
                e += (unsigned long long)(uint32_t)(a * a);
            }
        }
        v[q] = e;
    }
    unsigned long long run = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) run += v[q];
    unsigned long long incl = run;
    const int lane = t & 63, w = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long up = __shfl_up(incl, o);
        if (lane >= o) incl += up;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    unsigned long long pp = incl - run;
    for (int q = 0; q < w; q++) pp += wsum[q];
    const int s0 = rms_slot(t * PER);
#pragma unroll
    for (int q = 0; q < PER; q++) { pp += v[q]; P[s0 + q] = pp; }
    __syncthreads();
    constexpr int OUT = F / AMX_BLOCK;
    const uint32_t cfull = (uint32_t)C * (uint32_t)look;
    const double rfull = 1.0 / (double)cfull;
    const uint32_t rq = (uint32_t)cdp->rq[b];
    bool hot = false;
#pragma unroll
    for (int k = 0; k < OUT; k++) {
        const uint32_t nn = (uint32_t)t + (uint32_t)k * AMX_BLOCK;
        const uint32_t e1 = nn + (LP - 1), e0 = e1 - (uint32_t)look;
        const uint64_t S = P[e1 + (e1 >> 4)] - P[e0 + (e0 >> 4)];
        const int64_t i = base + nn;
        const bool head = i < look;
        const uint32_t cnt = head ? (uint32_t)C * (uint32_t)i : cfull;
        const uint32_t rms = rms_floor(S, cnt, head ? 1.0 / (double)cnt : rfull);
        hot |= i < ch.n && rms >= rq;
        if (i < rowlen) mo[i] = i < ch.n ? (uint16_t)rms : (uint16_t)0;
    }
    if (__syncthreads_or(hot) && t == 0 && bact[b] == 0) bact[b] = 1;
}

// every frame's attenuation from the checkpoint before it (k_gain_overlay's sequence),
// the gain on the frame's C samples (audioop.mul) and the 3-band overlay with pydub's
// ms-rounded lengths, into the C-channel output [frames][C].  A thread per 16 frames.
template <bool RCP>
__global__ void __launch_bounds__(AMX_BLOCK) k_mc_gain_overlay(const ChainDev *__restrict__ cdp,
                                                               const ChunkDev *__restrict__ chunks,
                                                               const ChunkDev *__restrict__ schunks,
                                                               const uint16_t *__restrict__ mm,
                                                               const double *__restrict__ tabs,
                                                               const double *__restrict__ ck,
                                                               const uint32_t *__restrict__ bands,
                                                               int64_t snloc, int64_t nloc, int C,
                                                               const int64_t *__restrict__ n1tab,
                                                               const int *__restrict__ bact,
                                                               int16_t *__restrict__ out) {
    const ChainDev &cd = *cdp;
    const int c = blockIdx.y;
    const ChunkDev ch = chunks[c];
    const int64_t i0 = ((int64_t)blockIdx.x * AMX_BLOCK + threadIdx.x) * AMX_ENV_TF_;
    const int64_t n = ch.n, n2 = ch.out_n, n1 = n1tab[c];
    if (i0 >= n2) return;
    const EnvBands eb = env_bands(bact);
    const uint32_t *xb = bands + schunks[c].loc_off;
    double att[3];
#pragma unroll
    for (int b = 0; b < 3; b++)
        att[b] = (i0 < n && eb.act(b)) ? ck[(b * nloc + ch.loc_off + i0) / AMX_ENV_TF_] : 0.0;
    for (int f = 0; f < AMX_ENV_TF_; f++) {
        const int64_t i = i0 + f;
        if (i >= n2) break;
        double fac[3];
#pragma unroll
        for (int b = 0; b < 3; b++) {
            const bool on = i < n && eb.act(b);
            const double m = on ? m_of(tabs + (int64_t)b * 3 * AMX_TAB, mm[b * nloc + ch.loc_off + i]) : 0.0;
            att[b] = env_step<RCP>(cd, att[b], m);
            fac[b] = gain_factor(cd, att[b]);
        }
        int16_t *o = out + (ch.out_off + i) * C;
        for (int k = 0; k < C; k++) {
            int16_t v = 0;
            if (i < n) {
                const int64_t q = i * C + k;
                const int g0 = mul16(lo16(xb[q]), fac[0]);
                const int g1 = mul16(lo16(xb[snloc + q]), fac[1]);
                const int g2 = mul16(lo16(xb[2 * snloc + q]), fac[2]);
                const int lm = i < n1 ? (int)sat16(g0 + g1) : 0;     // the first overlay's length
                v = sat16(lm + g2);
            }
            o[k] = v;
        }
    }
}

hipError_t launch_mc_rms(const DynLaunch &d, const ChunkDev *schunks, const int16_t *bands, int64_t snloc,
                         int C, uint16_t *m, int *bact) {
    if (d.look > AMX_RMS_MAXLOOK || C < 1 || C > 8) return hipErrorInvalidValue;
    hipError_t e = launch_zero(bact, 3 * sizeof(int), d.st);       // (k_xover2 clears them for C = 2)
    if (e != hipSuccess) return e;
    const uint32_t *x = reinterpret_cast<const uint32_t *>(bands);
#define MCR(LPV)                                                                                   \
    {                                                                                              \
        constexpr int F = AMX_RMS_N - LPV;                                                         \
        dim3 g((unsigned)((d.max_chunk_n + F - 1) / F), (unsigned)d.n_chunks, 3);                  \
        if (!empty(g))                                                                             \
            hipLaunchKernelGGL(k_mc_rms<LPV>, g, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks, schunks, x, \
                               snloc, C, m, d.nloc, bact);                                         \
    }
    if (d.look <= 256) MCR(256) else if (d.look <= 512) MCR(512) else MCR(1024)
#undef MCR
    return hipGetLastError();
}

hipError_t launch_mc_gain_overlay(const DynLaunch &d, const ChunkDev *schunks, const uint16_t *m,
                                  const double *ck, const int16_t *bands, int64_t snloc, int C,
                                  int64_t max_chunk_out, const int64_t *n1tab, const int *bact, int16_t *out) {
    dim3 g((unsigned)((max_chunk_out + AMX_ENV_TF_ * AMX_BLOCK - 1) / (AMX_ENV_TF_ * AMX_BLOCK)),
           (unsigned)d.n_chunks);
    if (empty(g)) return hipSuccess;
    const uint32_t *x = reinterpret_cast<const uint32_t *>(bands);
    if (d.rcp)
        hipLaunchKernelGGL(k_mc_gain_overlay<true>, g, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks, schunks, m,
                           d.tabs, ck, x, snloc, d.nloc, C, n1tab, bact, out);
    else
        hipLaunchKernelGGL(k_mc_gain_overlay<false>, g, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks, schunks, m,
                           d.tabs, ck, x, snloc, d.nloc, C, n1tab, bact, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------- launchers
template <int LP>
static void rms_t(const DynLaunch &d, const int16_t *bands, uint16_t *m, int *bact) {
    constexpr int N = LP == 256 ? AMX_RMS_N256 : AMX_RMS_N;
    constexpr int F = N - LP;
    dim3 g((unsigned)((d.max_chunk_n + F - 1) / F), (unsigned)d.n_chunks, 3);
    if (empty(g)) return;
    hipLaunchKernelGGL((k_rms<LP, N>), g, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks,
                       reinterpret_cast<const uint32_t *>(bands), m, d.nloc, bact);
}

hipError_t launch_rms(const DynLaunch &d, const int16_t *bands, uint16_t *m, int *bact) {
    if (d.look > AMX_RMS_MAXLOOK) return hipErrorInvalidValue;
    if (d.look <= 256) rms_t<256>(d, bands, m, bact);
    else if (d.look <= 512) rms_t<512>(d, bands, m, bact);
    else rms_t<1024>(d, bands, m, bact);
    return hipGetLastError();
}

// part 0: the speculation (k_env0); part 1: the parallel fix-up (k_envheads + k_envchain)
template <bool RCP>
static void env_launch_t(const DynLaunch &d, const uint16_t *m, double *ck, double *sv, double *ev,
                         int *act, int *list, int *hmark, int *prev, int *list0, int *flags, int rounds,
                         int part) {
    if (part == 0) {
        const int wg = d.env_wg >= 1 && d.env_wg <= AMX_ENV_WG ? d.env_wg : 1;
        const dim3 g0((unsigned)((d.n_es + 64 * wg - 1) / (64 * wg)), 3);
        hipLaunchKernelGGL((k_env0<RCP>), g0, dim3(64 * wg), d.env_pin ? AMX_ENV_LDS_PIN : 0, d.st, d.cd,
                           d.chunks, d.es, d.n_es, m, d.tabs, ck, sv, ev, act, d.nloc, d.warm, flags);
        return;
    }
    if (rounds <= 0) return;                             // everything is left to k_envseq
    const dim3 gs((unsigned)((d.n_es + 63) / 64), 3);
    hipLaunchKernelGGL(k_envneed<RCP>, gs, dim3(64), 0, d.st, d.cd, d.es, d.n_es, sv, ev, act, flags, prev, list0);
    hipLaunchKernelGGL(k_envwide<RCP>, dim3(AMX_ENV_CHAIN_WAVES), dim3(64), 0, d.st, d.cd, d.chunks, d.es, m,
                       d.tabs, ck, sv, ev, act, flags, prev, list0, d.nloc);
    hipLaunchKernelGGL(k_envheads<RCP>, dim3((unsigned)((d.n_es + 63) / 64), 3), dim3(64), 0, d.st, d.cd, d.es,
                       d.n_es, sv, ev, flags, list, hmark);
    hipLaunchKernelGGL(k_envchain<RCP>, dim3(AMX_ENV_CHAIN_WAVES), dim3(64), 0, d.st, d.cd, d.chunks, d.es, m,
                       d.tabs, ck, sv, ev, act, flags, list, hmark, d.nloc);
}

hipError_t launch_env(const DynLaunch &d, const uint16_t *m, double *ck, double *sv, double *ev,
                      int *act, int *list, int *hmark, int *prev, int *list0, int *flags, int rounds,
                      int part) {
    if (d.n_es <= 0) return hipSuccess;
    if (d.warm % (AMX_ENV_TF * AMX_ENV_PF) || d.Le % (AMX_ENV_TF * AMX_ENV_PF))
        return hipErrorInvalidValue;
    if (rounds < 0 || rounds > AMX_ENV_MAX_ROUNDS) return hipErrorInvalidValue;
    if (d.rcp) env_launch_t<true>(d, m, ck, sv, ev, act, list, hmark, prev, list0, flags, rounds, part);
    else env_launch_t<false>(d, m, ck, sv, ev, act, list, hmark, prev, list0, flags, rounds, part);
    return hipGetLastError();
}

hipError_t launch_envseq(const DynLaunch &d, const uint16_t *m, double *ck, double *sv, double *ev,
                         const int *act, const int *flags, int rounds) {
    if (d.n_es <= 0) return hipSuccess;
    const dim3 gr((unsigned)d.n_chunks, 3);
    const int fl = rounds > 0 ? AMX_ENV_LIST + 2 : -1;
    if (d.rcp)
        hipLaunchKernelGGL(k_envseq<true>, gr, dim3(64), 0, d.st, d.cd, d.chunks, d.es, d.n_es,
                           d.eseg0, d.neseg, m, d.tabs, ck, sv, ev, act, d.nloc, flags, fl);
    else
        hipLaunchKernelGGL(k_envseq<false>, gr, dim3(64), 0, d.st, d.cd, d.chunks, d.es, d.n_es,
                           d.eseg0, d.neseg, m, d.tabs, ck, sv, ev, act, d.nloc, flags, fl);
    return hipGetLastError();
}

hipError_t launch_gain_overlay(const DynLaunch &d, const uint16_t *m, const double *ck,
                               const int16_t *bands, int16_t *out, int64_t max_chunk_out,
                               const int64_t *n1tab, const int *act, const int *bact) {
    dim3 g((unsigned)((max_chunk_out + AMX_ENV_TF_ * AMX_BLOCK - 1) / (AMX_ENV_TF_ * AMX_BLOCK)),
           (unsigned)d.n_chunks);
    if (empty(g)) return hipSuccess;
    const uint32_t *x = reinterpret_cast<const uint32_t *>(bands);
    uint32_t *o = reinterpret_cast<uint32_t *>(out);
    // (a wave's 1024 frames lie in one envelope segment when the table's Le is a multiple of 1024)
    if (d.rcp)
        hipLaunchKernelGGL(k_gain_overlay<true>, g, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks, m, d.tabs, ck,
                           x, o, d.nloc, n1tab, act, d.eseg0, d.neseg, act ? 1 : 0, bact);
    else
        hipLaunchKernelGGL(k_gain_overlay<false>, g, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks, m, d.tabs, ck,
                           x, o, d.nloc, n1tab, act, d.eseg0, d.neseg, act ? 1 : 0, bact);
    return hipGetLastError();
}

}  // namespace amx
