// amx_dev.hpp -- device helpers shared by the libamx kernels (gfx950).
#pragma once
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
// float_array_to_audio_segment (:255-256): np.clip to [-1, 1], * 32767, astype(int16).
// The clip is one v_med3_f32 / a raw v_min_f64 + v_max_f64 pair instead of two compares
// and selects (each select waits on its compare's VCC): the same value for every
// non-NaN input, and the chain's values are never NaN (int16 samples through finite
// coefficients)
__device__ __forceinline__ int16_t f32_to_s16(float x) {
    const float v = __builtin_amdgcn_fmed3f(x, -1.0f, 1.0f) * 32767.0f;
    return (int16_t)(int)v;
}
__device__ __forceinline__ double f64_clip1_raw(double x);
__device__ __forceinline__ int16_t f64_to_s16(double x) {
    return (int16_t)(int)(f64_clip1_raw(x) * 32767.0);
}
// "%.2f" then float(): the exact decimal rounding (half-even on exact ties) of v (the
// loudnorm statistics strings the reference parses, :237-241)
__device__ __forceinline__ double round2(double v) {
    if (!isfinite(v)) return v;
    const double p = v * 100.0;
    const double err = fma(v, 100.0, -p);        // v*100 == p + err exactly
    double k = rint(p);
    if (fabs(p - k) == 0.5 && err != 0.0) k = err > 0.0 ? floor(p) + 1.0 : floor(p);
    return k / 100.0;
}
__device__ __forceinline__ int16_t sat16(int v) {
    return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}
__device__ __forceinline__ uint32_t pack2(int16_t a, int16_t b) {
    return (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)b << 16);
}
__device__ __forceinline__ int16_t lo16(uint32_t v) { return (int16_t)(v & 0xffff); }
__device__ __forceinline__ int16_t hi16(uint32_t v) { return (int16_t)(v >> 16); }

// libswresample's linear float kernel (resample.asm, FMA3) for the rates whose 192 kHz
// phase step is not an integer (22.05 / 11.025 kHz: 1024 phases): the dots with rows h
// (phase ph) and h2 (ph + 1) as two sets of 8 fused chains over taps k, k+8, k+16, k+24;
// each set folded to 4 lanes (a[k] + a[k+4]); per lane val + (v2 - val) wf as one FMA
// (wf = (float)frac * (1.0f / src_incr), the plan's table); then the common kernel's
// horizontal sum.  oracle/amx_oracle.c swr_dot_lin is the same sequence.
__device__ __forceinline__ float swr_dot_lin(const float *w, const float *__restrict__ h,
                                             const float *__restrict__ h2, float wf) {
    float a[8], c[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        float acc = __builtin_fmaf(w[k], h[k], 0.0f), acc2 = __builtin_fmaf(w[k], h2[k], 0.0f);
#pragma unroll
        for (int q = 8; q < 32; q += 8) {
            acc = __builtin_fmaf(w[k + q], h[k + q], acc);
            acc2 = __builtin_fmaf(w[k + q], h2[k + q], acc2);
        }
        a[k] = acc;
        c[k] = acc2;
    }
    float e[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const float b = a[k] + a[k + 4], d = (c[k] + c[k + 4]) - b;
        e[k] = __builtin_fmaf(d, wf, b);
    }
    return (e[0] + e[2]) + (e[1] + e[3]);
}

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
// tanh comes from the plan's 65536-entry table of numpy's float32 tanh over every
// int16 input (design.py), so the result is the reference's own rounding.
// the part after the tanh table: t0, t1 = tanh of the left / right sample.
// lfilter's zero initial state makes the reference add 0.0 to the first products
// (y0 = 0 + b0 x0, (0 + x0 b1), v0, (0 + u0 b2_1)); those adds are left out.  0 + p == p
// except for p = -0.0, and a zero of either sign meeting + - x with finite operands
// gives the same nonzero values and zeros of possibly other sign, which the int16
// conversion maps to the same 0: the outputs are those of the reference's sequence.
// The clip to [-1, 1] is a raw v_min_f64 / v_max_f64 pair (the values are never NaN:
// table values through finite coefficients).
__device__ __forceinline__ double f64_clip1_raw(double x) {
    double a, b;
    asm("v_min_f64 %0, %1, 1.0" : "=v"(a) : "v"(x));
    asm("v_max_f64 %0, %1, -1.0" : "=v"(b) : "v"(a));
    return b;
}
__device__ __forceinline__ void analog_shelves(const ChainDev &cd, float t0, float t1, int16_t &ol,
                                               int16_t &orr) {
    const double x0 = (double)t0;
    const double x1 = (double)t1;
    const double *b1 = cd.an_lo, *b2 = cd.an_hi;
    // first shelf (120 Hz low, +cf dB): y0 = b0*x0 ; Z0 = x0*b1 - y0*a1 ; y1 = Z0 + b0*x1
    const double y0 = b1[0] * x0;
    const double z0 = x0 * b1[1] - y0 * b1[4];
    const double y1 = z0 + b1[0] * x1;
    const double u0 = x0 + (y0 - x0) * cd.an_glo1;
    const double u1 = x1 + (y1 - x1) * cd.an_glo1;
    const double v0 = b2[0] * u0;
    const double w = u0 * b2[1] - v0 * b2[4];
    const double v1 = w + b2[0] * u1;
    const double o0 = u0 + (v0 - u0) * cd.an_ghi1;
    const double o1 = u1 + (v1 - u1) * cd.an_ghi1;
    ol = (int16_t)(int)(f64_clip1_raw(o0) * 32767.0);
    orr = (int16_t)(int)(f64_clip1_raw(o1) * 32767.0);
}

__device__ __forceinline__ void analog_frame(const ChainDev &cd, const float *__restrict__ lut,
                                             int16_t l, int16_t r, int16_t &ol, int16_t &orr) {
    analog_shelves(cd, lut[(int)l + 32768], lut[(int)r + 32768], ol, orr);
}

// --------------------------------------------------------------- EQ chain
template <int MASK>
struct EqDim {
    static constexpr int v = ((MASK & 1) ? 2 : 0) + ((MASK & 2) ? 8 : 0) + ((MASK & 4) ? 8 : 0) +
                             ((MASK & 8) ? 2 : 0);
};

template <int MASK>
struct EqQ {   // doubles of ChainDev::eqc used by the active stages
    static constexpr int n = ((MASK & 1) ? 6 : 0) + ((MASK & 2) ? 21 : 0) + ((MASK & 4) ? 21 : 0) +
                             ((MASK & 8) ? 6 : 0);
};

// DF-II-T biquad on packed coefficients q = b0 b1 b2 a1 a2 (FMA recursion)
__device__ __forceinline__ double bq_step(const double *q, double &z0, double &z1, double x) {
    const double y = fma(q[0], x, z0);
    z0 = fma(-q[3], y, fma(q[1], x, z1));
    z1 = fma(-q[4], y, q[2] * x);
    return y;
}

// One channel of _apply_eq_to_channel (:277-282) over the active stages of MASK.
// q = the stage coefficients (registers, ChainDev::eqc layout), z = compact state,
// negm bit s = stage s is a negative-gain shelf (:289: x*g + (y - x*g)).  The first
// active stage sees the float32 column, so a negative first shelf forms x*g as a
// float32 product (NEP 50); later stages see float64.
template <int MASK>
__device__ __forceinline__ float eq_chain(int negm, const double *q, double *z, float xf) {
    double x = (double)xf;
    int o = 0, c = 0;
    if constexpr ((MASK & 1) != 0) {
        const double y = bq_step(q + c, z[o], z[o + 1], x);
        if (!(negm & 1)) x = x + (y - x) * q[c + 5];
        else { const double xg = (double)(xf * (float)q[c + 5]); x = xg + (y - xg); }
        o += 2;
        c += 6;
    }
#pragma unroll
    for (int s = 1; s <= 2; s++) {
        if ((MASK >> s) & 1) {
            double b = x;
#pragma unroll
            for (int k = 0; k < 4; k++) b = bq_step(q + c + 5 * k, z[o + 2 * k], z[o + 2 * k + 1], b);
            x = x + b * q[c + 20];
            o += 8;
            c += 21;
        }
    }
    if constexpr ((MASK & 8) != 0) {
        const double y = bq_step(q + c, z[o], z[o + 1], x);
        if (!(negm & 8)) x = x + (y - x) * q[c + 5];
        else if constexpr ((MASK & 7) == 0) { const double xg = (double)(xf * (float)q[c + 5]); x = xg + (y - xg); }
        else { const double xg = x * q[c + 5]; x = xg + (y - xg); }
        o += 2;
    }
    (void)o;
    if constexpr (MASK == 0) return xf;
    return (float)x;
}

// Stage-major form of eq_chain over F frames of one channel (amx_chain.hip k_front2):
// each stage runs over all F frames before the next, so only that stage's
// coefficients are live, as SGPR operands of the FMAs.  The two peak stages share
// one loop body (`#pragma unroll 1`) over a per-iteration coefficient address, with
// their 8-double states swapped between iterations; otherwise the compiler hoists
// and merges every stage's scalar loads (~54 doubles > the SGPR file) and spills.
// Inside a stage the unrolled section x frame grid is one basic block, so section
// k+1 of frame f overlaps section k of frame f+1.
struct EqState {
    double s0[2], pa[8], pb[8], s3[2];
};

template <int MASK>
__device__ __forceinline__ void eq_state_load(EqState &st, const double *z) {
    int o = 0;
    if constexpr ((MASK & 1) != 0) { st.s0[0] = z[0]; st.s0[1] = z[1]; o = 2; }
    if constexpr ((MASK & 2) != 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) st.pa[i] = z[o + i];
        o += 8;
    }
    if constexpr ((MASK & 4) != 0) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if constexpr ((MASK & 2) != 0) st.pb[i] = z[o + i];
            else st.pa[i] = z[o + i];
        }
        o += 8;
    }
    if constexpr ((MASK & 8) != 0) { st.s3[0] = z[o]; st.s3[1] = z[o + 1]; }
}

template <int MASK, int F>
__device__ __forceinline__ void eq_tile(int negm, const double *__restrict__ sq, EqState &st,
                                        double *x, const float *xf) {
    constexpr int NP = ((MASK >> 1) & 1) + ((MASK >> 2) & 1);
    int c = 0;
    if constexpr ((MASK & 1) != 0) {
        double q[6];
#pragma unroll
        for (int i = 0; i < 6; i++) q[i] = sq[i];
        // the uniform branch is taken outside the frame loop, so the F frames stay
        // one basic block (a per-frame branch splits the schedule at every frame)
        if (!(negm & 1)) {
#pragma unroll
            for (int f = 0; f < F; f++) {
                const double y = bq_step(q, st.s0[0], st.s0[1], x[f]);
                x[f] = x[f] + (y - x[f]) * q[5];
            }
        } else {
#pragma unroll
            for (int f = 0; f < F; f++) {
                const double y = bq_step(q, st.s0[0], st.s0[1], x[f]);
                const double xg = (double)(xf[f] * (float)q[5]);
                x[f] = xg + (y - xg);
            }
        }
        c = 6;
    }
    if constexpr (NP > 0) {
#pragma unroll 1
        for (int sidx = 0; sidx < NP; sidx++) {
            const double *q = sq + c + 21 * sidx;
            double b[F];
#pragma unroll
            for (int f = 0; f < F; f++) b[f] = x[f];
#pragma unroll
            for (int k = 0; k < 4; k++)
#pragma unroll
                for (int f = 0; f < F; f++)
                    b[f] = bq_step(q + 5 * k, st.pa[2 * k], st.pa[2 * k + 1], b[f]);
            const double gm1 = q[20];
#pragma unroll
            for (int f = 0; f < F; f++) x[f] = x[f] + b[f] * gm1;
            if constexpr (NP == 2) {
#pragma unroll
                for (int i = 0; i < 8; i++) { const double tmp = st.pa[i]; st.pa[i] = st.pb[i]; st.pb[i] = tmp; }
            }
        }
        c += 21 * NP;
    }
    if constexpr ((MASK & 8) != 0) {
        double q[6];
#pragma unroll
        for (int i = 0; i < 6; i++) q[i] = sq[c + i];
        if (!(negm & 8)) {
#pragma unroll
            for (int f = 0; f < F; f++) {
                const double y = bq_step(q, st.s3[0], st.s3[1], x[f]);
                x[f] = x[f] + (y - x[f]) * q[5];
            }
        } else {
#pragma unroll
            for (int f = 0; f < F; f++) {
                const double y = bq_step(q, st.s3[0], st.s3[1], x[f]);
                if constexpr ((MASK & 7) == 0) {
                    const double xg = (double)(xf[f] * (float)q[5]);
                    x[f] = xg + (y - xg);
                } else {
                    const double xg = x[f] * q[5];
                    x[f] = xg + (y - xg);
                }
            }
        }
    }
}

__device__ __forceinline__ void width_frame(float w, float &l, float &r) {
    // apply_stereo_width (:269-270), float32, exact order
    float mid = (l + r) / 2.0f, side = (l - r) / 2.0f;
    side = side * w;
    float nl = mid + side, nr = mid - side;
    l = __builtin_amdgcn_fmed3f(nl, -1.0f, 1.0f);
    r = __builtin_amdgcn_fmed3f(nr, -1.0f, 1.0f);
}
// the one channel a lane keeps (chn 0: left = clip(mid + side), 1: right = clip(mid - side))
__device__ __forceinline__ float width_one(float w, float l, float r, int chn) {
    const float mid = (l + r) / 2.0f, side = ((l - r) / 2.0f) * w;
    return __builtin_amdgcn_fmed3f(chn ? mid - side : mid + side, -1.0f, 1.0f);
}

// ------------------------------------------------------- LDS tile stager
// A workgroup owns AMX_BLOCK segments (one per thread).  Row r's frames live at
// dword offset rb[r] (W dwords per frame).  Tiles of AMX_TF frames per row move
// global <-> LDS cooperatively with dword accesses: consecutive lanes touch
// consecutive dwords of a row, so each wave instruction covers 1-2 rows of
// 64-128 contiguous bytes instead of 64 scattered cache lines.  The row pitch is
// ROW+1 dwords so the per-thread row reads are LDS-bank-conflict free.
#define AMX_TF AMX_TF_FRAMES
template <int W, int ROWS = AMX_BLOCK>
struct Tile {
    static constexpr int ROW = AMX_TF * W;
    static constexpr int PITCH = ROW + 1;
    static constexpr int WORDS = ROWS * PITCH;
    static constexpr int ITER = ROWS * ROW / AMX_BLOCK;   // dwords per thread per tile
    static constexpr int RSTEP = AMX_BLOCK / ROW;         // rows covered per iteration
    static constexpr int RW = ROWS / (AMX_BLOCK / 64);    // rows per wave (LOCAL)
};

// Row of iteration m for this thread.  Block-wide (LOCAL false): thread t moves
// column t % ROW of rows t / ROW + m RSTEP, so a tile needs a workgroup barrier.
// Wave-local (LOCAL true): the wave moves exactly the RW rows it computes on
// (rows RW w .. RW w + RW - 1, i.e. compute row = thread / (AMX_BLOCK / ROWS)), so
// a wave only waits for itself (amx_wave_sync) and the waves of a workgroup run
// their tiles independently.
template <int W, int ROWS, bool LOCAL>
__device__ __forceinline__ int tile_row(int m) {
    using T = Tile<W, ROWS>;
    if constexpr (LOCAL) {
        static_assert(64 % T::ROW == 0 && T::RW * (AMX_BLOCK / 64) == ROWS, "wave-local tile rows");
        return T::RW * (threadIdx.x >> 6) + (threadIdx.x & 63) / T::ROW + m * (64 / T::ROW);
    } else {
        return threadIdx.x / T::ROW + m * T::RSTEP;
    }
}

// LDS hand-off among the lanes of one wave (its LDS operations execute in order;
// this only keeps the compiler from moving them across)
__device__ __forceinline__ void amx_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Row r (< ROWS) holds frames n in [lo[r], hi[r]) at dword rb[r] + n*W (lo == nullptr
// -> 0).  Loads are issued unconditionally from a clamped in-range address and
// masked afterwards: a load guarded by a per-element branch makes hipcc wait
// vmcnt(0) after every element (cdna_hip_programming.md §5 "Three .s-level traps"
// (c)), which serialises the tile into dependent HBM round trips.
template <int W, int ROWS = AMX_BLOCK, bool LOCAL = false>
__device__ __forceinline__ void tile_load(uint32_t *lds, const uint32_t *__restrict__ src,
                                          const int64_t *rb, const int *lo, const int *hi,
                                          int k) {
    using T = Tile<W, ROWS>;
    uint32_t v[T::ITER];
    bool ok[T::ITER];
    const int c = threadIdx.x % T::ROW;              // column is fixed per thread
    const int n = k + c / W;
#pragma unroll
    for (int m = 0; m < T::ITER; m++) {
        const int r = tile_row<W, ROWS, LOCAL>(m);
        const int l0 = lo ? lo[r] : 0, h0 = hi[r];
        ok[m] = n >= l0 && n < h0;
        const int nn = ok[m] ? n : (h0 > l0 ? l0 : 0);
        v[m] = src[rb[r] + (int64_t)nn * W + (c % W)];
    }
#pragma unroll
    for (int m = 0; m < T::ITER; m++) {
        const int r = tile_row<W, ROWS, LOCAL>(m);
        lds[r * T::PITCH + c] = ok[m] ? v[m] : 0u;
    }
}

// Split form of tile_load for software pipelining: tile_fetch issues the global
// loads of tile k into registers (no wait), tile_put masks and writes them to LDS.
// Fetching tile k+1 before computing tile k keeps its HBM latency off the
// critical path (the loads are only waited for at the next tile_put).
template <int W, int ROWS = AMX_BLOCK>
struct TileRegs {
    uint32_t v[Tile<W, ROWS>::ITER];
};

template <int W, int ROWS = AMX_BLOCK, bool LOCAL = false>
__device__ __forceinline__ void tile_fetch(TileRegs<W, ROWS> &R, const uint32_t *__restrict__ src,
                                           const int64_t *rb, const int *lo, const int *hi,
                                           int k) {
    using T = Tile<W, ROWS>;
    const int c = threadIdx.x % T::ROW;
    const int n = k + c / W;
#pragma unroll
    for (int m = 0; m < T::ITER; m++) {
        const int r = tile_row<W, ROWS, LOCAL>(m);
        const int l0 = lo ? lo[r] : 0, h0 = hi[r];
        const bool ok = n >= l0 && n < h0;
        const int nn = ok ? n : (h0 > l0 ? l0 : 0);
        R.v[m] = src[rb[r] + (int64_t)nn * W + (c % W)];
    }
}

template <int W, int ROWS = AMX_BLOCK, bool LOCAL = false>
__device__ __forceinline__ void tile_put(uint32_t *lds, const TileRegs<W, ROWS> &R,
                                         const int *lo, const int *hi, int k) {
    using T = Tile<W, ROWS>;
    const int c = threadIdx.x % T::ROW;
    const int n = k + c / W;
#pragma unroll
    for (int m = 0; m < T::ITER; m++) {
        const int r = tile_row<W, ROWS, LOCAL>(m);
        const int l0 = lo ? lo[r] : 0, h0 = hi[r];
        lds[r * T::PITCH + c] = (n >= l0 && n < h0) ? R.v[m] : 0u;
    }
}

template <int W, int ROWS = AMX_BLOCK, bool LOCAL = false>
__device__ __forceinline__ void tile_store(const uint32_t *lds, uint32_t *__restrict__ dst,
                                           const int64_t *rb, const int *hi, int k) {
    using T = Tile<W, ROWS>;
    const int c = threadIdx.x % T::ROW;
    const int n = k + c / W;
#pragma unroll
    for (int m = 0; m < T::ITER; m++) {
        const int r = tile_row<W, ROWS, LOCAL>(m);
        if (n < hi[r]) dst[rb[r] + (int64_t)n * W + (c % W)] = lds[r * T::PITCH + c];
    }
}

// the other lane of an even/odd lane pair (channel pairs, DPP quad_perm [1,0,3,2])
__device__ __forceinline__ float pair_swap(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ double pair_swap(double v) {
    const int64_t b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0xB1, 0xF, 0xF, false);
    return __longlong_as_double(((int64_t)hi << 32) | (uint32_t)lo);
}

static inline dim3 grid1(int64_t n) { return dim3((unsigned)((n + AMX_BLOCK - 1) / AMX_BLOCK)); }
static inline bool empty(dim3 g) { return g.x == 0 || g.y == 0 || g.z == 0; }

}  // namespace amx
