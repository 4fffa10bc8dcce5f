// amx_chain.hip -- the per-chunk linear chain on CDNA4 (gfx950):
//   quantise (A.1) -> analog character (:258-266) -> 4-stage EQ (:272-298)
//   -> width (:267-271) -> int16 (:254-257) [-> crossover bands (:300-305)]
//
// Every IIR runs time-parallel by a 2-pass state-space method:
// pass 1 = zero-state end state of each segment as a GEMV e = G x (independent
// FMAs, G rows wave-uniform -> scalar loads); an affine scan over segments
// (amx_scan.hip) gives the exact segment start states; pass 2 re-runs the
// recursion from the true state.  Chunks restart from rest (:185-204).
// Memory-less stages keep the reference's float32/float64 operation order exactly
// (-ffp-contract=off; FMAs only inside the IIR recursions).  Segment kernels
// stream their rows through LDS tiles (amx_dev.hpp tile_load / tile_store):
// coalesced dword traffic, recursion reads from LDS.
#include "amx_dev.hpp"

// AMX_VT_LATE (the segment kernels' tile movers: front1s_run, k_gemv16, vt_fetch): a
// prefetched tile is masked when it is put into LDS, not right after its load -- a select
// beside the load made the compiler wait for the prefetch at once -- and the prefetch is
// unconditional (past the last tile it re-reads the current one)
#ifndef AMX_VT_LATE
#define AMX_VT_LATE 1
#endif

namespace amx {

#define AMX_HALF_LUT 32769   // entries of the odd tanh table's half (tanh(s) = sign(s) half[|s|])

__device__ __forceinline__ void decode_in(const ChainDev &cd, const uint32_t *row, int f,
                                          int win, int16_t &l, int16_t &r) {
    if (win == 2) {
        l = q_f32_to_s16_ffmpeg(__uint_as_float(row[2 * f]));
        r = q_f32_to_s16_ffmpeg(__uint_as_float(row[2 * f + 1]));
    } else {
        const uint32_t w = row[f];
        if (cd.in_s16) {
            l = lo16(w);
            r = hi16(w);
        } else {
            l = r = q_f32_to_s16_ffmpeg(__uint_as_float(w));   // mono duplicated (:190)
        }
    }
}

// ------------------------------------------------ pass 1: quantise/analog + GEMV
// One thread per segment (both channels): frames stream through LDS tiles (fetched
// one ahead); the GEMV row G[n] is the same for every lane (wave-uniform -> scalar
// loads, SGPR operands), each used by both channels' FMAs.  The frame loop is
// unrolled by 2 only, so at most two G rows (2 x D doubles) are live in SGPRs: a
// full unroll spills SGPRs to VGPR lanes.  (A thread per (segment, channel) halves
// the reuse of each scalar-loaded G value and measured 35 % slower.)
// SC (a stream chain, amx_chain_desc.stream_chain): the input enters the EQ as
// lut[s + 32768] when a table is given (the analog character's tanh of a C > 2 stream),
// else as s / 32768
template <int D, int WIN, bool AN, bool SC = false>
__global__ void __launch_bounds__(AMX_BLOCK) k_front1(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const SegDev *__restrict__ segs, int n_seg,
                                                      int L, const uint32_t *__restrict__ in,
                                                      const float *__restrict__ lut,
                                                      uint32_t *__restrict__ a16,
                                                      const double *__restrict__ G,
                                                      double *__restrict__ e) {
    __shared__ uint32_t s_in[Tile<WIN>::WORDS];
    __shared__ uint32_t s_out[Tile<1>::WORDS];
    __shared__ int64_t rb_in[AMX_BLOCK], rb_out[AMX_BLOCK];
    __shared__ int rl[AMX_BLOCK];
    const ChainDev &cd = *cdp;
    const int t = threadIdx.x;
    const int j = blockIdx.x * AMX_BLOCK + t;
    bool need_e = false;
    rb_in[t] = 0;
    rb_out[t] = 0;
    rl[t] = 0;
    if (j < n_seg) {
        const SegDev sg = segs[j];
        const ChunkDev ch = chunks[sg.chunk];
        rb_in[t] = (ch.in_off + sg.pos) * WIN;
        rb_out[t] = ch.loc_off + sg.pos;
        rl[t] = sg.len;
        need_e = !sg.last;
    }
    double e0[D > 0 ? D : 1], e1[D > 0 ? D : 1];
#pragma unroll
    for (int d = 0; d < D; d++) { e0[d] = 0.0; e1[d] = 0.0; }
    __syncthreads();
    TileRegs<WIN> R;
    tile_fetch<WIN>(R, in, rb_in, nullptr, rl, 0);
    for (int k = 0; k < L; k += AMX_TF) {
        tile_put<WIN>(s_in, R, nullptr, rl, k);
        __syncthreads();
        if (k + AMX_TF < L) tile_fetch<WIN>(R, in, rb_in, nullptr, rl, k + AMX_TF);
        const uint32_t *row = s_in + t * Tile<WIN>::PITCH;
        uint32_t *orow = s_out + t * Tile<1>::PITCH;
#pragma unroll 2
        for (int f = 0; f < AMX_TF; f++) {
            int16_t l, r;
            decode_in(cd, row, f, WIN, l, r);
            if constexpr (AN) analog_frame(cd, lut, l, r, l, r);
            orow[f] = pack2(l, r);
            if constexpr (D > 0) {
                const double *g = G + (int64_t)(k + f) * D;   // wave-uniform row
                double x0, x1;
                if constexpr (SC) {
                    x0 = lut ? (double)lut[(int)l + 32768] : (double)((float)l / 32768.0f);
                    x1 = lut ? (double)lut[(int)r + 32768] : (double)((float)r / 32768.0f);
                } else {
                    x0 = (double)((float)l / 32768.0f);
                    x1 = (double)((float)r / 32768.0f);
                }
#pragma unroll
                for (int d = 0; d < D; d++) {
                    e0[d] = fma(g[d], x0, e0[d]);
                    e1[d] = fma(g[d], x1, e1[d]);
                }
            }
        }
        __syncthreads();
        tile_store<1>(s_out, a16, rb_out, rl, k);
    }
    if constexpr (D > 0) {
        if (need_e) {
            double *o = e + (int64_t)j * 2 * D;
#pragma unroll
            for (int d = 0; d < D; d++) { o[d] = e0[d]; o[D + d] = e1[d]; }
        }
    }
}

// Stereo float32 input (the product path): two threads per segment, each holding
// both channels' accumulators for half of the D state components (lanes 2i / 2i+1
// = components [0, D/2) / [D/2, D) of row i), so a G value read once feeds two
// FMAs and the launch has two waves per 64 segments.  The G rows of a tile go
// through LDS (ds_read_b128; scalar loads thrash the scalar cache on the 20 KB
// table).  Each lane quantises both samples (the analog stage couples the
// channels).  Tile loads are 16 B per lane from row pointers formed once (lane
// t: 16-B column t % 8 of rows t / 8 + 32 m), issued one tile ahead; only a
// workgroup with a partial (chunk-final) segment clamps addresses (PART).
#define AMX_F1_PITCH (2 * AMX_TF + 2)   // dwords per LDS row: 8-B aligned, conflict-free
template <int D, bool AN, bool PART>
__device__ __forceinline__ void front1s_run(const ChainDev &cd, const float *__restrict__ lut,
                                            const uint32_t *__restrict__ const *ip,
                                            const int *ilen, uint32_t *const *op,
                                            int c4, int rg, uint32_t *s_in,
                                            uint32_t *s_out, int row, int half, int L, int len,
                                            const double *__restrict__ G, double *sG,
                                            double *__restrict__ eo) {
    constexpr int H = D / 2;
    double a0[H > 0 ? H : 1], a1[H > 0 ? H : 1];
#pragma unroll
    for (int d = 0; d < H; d++) { a0[d] = 0.0; a1[d] = 0.0; }
    constexpr int GQ = AMX_TF * D / 2;                  // 16-B pieces of a G tile
    uint4 R[4], RG;
    auto fetch = [&](int k) {
        const int tt = threadIdx.x;
#if AMX_VT_LATE
        RG = *reinterpret_cast<const uint4 *>(G + (int64_t)k * D + 2 * (tt < GQ ? tt : 0));
#else
        RG = tt < GQ ? *reinterpret_cast<const uint4 *>(G + (int64_t)k * D + 2 * tt)
                     : make_uint4(0u, 0u, 0u, 0u);
#endif
#pragma unroll
        for (int m = 0; m < 4; m++) {
            if constexpr (PART) {
                const bool ok = k + 2 * c4 < ilen[m];          // frames k + 2 c4, +1
                R[m] = *reinterpret_cast<const uint4 *>(ip[m] + (ok ? 2 * k : -4 * c4));
#if !AMX_VT_LATE
                if (!ok) R[m] = make_uint4(0u, 0u, 0u, 0u);
#endif
            } else {
                R[m] = *reinterpret_cast<const uint4 *>(ip[m] + 2 * k);
            }
        }
    };
    fetch(0);
    const uint32_t *rp = s_in + row * AMX_F1_PITCH;
    for (int k = 0; k < L; k += AMX_TF) {
#pragma unroll
        for (int m = 0; m < 4; m++) {
            uint4 v = R[m];
#if AMX_VT_LATE
            if constexpr (PART) {                               // (AMX_VT_LATE: masked here)
                if (!(k + 2 * c4 < ilen[m])) v = make_uint4(0u, 0u, 0u, 0u);
            }
#endif
            uint32_t *w = s_in + (rg + 32 * m) * AMX_F1_PITCH + 4 * c4;
            *reinterpret_cast<uint2 *>(w) = make_uint2(v.x, v.y);
            *reinterpret_cast<uint2 *>(w + 2) = make_uint2(v.z, v.w);
        }
        if (threadIdx.x < GQ) reinterpret_cast<uint4 *>(sG)[threadIdx.x] = RG;
        __syncthreads();
#if AMX_VT_LATE
        fetch(k + AMX_TF < L ? k + AMX_TF : k);
#else
        if (k + AMX_TF < L) fetch(k + AMX_TF);
#endif
        if constexpr (AN) {
            // The analog stage couples the channels, so a lane takes whole frames: the
            // two lanes of a pair take every other frame (f = 2 i + half), both
            // channels, through the tanh table and the shelves -- each frame's analog
            // arithmetic is done once, not by both lanes -- and write its s16 pair
            // to the output row, from which the GEMV loop reads every frame.  The
            // table lookups of the tile are all issued first (a lookup per step left an
            // L2 round trip on every step).
            float t0[AMX_TF / 2], t1[AMX_TF / 2];
#pragma unroll
            for (int i = 0; i < AMX_TF / 2; i++) {
                const int f = 2 * i + half;
                const int q0 = (int)q_f32_to_s16_ffmpeg(__uint_as_float(rp[2 * f]));
                const int q1 = (int)q_f32_to_s16_ffmpeg(__uint_as_float(rp[2 * f + 1]));
                t0[i] = lut[q0 + 32768];
                t1[i] = lut[q1 + 32768];
            }
#pragma unroll
            for (int i = 0; i < AMX_TF / 2; i++) {
                int16_t l, r;
                analog_shelves(cd, t0[i], t1[i], l, r);
                s_out[row * (AMX_TF + 1) + 2 * i + half] = pack2(l, r);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll 1
        for (int f = 0; f < AMX_TF; f++) {
            int16_t l, r;
            if constexpr (AN) {
                const uint32_t w = s_out[row * (AMX_TF + 1) + f];
                l = lo16(w);
                r = hi16(w);
            } else {
                l = q_f32_to_s16_ffmpeg(__uint_as_float(rp[2 * f]));
                r = q_f32_to_s16_ffmpeg(__uint_as_float(rp[2 * f + 1]));
                if (half == 0) s_out[row * (AMX_TF + 1) + f] = pack2(l, r);
            }
            double x0 = (double)((float)l / 32768.0f), x1 = (double)((float)r / 32768.0f);
            if constexpr (PART) {
                x0 = k + f < len ? x0 : 0.0;
                x1 = k + f < len ? x1 : 0.0;
            }
            const double *g = sG + f * D + half * H;
#pragma unroll
            for (int d = 0; d < H; d++) {
                a0[d] = fma(g[d], x0, a0[d]);
                a1[d] = fma(g[d], x1, a1[d]);
            }
        }
        __syncthreads();
        // s16 tile -> a16: lane t stores frames 2 (t % 8), +1 of rows t / 8 + 32 m
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint32_t *so = s_out + (rg + 32 * m) * (AMX_TF + 1) + 2 * c4;
            const uint32_t w0 = so[0], w1 = so[1];
            if constexpr (PART) {
                if (k + 2 * c4 < ilen[m]) op[m][k] = w0;
                if (k + 2 * c4 + 1 < ilen[m]) op[m][k + 1] = w1;
            } else {
                *reinterpret_cast<uint2 *>(op[m] + k) = make_uint2(w0, w1);
            }
        }
    }
    if (eo) {
#pragma unroll
        for (int d = 0; d < H; d++) { eo[d] = a0[d]; eo[D + d] = a1[d]; }
    }
}

template <int D, bool AN>
__global__ void __launch_bounds__(AMX_BLOCK, 4) k_front1s(const ChainDev *__restrict__ cdp,
                                                          const ChunkDev *__restrict__ chunks,
                                                          const SegDev *__restrict__ segs,
                                                          int n_seg, int L,
                                                          const uint32_t *__restrict__ in,
                                                          const float *__restrict__ lut,
                                                          uint32_t *__restrict__ a16,
                                                          const double *__restrict__ G,
                                                          double *__restrict__ e) {
    constexpr int ROWS = AMX_BLOCK / 2;
    constexpr int H = D / 2;
    __shared__ uint32_t s_in[ROWS * AMX_F1_PITCH];
    __shared__ uint32_t s_out[ROWS * (AMX_TF + 1)];
    __shared__ __attribute__((aligned(16))) double sG[AMX_TF * (D > 0 ? D : 2)];
    __shared__ int64_t rb_in[ROWS], rb_out[ROWS];
    __shared__ int rl[ROWS];
    static_assert(AMX_TF * D / 2 <= AMX_BLOCK, "one 16-B piece of the G tile per thread");
    static_assert(D % 2 == 0, "state split in halves");
    const ChainDev &cd = *cdp;
    const int t = threadIdx.x, row = t >> 1, half = t & 1;
    const int j = blockIdx.x * ROWS + row;
    const bool valid = j < n_seg;
    const SegDev sg = segs[valid ? j : n_seg - 1];
    const ChunkDev ch = chunks[sg.chunk];
    const int len = valid ? sg.len : 0;
    if (half == 0) {
        rb_in[row] = valid ? (ch.in_off + sg.pos) * 2 : 0;
        rb_out[row] = valid ? ch.loc_off + sg.pos : 0;
        rl[row] = len;
    }
    const int part = __syncthreads_or(len < L);
    const int c4 = t & 7, rg = t >> 3;
    const uint32_t *ip[4];
    int ilen[4];
    uint32_t *op[4];
#pragma unroll
    for (int m = 0; m < 4; m++) {
        ip[m] = in + rb_in[rg + 32 * m] + 4 * c4;
        ilen[m] = rl[rg + 32 * m];
        op[m] = a16 + rb_out[rg + 32 * m] + 2 * c4;
    }
    double *eo = (D > 0 && valid && !sg.last) ? e + (int64_t)j * 2 * D + half * H : nullptr;
    if (part)
        front1s_run<D, AN, true>(cd, lut, ip, ilen, op, c4, rg, s_in, s_out, row, half, L, len,
                                 G, sG, eo);
    else
        front1s_run<D, AN, false>(cd, lut, ip, ilen, op, c4, rg, s_in, s_out, row, half, L, len,
                                  G, sG, eo);
}

// ----------------------------------- analog character as its own elementwise pass
// Float32 stereo input with the analog stage (:258-266): quantise (A.1), the tanh
// table, the two channel-axis shelves -> the chain's s16 input a16.  Every frame is
// independent (the shelves filter along the channel axis), so the launch has a wave per
// 256 frames: thousands of waves in flight, where the segment kernel did this work on 2
// waves per 64 segments beside its GEMV.  The EQ GEMV then runs over a16 (k_gemv16).
// The tanh table sits in LDS (measured: a global-table form is bound by the L2 -> L1
// traffic of its scattered table reads, 105 us at C3; a segment kernel holding the table
// in LDS, 150 us -- DESIGN.md §3.4).  numpy's float32 tanh table is odd (the plan checks
// every pair bit for bit), so the 32 769-entry half table (128 KB) sits in the LDS of one
// 1024-thread workgroup per CU (4 waves per SIMD), loaded once; the workgroups then
// stride over every chunk's 4-frame groups.
#ifndef AMX_AN_VEC
#define AMX_AN_VEC 1       // k_analog_h<true> where the plan allows it (0: always the general form)
#endif
#ifndef AMX_AN_DEPTH
#define AMX_AN_DEPTH 3     // input blocks held in registers (2: one block ahead)
#endif
__device__ __forceinline__ void analog_load8(const float *src, int64_t f, int64_t n, bool vin, float (&x)[8]) {
    if (f + 4 <= n && vin) {
        const float4 u0 = *reinterpret_cast<const float4 *>(src);
        const float4 u1 = *reinterpret_cast<const float4 *>(src + 4);
        x[0] = u0.x; x[1] = u0.y; x[2] = u0.z; x[3] = u0.w;
        x[4] = u1.x; x[5] = u1.y; x[6] = u1.z; x[7] = u1.w;
    } else {
#pragma unroll
        for (int e = 0; e < 8; e++) x[e] = f + e / 2 < n ? src[e] : 0.0f;
    }
}

// The workgroups stride over the 4096-frame blocks of all chunks in one sequence (block
// b of the job -> its chunk by a scalar walk over the chunk list, monotone per
// workgroup), so a chunk's last, partial round of blocks does not leave most workgroups
// idle before the next chunk starts (C3: 352 blocks per chunk over 256 workgroups;
// striding chunk by chunk measured 52.6 against 49.4 us)
// VEC (the host checks: every chunk starts at an even input frame, holds >= 4 frames, and
// the input is 16-B aligned): the loop moves whole quads only -- 16-B loads, no masks and
// no second load path, so the compiler keeps two blocks in flight over the third's
// compute -- and a chunk's last n % 4 frames are done after the loop, a lane each.
template <bool VEC>
__global__ void __launch_bounds__(1024) k_analog_h(const ChainDev *__restrict__ cdp,
                                                   const ChunkDev *__restrict__ chunks, int n_chunks,
                                                   const float *__restrict__ in,
                                                   const float *__restrict__ lut_half,
                                                   uint32_t *__restrict__ a16, int64_t n_blocks) {
    __shared__ float s_tab[AMX_HALF_LUT];
    for (int i = threadIdx.x; i < AMX_HALF_LUT; i += 1024) s_tab[i] = lut_half[i];
    __syncthreads();
    const ChainDev &cd = *cdp;
#if AMX_AN_DEPTH < 3
    auto work = [&](const ChunkDev &ch, const float (&x)[8], int64_t ff) {
        float t[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const int q = (int)q_f32_to_s16_ffmpeg(x[e]);
            // tanh(s) = sign(s) half[|s|]: half[] >= +0, so the sign is q's sign bit
            // OR-ed into the value's (the plan checked lut[-s] == -lut[s] bit for bit)
            const float v = s_tab[abs(q)];
            t[e] = __int_as_float(__float_as_int(v) | (q & (int)0x80000000));
        }
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            int16_t l, r;
            analog_shelves(cd, t[2 * i], t[2 * i + 1], l, r);
            o[i] = pack2(l, r);
        }
        uint32_t *dst = a16 + ch.loc_off + ff;
        if (ff + 4 <= ch.n && (ch.loc_off & 3) == 0) {
            *reinterpret_cast<uint4 *>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (ff + i < ch.n) dst[i] = o[i];
        }
    };
#endif
    constexpr int64_t BF = 1024 * 4;                   // frames per block
    int c = 0;
    int64_t cb0 = 0;                                    // first block of chunk c
#if AMX_AN_DEPTH >= 3
    // Three register sets: the next two blocks' input (64 KB per CU) is in flight while
    // one is computed; one block ahead (32 KB per CU) held the kernel at ~3.6 TB/s.  For
    // the loads to stay in flight, every pass through the loop issues at least the
    // steady state's memory operations in the same order (the counter the waits use is
    // in order, and a path with fewer operations after a load makes the compiler wait
    // for everything):
    //  - the chunk list is read through the constant address space (scalar loads, their
    //    own counter) -- as vector loads, each chunk change waited out every load;
    //  - a lane's quad is clamped to its chunk's last quad, so every lane of a block
    //    stores one 16-B quad: lanes past the end recompute the last quad from the same
    //    inputs and store the same bytes; frames past n read as 0 and land in the row's
    //    padding (rows are 16-frame aligned, amx_plan.cpp), whose content nobody reads;
    //  - a refill past the last block reloads its set's previous (valid) block, unused.
    struct Ck { int64_t in_off, loc_off, n; };
    auto kload = [&](int cix) -> Ck {                   // scalar loads (constant space)
        typedef const __attribute__((address_space(4))) int64_t *K64;
        const K64 q = (K64)(chunks + cix);
        return Ck{q[0], q[1], q[3]};                    // in_off, loc_off, n (ChunkDev order)
    };
    const bool inv = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
    auto load_q = [&](const Ck &cc, int64_t f, float (&x)[8]) {
        const float *src = in + (cc.in_off + f) * 2;
        if (VEC || (inv && (cc.in_off & 1) == 0 && f + 4 <= cc.n)) {        // 16-B aligned whole quad
            const float4 u0 = *reinterpret_cast<const float4 *>(src);
            const float4 u1 = *reinterpret_cast<const float4 *>(src + 4);
            x[0] = u0.x; x[1] = u0.y; x[2] = u0.z; x[3] = u0.w;
            x[4] = u1.x; x[5] = u1.y; x[6] = u1.z; x[7] = u1.w;
        } else {                                                    // dwords, clamped
            const float *rowp = in + cc.in_off * 2;
#pragma unroll
            for (int e = 0; e < 8; e++) {               // (masked in work_q: no wait here)
                const int64_t fr = f + e / 2;
                x[e] = rowp[(fr < cc.n ? fr : cc.n - 1) * 2 + (e & 1)];
            }
        }
    };
    auto work_q = [&](const Ck &cc, const float (&x)[8], int64_t f) {
        float t[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            const int q = VEC || f + e / 2 < cc.n ? (int)q_f32_to_s16_ffmpeg(x[e]) : 0;
            const float v = s_tab[abs(q)];
            t[e] = __int_as_float(__float_as_int(v) | (q & (int)0x80000000));
        }
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            int16_t l, r;
            analog_shelves(cd, t[2 * i], t[2 * i + 1], l, r);
            o[i] = pack2(l, r);
        }
        *reinterpret_cast<uint4 *>(a16 + cc.loc_off + f) = make_uint4(o[0], o[1], o[2], o[3]);
    };
    Ck ck = kload(0);
    int64_t nbk = (ck.n + BF - 1) / BF;
    auto seek_k = [&](int64_t b) -> bool {                // workgroup-uniform
        while (b >= cb0 + nbk) {
            cb0 += nbk;
            if (++c >= n_chunks) return false;
            ck = kload(c);
            nbk = (ck.n + BF - 1) / BF;
        }
        return true;
    };
    // this workgroup's blocks: k = 0 .. K-1 are job blocks blockIdx.x + k gridDim.x
    const int64_t K = n_blocks > (int64_t)blockIdx.x ? (n_blocks - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
    if (K == 0) return;
    int64_t kn = 0;                                     // the next block to issue
    auto issue = [&](float (&x)[8], Ck &cc, int64_t &f) {
        if (kn < K) {                                   // (scalar work only: the same
            const int64_t b = (int64_t)blockIdx.x + kn * gridDim.x;   //  vector memory ops
            seek_k(b);                                  //  on both sides)
            cc = ck;
            const int64_t fq = (b - cb0) * BF + threadIdx.x * 4;
            const int64_t ql = VEC ? (cc.n / 4 - 1) * 4 : (cc.n - 1) / 4 * 4;   // (VEC: whole quads)
            f = fq < ql ? fq : ql;
        }
        kn++;
        load_q(cc, f, x);
    };
    float xa[8], xb[8], xc[8];
    Ck ca = ck, cb = ck, cc = ck;
    int64_t fa = 0, fb = 0, fc = 0;
    issue(xa, ca, fa);
    cb = ca; fb = fa; cc = ca; fc = fa;
    issue(xb, cb, fb);
    issue(xc, cc, fc);
    // one exit, and every iteration issues the same memory operations in the same order
    int64_t k = 0;
    for (; k + 3 <= K; k += 3) {
        work_q(ca, xa, fa);
        issue(xa, ca, fa);
        work_q(cb, xb, fb);
        issue(xb, cb, fb);
        work_q(cc, xc, fc);
        issue(xc, cc, fc);
    }
    if (k < K) work_q(ca, xa, fa);
    if (k + 1 < K) work_q(cb, xb, fb);
    if constexpr (VEC) {
        // the chunks' last n % 4 frames, a lane each
        for (int cix = blockIdx.x; cix < n_chunks; cix += gridDim.x) {
            const Ck q = kload(cix);
            const int r = (int)(q.n & 3);
            if ((int)threadIdx.x < r) {
                const int64_t fr = q.n - r + threadIdx.x;
                const float *src = in + (q.in_off + fr) * 2;
                float t2[2];
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const int qq = (int)q_f32_to_s16_ffmpeg(src[e]);
                    const float v = s_tab[abs(qq)];
                    t2[e] = __int_as_float(__float_as_int(v) | (qq & (int)0x80000000));
                }
                int16_t l, rr;
                analog_shelves(cd, t2[0], t2[1], l, rr);
                a16[q.loc_off + fr] = pack2(l, rr);
            }
        }
    }
#else
    ChunkDev ch = chunks[0];
    int64_t nb = (ch.n + BF - 1) / BF;
    auto seek = [&](int64_t b) -> bool {                // workgroup-uniform
        while (b >= cb0 + nb) {
            cb0 += nb;
            if (++c >= n_chunks) return false;
            ch = chunks[c];
            nb = (ch.n + BF - 1) / BF;
        }
        return true;
    };
    int64_t b = blockIdx.x;
    if (!seek(b)) return;
    ChunkDev cc = ch;
    int64_t f = (b - cb0) * BF + threadIdx.x * 4;
    // two register sets: the next block's input is in flight while one is computed
    float xa[8], xb[8];
    analog_load8(in + (cc.in_off + f) * 2, f, cc.n, (cc.in_off & 1) == 0, xa);
    for (;;) {
        b += gridDim.x;
        const bool more = seek(b);
        const ChunkDev cn = ch;
        const int64_t fn = (b - cb0) * BF + threadIdx.x * 4;
        if (more) analog_load8(in + (cn.in_off + fn) * 2, fn, cn.n, (cn.in_off & 1) == 0, xb);
        if (f < cc.n) work(cc, xa, f);
        if (!more) break;
        cc = cn;
        f = fn;
        b += gridDim.x;
        const bool more2 = seek(b);
        const ChunkDev cn2 = ch;
        const int64_t fn2 = (b - cb0) * BF + threadIdx.x * 4;
        if (more2) analog_load8(in + (cn2.in_off + fn2) * 2, fn2, cn2.n, (cn2.in_off & 1) == 0, xa);
        if (f < cc.n) work(cc, xb, f);
        if (!more2) break;
        cc = cn2;
        f = fn2;
    }
#endif
}

// EQ pass 1 over the s16 stereo chain input a16 (after k_analog_h): the GEMV of
// k_front1s without the input conversion -- two threads per segment, each holding both
// channels' accumulators for half of the D state components, G tiles through LDS.  A
// row's 16-frame tile is 64 B: lane t loads 16-B piece t % 4 of rows t / 4 + 64 m
// (chunk rows are 16-frame aligned); frames at or past a row's length load as 0.  The
// accumulation order is k_front1s's, so e is the same to the bit.
#define AMX_G16_PITCH (AMX_TF + 4)   // dwords per LDS row (16-B aligned rows)
template <int D>
__global__ void __launch_bounds__(AMX_BLOCK, 4) k_gemv16(const ChainDev *__restrict__ cdp,
                                                         const ChunkDev *__restrict__ chunks,
                                                         const SegDev *__restrict__ segs,
                                                         int n_seg, int L,
                                                         const uint32_t *__restrict__ a16,
                                                         const double *__restrict__ G,
                                                         double *__restrict__ e) {
    constexpr int ROWS = AMX_BLOCK / 2;
    constexpr int H = D / 2;
    constexpr int GQ = AMX_TF * D / 2;                  // 16-B pieces of a G tile
    static_assert(GQ <= AMX_BLOCK && D % 2 == 0 && D > 0, "tile shape");
    __shared__ __attribute__((aligned(16))) uint32_t s_in[ROWS * AMX_G16_PITCH];
    __shared__ __attribute__((aligned(16))) double sG[AMX_TF * D];
    __shared__ int64_t rb[ROWS];
    __shared__ int rl[ROWS];
    const int t = threadIdx.x, row = t >> 1, half = t & 1;
    const int j = blockIdx.x * ROWS + row;
    const bool valid = j < n_seg;
    const SegDev sg = segs[valid ? j : n_seg - 1];
    if (half == 0) {
        rb[row] = valid ? chunks[sg.chunk].loc_off + sg.pos : 0;
        rl[row] = valid ? sg.len : 0;
    }
    __syncthreads();
    const int c4 = 4 * (t & 3);
    const uint32_t *ip[2];
    int ilen[2];
#pragma unroll
    for (int m = 0; m < 2; m++) {
        ip[m] = a16 + rb[(t >> 2) + 64 * m] + c4;
        ilen[m] = rl[(t >> 2) + 64 * m];
    }
    uint4 R[2], RG;
    // (AMX_VT_LATE, as vt_fetch / vt_put: the loads alone in fetch, the masks at the put,
    // an unconditional fetch -- so the next tile's loads stay in flight over this tile)
    auto fetch = [&](int k) {
#if AMX_VT_LATE
        RG = *reinterpret_cast<const uint4 *>(G + (int64_t)k * D + 2 * (t < GQ ? t : 0));
#else
        RG = t < GQ ? *reinterpret_cast<const uint4 *>(G + (int64_t)k * D + 2 * t) : make_uint4(0u, 0u, 0u, 0u);
#endif
#pragma unroll
        for (int m = 0; m < 2; m++) {
            const int n = k + c4;
            uint4 v = *reinterpret_cast<const uint4 *>(ip[m] + (n < ilen[m] ? k : 0));
#if !AMX_VT_LATE
            v.x = n < ilen[m] ? v.x : 0u;
            v.y = n + 1 < ilen[m] ? v.y : 0u;
            v.z = n + 2 < ilen[m] ? v.z : 0u;
            v.w = n + 3 < ilen[m] ? v.w : 0u;
#endif
            R[m] = v;
        }
    };
    double a0[H], a1[H];
#pragma unroll
    for (int d = 0; d < H; d++) { a0[d] = 0.0; a1[d] = 0.0; }
    fetch(0);
    const uint32_t *rp = s_in + row * AMX_G16_PITCH;
    for (int k = 0; k < L; k += AMX_TF) {
#pragma unroll
        for (int m = 0; m < 2; m++) {
            uint4 v = R[m];
#if AMX_VT_LATE
            const int n = k + c4;
            v.x = n < ilen[m] ? v.x : 0u;
            v.y = n + 1 < ilen[m] ? v.y : 0u;
            v.z = n + 2 < ilen[m] ? v.z : 0u;
            v.w = n + 3 < ilen[m] ? v.w : 0u;
#endif
            *reinterpret_cast<uint4 *>(s_in + ((t >> 2) + 64 * m) * AMX_G16_PITCH + c4) = v;
        }
        if (t < GQ) reinterpret_cast<uint4 *>(sG)[t] = RG;
        __syncthreads();
#if AMX_VT_LATE
        fetch(k + AMX_TF < L ? k + AMX_TF : k);
#else
        if (k + AMX_TF < L) fetch(k + AMX_TF);
#endif
#pragma unroll 1
        for (int f = 0; f < AMX_TF; f++) {
            const uint32_t w = rp[f];
            const double x0 = (double)((float)lo16(w) / 32768.0f);
            const double x1 = (double)((float)hi16(w) / 32768.0f);
            const double *g = sG + f * D + half * H;
#pragma unroll
            for (int d = 0; d < H; d++) {
                a0[d] = fma(g[d], x0, a0[d]);
                a1[d] = fma(g[d], x1, a1[d]);
            }
        }
        __syncthreads();
    }
    if (valid && !sg.last) {
        double *eo = e + (int64_t)j * 2 * D + half * H;
#pragma unroll
        for (int d = 0; d < H; d++) { eo[d] = a0[d]; eo[D + d] = a1[d]; }
    }
}

// ------------------------------------------- pass 2: EQ from true state -> int16
// One thread per (segment, channel): lanes 2i / 2i+1 are the L / R channel of row
// i.  The EQ runs stage-major over sub-tiles of AMX_EQ_F frames (eq_tile), so only
// one stage's coefficients and a few frames are live: ~90 VGPRs, 5 waves/SIMD to
// cover the fp64 recursion latency.  Width couples the channels: the pair
// exchanges its float32 EQ output with one DPP swap per frame.  Tiles are fetched
// one ahead (tile_fetch / tile_put).
// MB: also accumulate the crossover's zero-state end state (GEMV) for its scan.
// KW (no multiband, K-filter segments == these segments): also the loudness pass-1
// work on the output just produced -- the K filter's zero-state end state (GEMV
// over Gkw, right-aligned for a span's final partial segment like k_kw1) and the
// per-(segment, channel) sample peak -- so the track is not read again for it.
#define AMX_EQ_F 4   // frames per stage-major sub-tile (must divide AMX_TF)
// Wave-local 16-B tile mover (rows of AMX_TF frames x 4 B, chunk rows 16-frame
// aligned; a store row that is not falls back to dwords): the wave's 32 rows, mover lane l moves 16-B piece l % 4 (frames
// 4 (l % 4) .. + 3) of rows l / 4 and l / 4 + 16 -- two vector loads / stores per
// lane per tile from row offsets formed once, instead of a dword per element with
// its row offset and bound re-read from LDS (tile_fetch / tile_store).  Frames at or
// past a row's length load as 0 and are not stored.
#define AMX_VT_PITCH 20   // dwords per LDS row (16-B aligned rows)
typedef uint32_t vt4 __attribute__((ext_vector_type(4)));
struct VRows {
    int32_t base[2];      // dword offset of the row's frame 0 (an invalid row: 0; plans
                          // hold < 2^31 frames, amx_plan_create)
    int len[2];           // frames in the row (an invalid row: 0)
};

// AMX_VT_LATE: the frames past a row's length are zeroed when the tile is put into LDS,
// not right after its load -- a select beside the load made the compiler wait for the
// prefetched tile at once (vmcnt(0) right after the fetch: no overlap with the tile's
// compute); and the fetch is unconditional (the last one re-reads the current tile), so
// every pass through the tile loop issues the same memory operations
__device__ __forceinline__ void vt_fetch(vt4 (&R)[2], const uint32_t *__restrict__ src, const VRows &vr,
                                         int k) {
    const int c4 = 4 * (threadIdx.x & 3);
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const int n = k + c4;
        const bool ok = n < vr.len[i];
        vt4 v = *reinterpret_cast<const vt4 *>(src + vr.base[i] + (ok ? n : 0));
#if !AMX_VT_LATE
#pragma unroll
        for (int e = 0; e < 4; e++) v[e] = n + e < vr.len[i] ? v[e] : 0u;
#endif
        R[i] = v;
    }
}

// the tile of frames k .. k + AMX_TF - 1 (vt_fetch's R) into LDS
__device__ __forceinline__ void vt_put(uint32_t *lds, const vt4 (&R)[2], const VRows &vr, int k) {
    const int r0 = (threadIdx.x & 63) >> 2, c4 = 4 * (threadIdx.x & 3);
    vt4 v0 = R[0], v1 = R[1];
#if AMX_VT_LATE
    const int n = k + c4;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        v0[e] = n + e < vr.len[0] ? v0[e] : 0u;
        v1[e] = n + e < vr.len[1] ? v1[e] : 0u;
    }
#endif
    *reinterpret_cast<vt4 *>(lds + r0 * AMX_VT_PITCH + c4) = v0;
    *reinterpret_cast<vt4 *>(lds + (r0 + 16) * AMX_VT_PITCH + c4) = v1;
}

// the next tile's fetch: unconditional with AMX_VT_LATE (past the last tile it re-reads tile k)
__device__ __forceinline__ void vt_next(vt4 (&R)[2], const uint32_t *__restrict__ src, const VRows &vr,
                                        int k, int L) {
#if AMX_VT_LATE
    vt_fetch(R, src, vr, k + AMX_TF < L ? k + AMX_TF : k);
#else
    if (k + AMX_TF < L) vt_fetch(R, src, vr, k + AMX_TF);
#endif
}

__device__ __forceinline__ void vt_store(const uint32_t *lds, uint32_t *__restrict__ dst, const VRows &vr,
                                         int k) {
    const int r0 = (threadIdx.x & 63) >> 2, c4 = 4 * (threadIdx.x & 3);
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const vt4 v = *reinterpret_cast<const vt4 *>(lds + (r0 + 16 * i) * AMX_VT_PITCH + c4);
        const int n = k + c4;
        uint32_t *d = dst + vr.base[i] + n;
        if (n + 4 <= vr.len[i] && (vr.base[i] & 3) == 0) {   // (d_out rows need not be 16-B aligned)
            *reinterpret_cast<vt4 *>(d) = v;
        } else {
#pragma unroll
            for (int e = 0; e < 4; e++)
                if (n + e < vr.len[i]) d[e] = v[e];
        }
    }
}

// the mover rows of this lane, from the compute lanes (lane 2 r holds row r's offset)
__device__ __forceinline__ VRows vt_rows(int32_t base, int len) {
    VRows vr;
    const int r0 = (threadIdx.x & 63) >> 2;
#pragma unroll
    for (int i = 0; i < 2; i++) {
        vr.base[i] = __shfl(base, 2 * (r0 + 16 * i));
        vr.len[i] = __shfl(len, 2 * (r0 + 16 * i));
    }
    return vr;
}

// SC: a stream chain (amx_chain_desc.stream_chain; no width): the input through slut
// when given (as k_front1), and the EQ's float64 result clipped and scaled in float64
// (:273-275 keep a 1-D stream's float64 result; float32 only when no stage ran)
template <int MASK, bool MB, bool KW, bool SC = false>
__global__ void __launch_bounds__(AMX_BLOCK, (MB || KW) ? 4 : 5) k_front2(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const SegDev *__restrict__ segs, int n_seg,
                                                      int L, const uint32_t *__restrict__ a16,
                                                      const double *__restrict__ s_eq,
                                                      uint32_t *__restrict__ dst, int to_out,
                                                      const double *__restrict__ Gx,
                                                      double *__restrict__ e_x,
                                                      const double *__restrict__ Gkw,
                                                      double *__restrict__ e_kw,
                                                      uint32_t *__restrict__ pk,
                                                      const float *__restrict__ slut) {
    constexpr int D = EqDim<MASK>::v;
    constexpr int ROWS = AMX_BLOCK / 2;
    constexpr int WV = AMX_BLOCK / 64;
    __shared__ __attribute__((aligned(16))) uint32_t s_in_all[WV][32 * AMX_VT_PITCH];
    __shared__ __attribute__((aligned(16))) uint32_t s_out_all[WV][32 * AMX_VT_PITCH];
    __shared__ int2 s_orow[WV][32];   // per row: output dword offset, frames (read at the store)
    const ChainDev &cd = *cdp;
    const int t = threadIdx.x, wv = t >> 6, row = (t & 63) >> 1, chn = t & 1;
    const int j = blockIdx.x * ROWS + wv * 32 + row;
    bool need_x = false;
    int32_t b_in = 0, b_out = 0;
    int len = 0;
    double z[D > 0 ? D : 1];
#pragma unroll
    for (int d = 0; d < D; d++) z[d] = 0.0;
    if (j < n_seg) {
        const SegDev sg = segs[j];
        const ChunkDev ch = chunks[sg.chunk];
        b_in = (int32_t)(ch.loc_off + sg.pos);
        b_out = (int32_t)((to_out ? ch.out_off : ch.loc_off) + sg.pos);
        len = sg.len;
        need_x = MB && !sg.last;
        if constexpr (D > 0) {
            const double *s = s_eq + ((int64_t)j * 2 + chn) * D;
#pragma unroll
            for (int d = 0; d < D; d++) z[d] = s[d];
        }
    }
    EqState est;
    eq_state_load<MASK>(est, z);
    double xv[MB ? AMX_XO_DIM : 1];
#pragma unroll
    for (int d = 0; d < (MB ? AMX_XO_DIM : 1); d++) xv[d] = 0.0;
    double kv[KW ? AMX_KW_DIM : 1];
#pragma unroll
    for (int d = 0; d < (KW ? AMX_KW_DIM : 1); d++) kv[d] = 0.0;
    int kmax = 0;
    const int klen = (j < n_seg) ? segs[j].len : 0;
    const int negm = (cd.st[0].neg ? 1 : 0) | (cd.st[3].neg ? 8 : 0);
    const float w = cd.width;
    const int won = cd.width_on;
    // tiles are wave-local: a wave stages, computes and stores only its own 32 rows
    // (the vector mover), so it never waits for the other waves of the workgroup
    const VRows vin = vt_rows(b_in, len);
    if (chn == 0) s_orow[wv][row] = make_int2(b_out, len);
    uint32_t *s_in = s_in_all[wv], *s_out = s_out_all[wv];
    vt4 R[2];
    vt_fetch(R, a16, vin, 0);
    for (int k = 0; k < L; k += AMX_TF) {
        vt_put(s_in, R, vin, k);
        amx_wave_sync();
        vt_next(R, a16, vin, k, L);
        const uint32_t *rp = s_in + row * AMX_VT_PITCH;
        uint32_t *op = s_out + row * AMX_VT_PITCH;
#pragma unroll 1
        for (int f0 = 0; f0 < AMX_TF; f0 += AMX_EQ_F) {
            float xf[AMX_EQ_F];
            double x[AMX_EQ_F];
#pragma unroll
            for (int f = 0; f < AMX_EQ_F; f++) {
                const uint32_t p = rp[f0 + f];
                const int16_t sv = chn ? hi16(p) : lo16(p);
                if constexpr (SC) xf[f] = slut ? slut[(int)sv + 32768] : (float)sv / 32768.0f;
                else xf[f] = (float)sv / 32768.0f;
                x[f] = (double)xf[f];
            }
            // cd.pad0_ == 0: the offset makes the coefficient address depend on the
            // loop, so the scalar loads stay per tile (no hoisting, no SGPR spill)
            eq_tile<MASK, AMX_EQ_F>(negm, cd.eqc + (f0 & cd.pad0_), est, x, xf);
#pragma unroll
            for (int f = 0; f < AMX_EQ_F; f++) {
                int16_t qv;
                if constexpr (SC) {
                    qv = MASK ? f64_to_s16(x[f]) : f32_to_s16(xf[f]);
                } else {
                    float v = MASK ? (float)x[f] : xf[f];
                    if (won) {
                        const float o = pair_swap(v);
                        v = width_one(w, chn ? o : v, chn ? v : o, chn);
                    }
                    qv = f32_to_s16(v);
                }
                const int other = __builtin_amdgcn_update_dpp(0, (int)qv, 0xB1, 0xF, 0xF, false);
                if (chn == 0) op[f0 + f] = pack2(qv, (int16_t)other);
                if constexpr (MB) {
                    const double *g = Gx + (int64_t)(k + f0 + f) * AMX_XO_DIM;
                    const double xd = (double)((float)qv / 32768.0f);
#pragma unroll
                    for (int d = 0; d < AMX_XO_DIM; d++) xv[d] = fma(g[d], xd, xv[d]);
                }
                if constexpr (KW) {
                    // rows are used as if every segment were L long (a wave-uniform row:
                    // scalar loads, SGPR operands); a span's partial last segment is
                    // re-done right-aligned by k_peak_reduce (kw_fix)
                    const int n = k + f0 + f;
                    const bool act = n < klen;
                    kmax = max(kmax, act ? abs((int)qv) : 0);
                    const double xs = act ? (double)qv * (1.0 / 32768.0) : 0.0;
                    const double *g = Gkw + (int64_t)n * AMX_KW_DIM;
#pragma unroll
                    for (int d = 0; d < AMX_KW_DIM; d++) kv[d] = fma(g[d], xs, kv[d]);
                }
            }
        }
        amx_wave_sync();
        {
            // the output rows from LDS: kept in registers they spill the 5-wave variants
            const int r0 = (t & 63) >> 2;
            const int2 o0 = s_orow[wv][r0], o1 = s_orow[wv][r0 + 16];
            VRows vout;
            vout.base[0] = o0.x; vout.len[0] = o0.y;
            vout.base[1] = o1.x; vout.len[1] = o1.y;
            vt_store(s_out, dst, vout, k);
        }
        amx_wave_sync();                    // s_in / s_out are rewritten by the next tile
    }
    if constexpr (MB) {
        if (need_x) {
            double *o = e_x + ((int64_t)j * 2 + chn) * AMX_XO_DIM;
#pragma unroll
            for (int d = 0; d < AMX_XO_DIM; d++) o[d] = xv[d];
        }
    }
    if constexpr (KW) {
        if (j < n_seg) {
            double *o = e_kw + ((int64_t)j * 2 + chn) * AMX_KW_DIM;
#pragma unroll
            for (int d = 0; d < AMX_KW_DIM; d++) o[d] = kv[d];
            pk[(int64_t)j * 2 + chn] = (uint32_t)kmax;
        }
    }
}

// ------------------------------------------------ crossover pass 2 -> 3 bands
// One thread per (segment, channel); mid = (x - low) - high in float64 (:304).
// Wave-local tiles through the vector mover; the L lane writes the low and mid
// pairs, the R lane the high pair.
__global__ void __launch_bounds__(AMX_BLOCK) k_xover2(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const SegDev *__restrict__ segs, int n_seg,
                                                      int L, const uint32_t *__restrict__ p16,
                                                      const double *__restrict__ s_x,
                                                      uint32_t *__restrict__ bands, int64_t nloc,
                                                      int *__restrict__ bact) {
    constexpr int WV = AMX_BLOCK / 64;
    __shared__ __attribute__((aligned(16))) uint32_t s_in[WV][32 * AMX_VT_PITCH];
    __shared__ __attribute__((aligned(16))) uint32_t s_b[WV][2][32 * AMX_VT_PITCH];
    __shared__ double s_c[24];
    const ChainDev &cd = *cdp;
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63, row = lane >> 1, chn = lane & 1;
    const int j = blockIdx.x * (AMX_BLOCK / 2) + wv * 32 + row;
    if (t < 12) s_c[t] = cd.xlo[t];
    else if (t < 24) s_c[t] = cd.xhi[t - 12];
    // the step's band-activity words start clear (k_rms sets them; amx_dyn.hip)
    if (blockIdx.x == 0 && t < 3) bact[t] = 0;
    double z[AMX_XO_DIM];
#pragma unroll
    for (int d = 0; d < AMX_XO_DIM; d++) z[d] = 0.0;
    int32_t base = 0;
    int len = 0;
    if (j < n_seg) {
        const SegDev sg = segs[j];
        const ChunkDev ch = chunks[sg.chunk];
        base = (int32_t)(ch.loc_off + sg.pos);
        len = sg.len;
        const double *s = s_x + ((int64_t)j * 2 + chn) * AMX_XO_DIM;
#pragma unroll
        for (int d = 0; d < AMX_XO_DIM; d++) z[d] = s[d];
    }
    const VRows vr = vt_rows(base, len);
    __syncthreads();
    double c[20];   // 4 sections x (b0 b1 b2 a1 a2): low 1, low 2, high 1, high 2
#pragma unroll
    for (int sc = 0; sc < 4; sc++) {
        c[5 * sc + 0] = s_c[6 * sc + 0];
        c[5 * sc + 1] = s_c[6 * sc + 1];
        c[5 * sc + 2] = s_c[6 * sc + 2];
        c[5 * sc + 3] = s_c[6 * sc + 4];
        c[5 * sc + 4] = s_c[6 * sc + 5];
    }
    // the high band goes back through the input tile (read into registers first)
    uint32_t *si = s_in[wv], *slo = s_b[wv][0], *smi = s_b[wv][1], *shi = si;
    vt4 R[2];
    vt_fetch(R, p16, vr, 0);
    for (int k = 0; k < L; k += AMX_TF) {
        vt_put(si, R, vr, k);
        amx_wave_sync();
        vt_next(R, p16, vr, k, L);
        uint32_t xin[AMX_TF];
#pragma unroll
        for (int q = 0; q < AMX_TF / 4; q++) {
            const vt4 v = *reinterpret_cast<const vt4 *>(si + row * AMX_VT_PITCH + 4 * q);
            xin[4 * q] = v.x; xin[4 * q + 1] = v.y; xin[4 * q + 2] = v.z; xin[4 * q + 3] = v.w;
        }
        const int o = row * AMX_VT_PITCH;
#pragma unroll 4
        for (int f = 0; f < AMX_TF; f++) {
            const uint32_t p = xin[f];
            const int16_t v = chn ? hi16(p) : lo16(p);
            const double x = (double)((float)v / 32768.0f);   // :300 float32 then float64
            double l = bq_step(c, z[0], z[1], x);
            l = bq_step(c + 5, z[2], z[3], l);
            double h = bq_step(c + 10, z[4], z[5], x);
            h = bq_step(c + 15, z[6], z[7], h);
            const double m = (x - l) - h;                      // :304
            const int ql = f64_to_s16(l), qm = f64_to_s16(m), qh = f64_to_s16(h);
            const int ol = __builtin_amdgcn_update_dpp(0, ql, 0xB1, 0xF, 0xF, false);
            const int om = __builtin_amdgcn_update_dpp(0, qm, 0xB1, 0xF, 0xF, false);
            const int oh = __builtin_amdgcn_update_dpp(0, qh, 0xB1, 0xF, 0xF, false);
            if (chn == 0) {
                slo[o + f] = pack2((int16_t)ql, (int16_t)ol);
                smi[o + f] = pack2((int16_t)qm, (int16_t)om);
            } else {
                shi[o + f] = pack2((int16_t)oh, (int16_t)qh);
            }
        }
        amx_wave_sync();
        vt_store(slo, bands, vr, k);
        vt_store(smi, bands + nloc, vr, k);
        vt_store(shi, bands + 2 * nloc, vr, k);
        amx_wave_sync();
    }
}

// ================================================================ launchers
template <int D, int WIN, bool AN, bool SC = false>
static hipError_t front1_t(const Launch &l, const uint32_t *in, const float *lut, uint32_t *a16,
                           const double *G, double *e) {
    hipLaunchKernelGGL((k_front1<D, WIN, AN, SC>), grid1(l.n_seg), dim3(AMX_BLOCK), 0, l.stream, l.cd,
                       l.chunks, l.segs, l.n_seg, l.L, in, lut, a16, G, e);
    return hipGetLastError();
}

static int cu_count() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

template <int D, bool AN>
static hipError_t front1s_t(const Launch &l, const uint32_t *in, const float *lut, uint32_t *a16,
                            const double *G, double *e) {
    const int rows = AMX_BLOCK / 2;
    if constexpr (AN) {
        if (l.f1_mode == AMX_F1_SPLIT && l.lut_half) {
            // analog as an elementwise pass (the half table in LDS), then the GEMV over its
            // s16 output; else (a tanh table that is not odd) k_front1s with the full table
            const int64_t wgs = l.an_blocks;
            const dim3 gh((unsigned)(wgs < cu_count() ? (wgs > 0 ? wgs : 1) : cu_count()));
            const bool vec = AMX_AN_VEC && l.an_vec && (reinterpret_cast<uintptr_t>(in) & 15) == 0;
            if (vec)
                hipLaunchKernelGGL(k_analog_h<true>, gh, dim3(1024), 0, l.stream, l.cd, l.chunks, l.n_chunks,
                                   reinterpret_cast<const float *>(in), l.lut_half, a16, l.an_blocks);
            else
                hipLaunchKernelGGL(k_analog_h<false>, gh, dim3(1024), 0, l.stream, l.cd, l.chunks, l.n_chunks,
                                   reinterpret_cast<const float *>(in), l.lut_half, a16, l.an_blocks);
            if constexpr (D > 0) {
                hipLaunchKernelGGL((k_gemv16<D>), dim3((unsigned)((l.n_seg + rows - 1) / rows)), dim3(AMX_BLOCK), 0,
                                   l.stream, l.cd, l.chunks, l.segs, l.n_seg, l.L, a16, G, e);
            }
            return hipGetLastError();
        }
    }
    dim3 grid((unsigned)((l.n_seg + rows - 1) / rows));
    hipLaunchKernelGGL((k_front1s<D, AN>), grid, dim3(AMX_BLOCK), 0, l.stream, l.cd, l.chunks,
                       l.segs, l.n_seg, l.L, in, lut, a16, G, e);
    return hipGetLastError();
}

template <int D, int WIN>
static hipError_t front1_an(const Launch &l, bool an, const uint32_t *in, const float *lut,
                            uint32_t *a16, const double *G, double *e) {
    if constexpr (WIN == 2) {
        if (l.L % AMX_TF) return hipErrorInvalidValue;
        return an ? front1s_t<D, true>(l, in, lut, a16, G, e)
                  : front1s_t<D, false>(l, in, lut, a16, G, e);
    }
    return an ? front1_t<D, WIN, true>(l, in, lut, a16, G, e)
              : front1_t<D, WIN, false>(l, in, lut, a16, G, e);
}

hipError_t launch_front1(const Launch &l, int D, int win, bool analog, const float *in,
                         const float *lut, int16_t *a16, const double *G, double *e, bool sc) {
    if (l.n_seg <= 0) return hipSuccess;
    if (analog && !lut) return hipErrorInvalidValue;
    if (sc && (analog || win != 1)) return hipErrorInvalidValue;   // a stream chain reads int16 pairs
    const uint32_t *i32 = reinterpret_cast<const uint32_t *>(in);
    uint32_t *a = reinterpret_cast<uint32_t *>(a16);
#define F1(DD)                                                                   \
    case DD:                                                                     \
        if (sc) return front1_t<DD, 1, false, true>(l, i32, lut, a, G, e);       \
        return win == 2 ? front1_an<DD, 2>(l, analog, i32, lut, a, G, e)         \
                        : front1_an<DD, 1>(l, analog, i32, lut, a, G, e);
    switch (D) { F1(0) F1(2) F1(4) F1(8) F1(10) F1(12) F1(16) F1(18) F1(20) }
#undef F1
    return hipErrorInvalidValue;
}

template <int MASK, bool MB, bool KW, bool SC = false>
static hipError_t front2_t(const Launch &l, const uint32_t *a16, const double *s_eq,
                           uint32_t *dst, int to_out, const double *Gx, double *e_x,
                           const double *Gkw, double *e_kw, uint32_t *pk, const float *slut = nullptr) {
    const int rows = AMX_BLOCK / 2;
    dim3 grid((unsigned)((l.n_seg + rows - 1) / rows));
    hipLaunchKernelGGL((k_front2<MASK, MB, KW, SC>), grid, dim3(AMX_BLOCK), 0, l.stream, l.cd,
                       l.chunks, l.segs, l.n_seg, l.L, a16, s_eq, dst, to_out, Gx, e_x, Gkw, e_kw,
                       pk, slut);
    return hipGetLastError();
}

#define AMX_MASK_CASES(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

hipError_t launch_front2(const Launch &l, int mask, const int16_t *a16, const double *s_eq,
                         int16_t *dst, int to_out, const double *Gx, double *e_x,
                         const double *Gkw, double *e_kw, uint32_t *pk, bool sc, const float *slut) {
    if (l.n_seg <= 0) return hipSuccess;
    const uint32_t *a = reinterpret_cast<const uint32_t *>(a16);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    const bool mb = Gx != nullptr, kw = Gkw != nullptr;
    if (mb && kw) return hipErrorInvalidValue;
    if (sc && kw) return hipErrorInvalidValue;          // a stream chain measures elsewhere
    switch (mask) {
#define C2(M)                                                                           \
    case M:                                                                             \
        if (sc) return mb ? front2_t<M, true, false, true>(l, a, s_eq, d, to_out, Gx, e_x, Gkw, e_kw, pk, slut) \
                          : front2_t<M, false, false, true>(l, a, s_eq, d, to_out, Gx, e_x, Gkw, e_kw, pk, slut); \
        return mb ? front2_t<M, true, false>(l, a, s_eq, d, to_out, Gx, e_x, Gkw, e_kw, pk) \
             : kw ? front2_t<M, false, true>(l, a, s_eq, d, to_out, Gx, e_x, Gkw, e_kw, pk) \
                  : front2_t<M, false, false>(l, a, s_eq, d, to_out, Gx, e_x, Gkw, e_kw, pk);
        AMX_MASK_CASES(C2)
#undef C2
    }
    return hipErrorInvalidValue;
}

hipError_t launch_xover2(const Launch &l, const int16_t *p16, const double *s_x,
                         int16_t *bands, int64_t nloc, int *bact) {
    if (l.n_seg <= 0) return hipSuccess;
    const int rows = AMX_BLOCK / 2;
    dim3 grid((unsigned)((l.n_seg + rows - 1) / rows));
    hipLaunchKernelGGL(k_xover2, grid, dim3(AMX_BLOCK), 0, l.stream, l.cd, l.chunks, l.segs,
                       l.n_seg, l.L, reinterpret_cast<const uint32_t *>(p16), s_x,
                       reinterpret_cast<uint32_t *>(bands), nloc, bact);
    return hipGetLastError();
}

}  // namespace amx
