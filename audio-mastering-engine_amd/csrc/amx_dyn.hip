// amx_dyn.hip -- multiband compressor dynamics (pydub compress_dynamic_range,
// audio_mastering_engine.py:306-308) and the overlay (:309).
#include "amx_dev.hpp"

namespace amx {

// --------------------------------------------- compressor RMS detector (exact)
// r_i = audioop.rms of frames [max(i-look,0), i) of the band, both channels:
// (unsigned)sqrt(S / count) with S the exact integer sum of squares.
__global__ void __launch_bounds__(AMX_BLOCK) k_rms(const ChainDev *__restrict__ cdp,
                                                   const ChunkDev *__restrict__ chunks,
                                                   const SegDev *__restrict__ segs, int n_seg,
                                                   const uint32_t *__restrict__ bands,
                                                   uint16_t *__restrict__ rr, int64_t nloc) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    int b = blockIdx.y;
    if (j >= n_seg) return;
    const int look = cdp->look;
    const SegDev sg = segs[j];
    const ChunkDev ch = chunks[sg.chunk];
    const uint32_t *x = bands + b * nloc + ch.loc_off;
    uint16_t *r = rr + b * nloc + ch.loc_off;
    const int64_t p0 = sg.pos;
    int64_t lo = p0 - look < 0 ? 0 : p0 - look;
    int64_t S = 0;
    for (int64_t f = lo; f < p0; f++) {
        uint32_t v = x[f];
        int64_t a = lo16(v), c = hi16(v);
        S += a * a + c * c;
    }
    for (int n = 0; n < sg.len; n++) {
        int64_t i = p0 + n;
        int64_t wlo = i - look < 0 ? 0 : i - look;
        int64_t cnt = 2 * (i - wlo);
        uint32_t rms = cnt ? (uint32_t)sqrt((double)S / (double)cnt) : 0u;
        r[i] = (uint16_t)(rms > 65535u ? 65535u : rms);
        // slide: add frame i, drop frame i-look
        uint32_t v = x[i];
        int64_t a = lo16(v), c = hi16(v);
        S += a * a + c * c;
        if (i - look >= 0) {
            uint32_t u = x[i - look];
            int64_t a2 = lo16(u), c2 = hi16(u);
            S -= a2 * a2 + c2 * c2;
        }
    }
}

// pydub envelope step (compress_dynamic_range inner loop), exact.
__device__ __forceinline__ double env_step(double att, bool over, double m, double inc,
                                           double dec) {
    if (over && att <= m) {
        att = att + inc;
        att = (m < att) ? m : att;          // min(attenuation, max_attenuation)
    } else {
        att = att - dec;
        att = (0.0 > att) ? 0.0 : att;      // max(attenuation, 0)
    }
    return att;
}

#define AMX_TAB 32769
// speculative envelope: guess from a warm-up started at att = 0
__global__ void __launch_bounds__(AMX_BLOCK) k_env(const ChainDev *__restrict__ cdp,
                                                   const ChunkDev *__restrict__ chunks,
                                                   const SegDev *__restrict__ segs, int n_seg,
                                                   const uint16_t *__restrict__ rr,
                                                   const double *__restrict__ tabs,
                                                   double *__restrict__ att_out,
                                                   double *__restrict__ guess,
                                                   double *__restrict__ endv, int64_t nloc,
                                                   int warm) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    int b = blockIdx.y;
    if (j >= n_seg) return;
    const SegDev sg = segs[j];
    const ChunkDev ch = chunks[sg.chunk];
    const uint16_t *r = rr + b * nloc + ch.loc_off;
    double *ao = att_out + b * nloc + ch.loc_off;
    const double *mt = tabs + (int64_t)b * 3 * AMX_TAB;
    const double *it = mt + AMX_TAB, *dt = mt + 2 * AMX_TAB;
    const int rthr = cdp->rthr[b];
    double att = 0.0;
    int64_t w0 = sg.pos - warm;
    if (w0 < 0) w0 = 0;
    for (int64_t f = w0; f < sg.pos; f++) {
        int rv = r[f];
        att = env_step(att, rv >= rthr, mt[rv], it[rv], dt[rv]);
    }
    guess[(int64_t)b * n_seg + j] = att;
    for (int n = 0; n < sg.len; n++) {
        int rv = r[sg.pos + n];
        att = env_step(att, rv >= rthr, mt[rv], it[rv], dt[rv]);
        ao[sg.pos + n] = att;
    }
    endv[(int64_t)b * n_seg + j] = att;
}

// verification / fix-up: one wave per (chunk, band).  Walks the chunk's segment
// hand-offs; each mismatch (guess_j != end_{j-1}) is re-run from the exact start
// until the new trajectory coincides with the stored one.
__global__ void __launch_bounds__(64) k_fix(const ChainDev *__restrict__ cdp,
                                            const ChunkDev *__restrict__ chunks,
                                            const SegDev *__restrict__ segs, int n_seg,
                                            const uint16_t *__restrict__ rr,
                                            const double *__restrict__ tabs,
                                            double *__restrict__ att_arr,
                                            double *__restrict__ guess,
                                            double *__restrict__ endv, int64_t nloc) {
    const int c = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    const ChunkDev ch = chunks[c];
    const uint16_t *r = rr + b * nloc + ch.loc_off;
    double *aa = att_arr + b * nloc + ch.loc_off;
    double *gs = guess + (int64_t)b * n_seg;
    double *en = endv + (int64_t)b * n_seg;
    const double *mt = tabs + (int64_t)b * 3 * AMX_TAB;
    const double *it = mt + AMX_TAB, *dt = mt + 2 * AMX_TAB;
    const int rthr = cdp->rthr[b];
    const int s0 = ch.seg0, s1 = ch.seg0 + ch.nseg;
    int cur = s0 + 1;
    while (true) {
        int found = 0x7fffffff;
        for (int base = cur; base < s1; base += 64) {
            int jj = base + lane;
            bool bad = false;
            if (jj < s1) bad = !(gs[jj] == en[jj - 1]);
            unsigned long long m = __ballot(bad);
            if (m) { found = base + __ffsll((long long)m) - 1; break; }
        }
        if (found >= s1) break;
        const SegDev sg = segs[found];
        double att = en[found - 1];
        bool coincided = false;
        for (int base = 0; base < sg.len && !coincided; base += 64) {
            const int n = base + lane;
            const bool valid = n < sg.len;
            const int64_t f = sg.pos + n;
            int rv = valid ? (int)r[f] : 0;
            double mv = mt[rv], iv = it[rv], dv = dt[rv];
            bool over = valid && rv >= rthr;
            double old = valid ? aa[f] : 0.0;
            double nv;
            if (__ballot(over) == 0ull) {
                nv = att;                       // below threshold: state held
            } else {
                nv = 0.0;
                const int cnt = sg.len - base < 64 ? sg.len - base : 64;
                for (int k = 0; k < cnt; k++) {
                    double mk = __shfl(mv, k), ik = __shfl(iv, k), dk = __shfl(dv, k);
                    int ok = __shfl((int)over, k);
                    att = env_step(att, ok != 0, mk, ik, dk);
                    if (lane == k) nv = att;
                }
            }
            unsigned long long same = __ballot(valid && nv == old);
            if (same) {
                int k = __ffsll((long long)same) - 1;
                if (valid && lane < k) aa[f] = nv;
                coincided = true;
            } else if (valid) {
                aa[f] = nv;
            }
        }
        if (!coincided && lane == 0) en[found] = att;
        if (lane == 0) gs[found] = en[found - 1];
        __threadfence_block();
        __syncthreads();
        cur = found + 1;
    }
}

// audioop.mul clamp + floor (CPython Modules/audioop.c fbound)
__device__ __forceinline__ int mul16(int v, double f) {
    double val = (double)v * f;
    if (val > 32767.0) val = 32767.0;
    else if (val < -32768.0 + 1.0) val = -32768.0;
    return (int)floor(val);
}

// gains + overlay (:306-309) -> chunk output (pydub ms-rounded length)
__global__ void __launch_bounds__(AMX_BLOCK) k_apply(const ChunkDev *__restrict__ chunks,
                                                     const uint32_t *__restrict__ bands,
                                                     const double *__restrict__ att,
                                                     uint32_t *__restrict__ out, int64_t nloc,
                                                     const int64_t *__restrict__ n2tab) {
    const int c = blockIdx.y;
    const ChunkDev ch = chunks[c];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n2 = ch.out_n;            // final (second overlay) length
    if (i >= n2) return;
    const int64_t n1 = n2tab[c];            // first overlay length
    uint32_t res = 0;
    if (i < ch.n) {
        int acc[3][2];
#pragma unroll
        for (int b = 0; b < 3; b++) {
            uint32_t v = bands[b * nloc + ch.loc_off + i];
            double a = att[b * nloc + ch.loc_off + i];
            int l = lo16(v), r = hi16(v);
            if (a != 0.0) {
                double f = exp10(-a / 20.0);
                l = mul16(l, f);
                r = mul16(r, f);
            }
            acc[b][0] = l;
            acc[b][1] = r;
        }
        int16_t o[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            int s1 = i < n1 ? (int)sat16(acc[0][k] + acc[1][k]) : 0;
            o[k] = sat16(s1 + acc[2][k]);
        }
        res = pack2(o[0], o[1]);
    }
    out[ch.out_off + i] = res;
}

// ---------------------------------------------------------------- launchers
hipError_t launch_rms(const Launch &l, const int16_t *bands, uint16_t *r, int64_t nloc) {
    dim3 g = grid1(l.n_seg);
    g.y = 3;
    hipLaunchKernelGGL(k_rms, g, dim3(AMX_BLOCK), 0, l.stream, l.cd, l.chunks, l.segs, l.n_seg,
                       reinterpret_cast<const uint32_t *>(bands), r, nloc);
    return hipGetLastError();
}

hipError_t launch_env(const Launch &l, const uint16_t *r, const double *tabs, double *att,
                      double *guess, double *endv, int64_t nloc, int warm) {
    dim3 g = grid1(l.n_seg);
    g.y = 3;
    hipLaunchKernelGGL(k_env, g, dim3(AMX_BLOCK), 0, l.stream, l.cd, l.chunks, l.segs, l.n_seg,
                       r, tabs, att, guess, endv, nloc, warm);
    return hipGetLastError();
}

hipError_t launch_fix(const Launch &l, const uint16_t *r, const double *tabs, double *att,
                      double *guess, double *endv, int64_t nloc) {
    if (l.n_chunks <= 0) return hipSuccess;
    dim3 g((unsigned)l.n_chunks, 3);
    hipLaunchKernelGGL(k_fix, g, dim3(64), 0, l.stream, l.cd, l.chunks, l.segs, l.n_seg, r, tabs,
                       att, guess, endv, nloc);
    return hipGetLastError();
}

hipError_t launch_apply_n1(const Launch &l, const int16_t *bands, const double *att,
                           int16_t *out, int64_t nloc, int64_t max_chunk_out,
                           const int64_t *n1tab) {
    dim3 g = grid1(max_chunk_out);
    g.y = (unsigned)l.n_chunks;
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_apply, g, dim3(AMX_BLOCK), 0, l.stream, l.chunks,
                       reinterpret_cast<const uint32_t *>(bands), att,
                       reinterpret_cast<uint32_t *>(out), nloc, n1tab);
    return hipGetLastError();
}


}  // namespace amx
