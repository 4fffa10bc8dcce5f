// amx_dyn.hip -- multiband compressor dynamics (pydub compress_dynamic_range,
// audio_mastering_engine.py:306-308) and the overlay (:309).
//
// Per band b and frame i:
//   r_i   = audioop.rms of frames [max(i-look, 0), i)          (exact integer sums)
//   m_i   = (1 - 1/ratio) * max(20 log10(r_i / thr), 0)        (host tables, C libm)
//   att  <- (r_i > thr and att <= m_i) ? min(att + m_i/A, m_i) : max(att - m_i/R, 0)
//   out_i = audioop.mul(frame_i, 10^(-att/20))   if att != 0
//
// r is embarrassingly parallel (k_rms: block prefix sums).  The envelope is a
// sequential nonlinear recurrence; it is parallelised by exact speculation:
//   round 0 (k_env0): every envelope segment of Le frames runs from att = 0 started
//     W frames earlier (the trajectories of this recurrence coincide after clamp
//     events, so the warm-up usually lands exactly on the true state) and writes its
//     gained output, its start guess s_j and end state e_j;
//   rounds 1..R (k_envfix): segment j takes its true start from the end of the
//     nearest earlier segment that has any over-threshold frame (below-threshold
//     frames hold the state: m = 0 makes both steps the identity), and if it differs
//     from s_j re-runs both trajectories in lockstep until they coincide, rewriting
//     the gained output up to there;
//   k_envseq: a final in-order walk per (chunk, band) fixes whatever is still
//     inconsistent, so the result is exact whatever the signal; it costs one parallel
//     consistency scan when the rounds already converged.
// Every value is produced by the reference's own operation sequence from the true
// start state, so the envelope is bit-exact, not approximate.
#include "amx_dev.hpp"

namespace amx {

#define AMX_TAB 32769

// ----------------------------------------- compressor RMS detector (exact)
// One workgroup = AMX_RMS_F frames of one (chunk, band); squares of the window
// [base - look, base + AMX_RMS_F) are prefix-summed in LDS (exact int64), so
// S_i = P(i) - P(max(i - look, 0)) with no sequential sliding window.
#define AMX_RMS_F 1024
#define AMX_RMS_MAXLOOK 1024
// It also looks up m_i = max_attenuation(r_i) once per frame (consecutive frames
// have similar r, so these gathers are cache friendly) for the envelope kernels,
// which then stream (r, m) and derive inc = m/A, dec = m/R by IEEE division --
// the same correctly rounded quotients the host tables hold.
__global__ void __launch_bounds__(AMX_BLOCK) k_rms(const ChainDev *__restrict__ cdp,
                                                   const ChunkDev *__restrict__ chunks,
                                                   const uint32_t *__restrict__ bands,
                                                   const double *__restrict__ tabs,
                                                   uint16_t *__restrict__ rr,
                                                   double *__restrict__ mm, int64_t nloc) {
    constexpr int N = AMX_RMS_F + AMX_RMS_MAXLOOK;
    constexpr int PER = N / AMX_BLOCK;                 // 8 values per thread
    __shared__ long long P[N];
    __shared__ long long wsum[AMX_BLOCK / 64];
    const int look = cdp->look;
    const int c = blockIdx.y, b = blockIdx.z;
    const ChunkDev ch = chunks[c];
    const int64_t base = (int64_t)blockIdx.x * AMX_RMS_F;
    if (base >= ch.n) return;                          // block-uniform
    const uint32_t *x = bands + b * nloc + ch.loc_off;
    uint16_t *r = rr + b * nloc + ch.loc_off;
    double *mo = mm + b * nloc + ch.loc_off;
    const double *mt = tabs + (int64_t)b * 3 * AMX_TAB;
    // LDS slot k holds frame base - look + k (frames before the chunk count as 0)
    const int64_t f0 = base - look;
    const int t = threadIdx.x;
    long long v[PER];
#pragma unroll
    for (int q = 0; q < PER; q++) {
        const int k = t * PER + q;
        const int64_t f = f0 + k;
        const bool ok = f >= 0 && f < ch.n && k < AMX_RMS_F + look;
        const uint32_t u = x[ok ? f : 0];
        const long long a = lo16(u), d = hi16(u);
        v[q] = ok ? a * a + d * d : 0;
    }
    // block inclusive scan: per-thread serial, wave scan of totals, cross-wave
    long long run = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) { run += v[q]; v[q] = run; }
    long long incl = run;
    const int lane = t & 63, w = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long up = __shfl_up(incl, o);
        if (lane >= o) incl += up;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    long long wpre = 0;
    for (int q = 0; q < w; q++) wpre += wsum[q];
    const long long excl = wpre + incl - run;
#pragma unroll
    for (int q = 0; q < PER; q++) P[t * PER + q] = excl + v[q];
    __syncthreads();
    // frame i = base + n uses slots [n, n + look) -> P[n + look - 1] - P[n - 1]
    for (int n = t; n < AMX_RMS_F; n += AMX_BLOCK) {
        const int64_t i = base + n;
        if (i >= ch.n) break;
        const int64_t wlo = i - look < 0 ? 0 : i - look;
        const int64_t cnt = 2 * (i - wlo);
        const long long S = P[n + look - 1] - (n > 0 ? P[n - 1] : 0);
        const uint32_t rms = cnt ? (uint32_t)sqrt((double)S / (double)cnt) : 0u;
        const uint32_t rc = rms > 32768u ? 32768u : rms;      // |sample| <= 32768
        r[i] = (uint16_t)rc;
        mo[i] = mt[rc];
    }
}

// --------------------------------------------------------- envelope helpers
struct EnvTab {
    const double *m;     // per-frame max_attenuation (k_rms)
    double A, R;         // attack / release frames (pydub frame_count(ms=5 / 50))
    int rthr;
};

// pydub envelope step, exact, branch-free (both candidates, then select)
__device__ __forceinline__ double env_step(double att, bool over, double m, double inc,
                                           double dec) {
    const double up = fmin(att + inc, m);          // attenuation += inc; min(., max_att)
    const double dn = fmax(att - dec, 0.0);        // attenuation -= dec; max(., 0)
    return (over && att <= m) ? up : dn;
}

// audioop.mul clamp + floor (CPython Modules/audioop.c fbound)
__device__ __forceinline__ int mul16(int v, double f) {
    double val = (double)v * f;
    if (val > 32767.0) val = 32767.0;
    else if (val < -32768.0 + 1.0) val = -32768.0;
    return (int)floor(val);
}

// the gained frame for attenuation att (:306-308 output, audioop.mul)
__device__ __forceinline__ uint32_t gain_frame(uint32_t v, double att) {
    if (att == 0.0) return v;
    const double f = exp10(-att / 20.0);
    return pack2((int16_t)mul16(lo16(v), f), (int16_t)mul16(hi16(v), f));
}

#define AMX_ENV_B 8   // frames per batch: table gathers issued ahead of the chain

// run the envelope over frames [f0, f1) of r from att; optionally write gained output
template <bool OUT>
__device__ __forceinline__ double env_run(const EnvTab &T, const uint16_t *r, int64_t f0,
                                          int64_t f1, double att, bool &any_over,
                                          const uint32_t *x, uint32_t *g) {
    for (int64_t f = f0; f < f1; f += AMX_ENV_B) {
        double m[AMX_ENV_B], inc[AMX_ENV_B], dec[AMX_ENV_B];
        bool ov[AMX_ENV_B];
        uint32_t xv[AMX_ENV_B];
#pragma unroll
        for (int q = 0; q < AMX_ENV_B; q++) {
            const bool ok = f + q < f1;
            const int64_t fc = ok ? f + q : f0;        // clamped, unconditional (tile_load)
            const int rv = r[fc];
            const double mv = T.m[fc];
            ov[q] = ok && rv >= T.rthr;
            m[q] = ok ? mv : 0.0;
            inc[q] = m[q] / T.A;
            dec[q] = m[q] / T.R;
            if (OUT) xv[q] = x[ok ? f + q : f0];
        }
#pragma unroll
        for (int q = 0; q < AMX_ENV_B; q++) {
            if (f + q >= f1) break;
            att = env_step(att, ov[q], m[q], inc[q], dec[q]);
            any_over |= ov[q];
            if (OUT) g[f + q] = gain_frame(xv[q], att);
        }
    }
    return att;
}

// ------------------------------------------------------- round 0: speculation
// One thread per (envelope segment, band).  s = state at the segment start from a
// warm-up of W frames begun at rest; e = state at the segment end; act = the
// segment has an over-threshold frame (else its transfer is the identity).
__global__ void __launch_bounds__(AMX_BLOCK) k_env0(const ChainDev *__restrict__ cdp,
                                                    const ChunkDev *__restrict__ chunks,
                                                    const SegDev *__restrict__ es, int n_es,
                                                    const uint16_t *__restrict__ rr,
                                                    const uint32_t *__restrict__ bands,
                                                    const double *__restrict__ mm,
                                                    uint32_t *__restrict__ gained,
                                                    double *__restrict__ sv,
                                                    double *__restrict__ ev,
                                                    int *__restrict__ act, int64_t nloc,
                                                    int warm) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (j >= n_es) return;
    const SegDev sg = es[j];
    const ChunkDev ch = chunks[sg.chunk];
    const uint16_t *r = rr + b * nloc + ch.loc_off;
    const uint32_t *x = bands + b * nloc + ch.loc_off;
    uint32_t *g = gained + b * nloc + ch.loc_off;
    const EnvTab T{mm + b * nloc + ch.loc_off, 5.0 * (cdp->fs / 1000.0), 50.0 * (cdp->fs / 1000.0),
                   cdp->rthr[b]};
    int64_t w0 = sg.pos - warm;
    if (w0 < 0) w0 = 0;
    bool any = false, dummy = false;
    double att = env_run<false>(T, r, w0, sg.pos, 0.0, dummy, nullptr, nullptr);
    sv[(int64_t)b * n_es + j] = att;
    att = env_run<true>(T, r, sg.pos, sg.pos + sg.len, att, any, x, g);
    ev[(int64_t)b * n_es + j] = att;
    act[(int64_t)b * n_es + j] = any ? 1 : 0;
}

// prev[j] = the nearest earlier active segment of the same chunk (or -1): the
// segment whose end state is segment j's true start.  One wave per (chunk, band).
__global__ void __launch_bounds__(64) k_env_prev(const ChunkDev *__restrict__ chunks,
                                                 const int *__restrict__ eseg0,
                                                 const int *__restrict__ neseg, int n_es,
                                                 const int *__restrict__ act,
                                                 int *__restrict__ prev) {
    const int c = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    const int s0 = eseg0[c], s1 = s0 + neseg[c];
    const int *A = act + (int64_t)b * n_es;
    int *P = prev + (int64_t)b * n_es;
    int carry = -1;                                    // last active index before the batch
    for (int base = s0; base < s1; base += 64) {
        const int j = base + lane;
        const bool a = j < s1 && A[j] != 0;
        // inclusive max-scan of (a ? j : -1); prev[j] = exclusive value
        int v = a ? j : -1;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int up = __shfl_up(v, o);
            if (lane >= o) v = max(v, up);
        }
        int excl = __shfl_up(v, 1);
        if (lane == 0) excl = -1;
        excl = max(excl, carry);
        if (j < s1) P[j] = excl;
        carry = max(carry, __shfl(v, 63));
    }
}

// re-run segment j from the new start `ns` while re-running the stored trajectory
// from `os` in lockstep; rewrite the gained output until the two coincide.
// Returns the segment's end state (old end if they coincided).
__device__ double env_rerun(const EnvTab &T, const uint16_t *r, const uint32_t *x, uint32_t *g,
                            int64_t f0, int64_t f1, double os, double ns, double old_end) {
    double a = os, c = ns;
    for (int64_t f = f0; f < f1; f += AMX_ENV_B) {
        double m[AMX_ENV_B], inc[AMX_ENV_B], dec[AMX_ENV_B];
        bool ov[AMX_ENV_B];
        uint32_t xv[AMX_ENV_B];
#pragma unroll
        for (int q = 0; q < AMX_ENV_B; q++) {
            const bool ok = f + q < f1;
            const int64_t fc = ok ? f + q : f0;        // clamped, unconditional (tile_load)
            const int rv = r[fc];
            const double mv = T.m[fc];
            ov[q] = ok && rv >= T.rthr;
            m[q] = ok ? mv : 0.0;
            inc[q] = m[q] / T.A;
            dec[q] = m[q] / T.R;
            xv[q] = x[ok ? f + q : f0];
        }
#pragma unroll
        for (int q = 0; q < AMX_ENV_B; q++) {
            if (f + q >= f1) return c;
            a = env_step(a, ov[q], m[q], inc[q], dec[q]);
            c = env_step(c, ov[q], m[q], inc[q], dec[q]);
            if (a == c) return old_end;                // identical from here on
            g[f + q] = gain_frame(xv[q], c);
        }
    }
    return c;
}

// ------------------------------------------------ rounds: parallel fix-up
// Reads e_in (previous round), writes e_out; s is updated in place (segment-owned).
__global__ void __launch_bounds__(AMX_BLOCK) k_envfix(const ChainDev *__restrict__ cdp,
                                                      const ChunkDev *__restrict__ chunks,
                                                      const SegDev *__restrict__ es, int n_es,
                                                      const uint16_t *__restrict__ rr,
                                                      const uint32_t *__restrict__ bands,
                                                      const double *__restrict__ mm,
                                                      uint32_t *__restrict__ gained,
                                                      double *__restrict__ sv,
                                                      const double *__restrict__ e_in,
                                                      double *__restrict__ e_out,
                                                      const int *__restrict__ act,
                                                      const int *__restrict__ prev,
                                                      int64_t nloc) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (j >= n_es) return;
    const int64_t k = (int64_t)b * n_es + j;
    const int p = prev[k];
    const double ns = p >= 0 ? e_in[(int64_t)b * n_es + p] : 0.0;
    const double os = sv[k];
    if (ns == os) { e_out[k] = e_in[k]; return; }
    const SegDev sg = es[j];
    const ChunkDev ch = chunks[sg.chunk];
    const uint32_t *x = bands + b * nloc + ch.loc_off;
    uint32_t *g = gained + b * nloc + ch.loc_off;
    if (!act[k]) {
        // identity transfer: the held state is the new start for every frame
        for (int64_t f = sg.pos; f < sg.pos + sg.len; f++) g[f] = gain_frame(x[f], ns);
        e_out[k] = ns;
    } else {
        const uint16_t *r = rr + b * nloc + ch.loc_off;
        const EnvTab T{mm + b * nloc + ch.loc_off, 5.0 * (cdp->fs / 1000.0),
                       50.0 * (cdp->fs / 1000.0), cdp->rthr[b]};
        e_out[k] = env_rerun(T, r, x, g, sg.pos, sg.pos + sg.len, os, ns, e_in[k]);
    }
    sv[k] = ns;
}

// --------------------------------------- final in-order walk (exactness net)
// One wave per (chunk, band): find the first segment whose start disagrees with
// its predecessor's end (64 at a time), fix it on lane 0, continue after it.
__global__ void __launch_bounds__(64) k_envseq(const ChainDev *__restrict__ cdp,
                                               const ChunkDev *__restrict__ chunks,
                                               const SegDev *__restrict__ es, int n_es,
                                               const int *__restrict__ eseg0,
                                               const int *__restrict__ neseg,
                                               const uint16_t *__restrict__ rr,
                                               const uint32_t *__restrict__ bands,
                                               const double *__restrict__ mm,
                                               uint32_t *__restrict__ gained,
                                               double *__restrict__ sv, double *__restrict__ ev,
                                               const int *__restrict__ act,
                                               const int *__restrict__ prev, int64_t nloc) {
    const int c = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    const int s0 = eseg0[c], s1 = s0 + neseg[c];
    const ChunkDev ch = chunks[c];
    const uint16_t *r = rr + b * nloc + ch.loc_off;
    const uint32_t *x = bands + b * nloc + ch.loc_off;
    uint32_t *g = gained + b * nloc + ch.loc_off;
    const EnvTab T{mm + b * nloc + ch.loc_off, 5.0 * (cdp->fs / 1000.0), 50.0 * (cdp->fs / 1000.0),
                   cdp->rthr[b]};
    double *S = sv + (int64_t)b * n_es, *E = ev + (int64_t)b * n_es;
    const int *A = act + (int64_t)b * n_es, *Pv = prev + (int64_t)b * n_es;
    int cur = s0;
    while (cur < s1) {
        int found = s1;
        for (int base = cur; base < s1; base += 64) {
            const int j = base + lane;
            bool bad = false;
            if (j < s1) {
                const int p = Pv[j];
                const double ns = p >= 0 ? E[p] : 0.0;
                bad = !(ns == S[j]);
            }
            const unsigned long long m = __ballot(bad);
            if (m) { found = base + __ffsll((long long)m) - 1; break; }
        }
        if (found >= s1) break;
        if (lane == 0) {
            const SegDev sg = es[found];
            const int p = Pv[found];
            const double ns = p >= 0 ? E[p] : 0.0;
            if (!A[found]) {
                for (int64_t f = sg.pos; f < sg.pos + sg.len; f++) g[f] = gain_frame(x[f], ns);
                E[found] = ns;
            } else {
                E[found] = env_rerun(T, r, x, g, sg.pos, sg.pos + sg.len, S[found], ns, E[found]);
            }
            S[found] = ns;
        }
        __threadfence_block();
        cur = found + 1;
    }
}

// ------------------------------------------------------------------- overlay
// low.overlay(mid).overlay(high) (:309) of the gained bands -> chunk output with
// pydub's ms-rounded lengths: n1 after the first overlay, n2 = out_n after the second.
__global__ void __launch_bounds__(AMX_BLOCK) k_overlay(const ChunkDev *__restrict__ chunks,
                                                       const uint32_t *__restrict__ gained,
                                                       uint32_t *__restrict__ out, int64_t nloc,
                                                       const int64_t *__restrict__ n1tab) {
    const int c = blockIdx.y;
    const ChunkDev ch = chunks[c];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n2 = ch.out_n;
    if (i >= n2) return;
    const int64_t n1 = n1tab[c];
    uint32_t res = 0;
    if (i < ch.n) {
        const uint32_t v0 = gained[ch.loc_off + i];
        const uint32_t v1 = gained[nloc + ch.loc_off + i];
        const uint32_t v2 = gained[2 * nloc + ch.loc_off + i];
        int16_t o[2];
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int a0 = k ? hi16(v0) : lo16(v0), a1 = k ? hi16(v1) : lo16(v1);
            const int a2 = k ? hi16(v2) : lo16(v2);
            const int s1 = i < n1 ? (int)sat16(a0 + a1) : 0;
            o[k] = sat16(s1 + a2);
        }
        res = pack2(o[0], o[1]);
    }
    out[ch.out_off + i] = res;
}

// ---------------------------------------------------------------- launchers
hipError_t launch_rms(const DynLaunch &d, const int16_t *bands, uint16_t *r, double *m) {
    if (d.look > AMX_RMS_MAXLOOK) return hipErrorInvalidValue;
    dim3 g((unsigned)((d.max_chunk_n + AMX_RMS_F - 1) / AMX_RMS_F), (unsigned)d.n_chunks, 3);
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_rms, g, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks,
                       reinterpret_cast<const uint32_t *>(bands), d.tabs, r, m, d.nloc);
    return hipGetLastError();
}

hipError_t launch_env(const DynLaunch &d, const uint16_t *r, const double *m, const int16_t *bands,
                      int16_t *gained, double *sv, double *e0, double *e1, int *act, int *prev,
                      int rounds) {
    if (d.n_es <= 0) return hipSuccess;
    const uint32_t *x = reinterpret_cast<const uint32_t *>(bands);
    uint32_t *g = reinterpret_cast<uint32_t *>(gained);
    dim3 grid = grid1(d.n_es);
    grid.y = 3;
    hipLaunchKernelGGL(k_env0, grid, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks, d.es, d.n_es, r, x,
                       m, g, sv, e0, act, d.nloc, d.warm);
    hipLaunchKernelGGL(k_env_prev, dim3((unsigned)d.n_chunks, 3), dim3(64), 0, d.st, d.chunks,
                       d.eseg0, d.neseg, d.n_es, act, prev);
    double *ein = e0, *eout = e1;
    for (int k = 0; k < rounds; k++) {
        hipLaunchKernelGGL(k_envfix, grid, dim3(AMX_BLOCK), 0, d.st, d.cd, d.chunks, d.es, d.n_es,
                           r, x, m, g, sv, ein, eout, act, prev, d.nloc);
        double *tmp = ein;
        ein = eout;
        eout = tmp;
    }
    return hipGetLastError();
}

// ends: the array the last round wrote (e0 if rounds is even, else e1)
hipError_t launch_envseq(const DynLaunch &d, const uint16_t *r, const double *m,
                         const int16_t *bands,
                         int16_t *gained, double *sv, double *ends, const int *act,
                         const int *prev) {
    if (d.n_es <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_envseq, dim3((unsigned)d.n_chunks, 3), dim3(64), 0, d.st, d.cd, d.chunks,
                       d.es, d.n_es, d.eseg0, d.neseg, r,
                       reinterpret_cast<const uint32_t *>(bands), m,
                       reinterpret_cast<uint32_t *>(gained), sv, ends, act, prev, d.nloc);
    return hipGetLastError();
}

hipError_t launch_overlay(const DynLaunch &d, const int16_t *gained, int16_t *out,
                          int64_t max_chunk_out, const int64_t *n1tab) {
    dim3 g = grid1(max_chunk_out);
    g.y = (unsigned)d.n_chunks;
    if (empty(g)) return hipSuccess;
    hipLaunchKernelGGL(k_overlay, g, dim3(AMX_BLOCK), 0, d.st, d.chunks,
                       reinterpret_cast<const uint32_t *>(gained),
                       reinterpret_cast<uint32_t *>(out), d.nloc, n1tab);
    return hipGetLastError();
}

}  // namespace amx
