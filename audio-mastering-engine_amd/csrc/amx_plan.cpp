// amx_plan.cpp -- host side of libamx.so: plan construction (state-space models,
// scan matrices, segment tables, compressor tables) and the C ABI of include/amx.h.
#include "../../include/amx.h"
#include "amx_internal.hpp"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return fail(AMX_EHIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

// ------------------------------------------------------------ dense helpers
// The scan tables (GEMV rows A^n B, A^L, block powers) are computed in long double (x86
// 80-bit, 64-bit mantissa) and rounded to double once: built in double by repeated
// products they carried ~1e-12 of error into the segment start states at 96 kHz
// (DESIGN.md §3.1), 20x the sequential recursion's own rounding; rounded once they
// carry less than it.
using LD = long double;
using Mat = std::vector<double>;  // row-major D x D
using MatL = std::vector<LD>;

MatL matmul(const MatL &a, const MatL &b, int D) {
    MatL c((size_t)D * D, 0.0L);
    for (int i = 0; i < D; i++)
        for (int k = 0; k < D; k++) {
            const LD v = a[(size_t)i * D + k];
            if (v == 0.0L) continue;
            for (int j = 0; j < D; j++) c[(size_t)i * D + j] += v * b[(size_t)k * D + j];
        }
    return c;
}
MatL matpow(const MatL &a, int64_t p, int D) {
    MatL r((size_t)D * D, 0.0L), b = a;
    for (int i = 0; i < D; i++) r[(size_t)i * D + i] = 1.0L;
    while (p > 0) {
        if (p & 1) r = matmul(r, b, D);
        b = matmul(b, b, D);
        p >>= 1;
    }
    return r;
}
LD norm_inf(const MatL &a, int D) {
    LD m = 0.0L;
    for (int i = 0; i < D; i++) {
        LD s = 0.0L;
        for (int j = 0; j < D; j++) s += std::fabs(a[(size_t)i * D + j]);
        m = s > m ? s : m;
    }
    return m;
}
Mat to_double(const MatL &a) { return Mat(a.begin(), a.end()); }

// A linear time-invariant model s' = A s + B x of a chain, derived (in long double) by
// stepping a host copy of the chain from unit states / a unit input.
struct Lti {
    int D = 0;
    MatL A;
    std::vector<LD> B;
    template <class Step>
    void derive(int dim, Step step) {
        D = dim;
        A.assign((size_t)D * D, 0.0L);
        B.assign(D, 0.0L);
        std::vector<LD> s(D);
        for (int k = 0; k < D; k++) {
            std::fill(s.begin(), s.end(), 0.0L);
            s[k] = 1.0L;
            step(s.data(), 0.0L);
            for (int i = 0; i < D; i++) A[(size_t)i * D + k] = s[i];
        }
        std::fill(s.begin(), s.end(), 0.0L);
        step(s.data(), 1.0L);
        for (int i = 0; i < D; i++) B[i] = s[i];
    }
    Mat pow(int64_t p) const { return to_double(matpow(A, p, D)); }
    // G[n][d] = (A^{L-1-n} B)[d]
    std::vector<double> gemv_table(int L) const {
        std::vector<double> G((size_t)L * D);
        std::vector<LD> v = B, t(D);
        for (int n = L - 1; n >= 0; n--) {
            for (int d = 0; d < D; d++) G[(size_t)n * D + d] = (double)v[d];
            for (int i = 0; i < D; i++) {
                LD acc = 0.0L;
                for (int k = 0; k < D; k++) acc += A[(size_t)i * D + k] * v[k];
                t[i] = acc;
            }
            v = t;
        }
        return G;
    }
    // window powers Mb^k, k = 1 .. K-1, of Mb = A^LS; K = the first k with
    // ||Mb^k|| <= tol (the block scan sums the previous K-1 blocks' contributions).
    int window_powers(int64_t LS, double tol, int max_k, std::vector<double> &out) const {
        MatL Mb = matpow(A, LS, D);
        MatL cur = Mb;
        out.clear();
        int K = 1;
        while (norm_inf(cur, D) > tol) {
            for (LD v : cur) out.push_back((double)v);
            cur = matmul(cur, Mb, D);
            K++;
            if (K > max_k) return -1;
        }
        return K;
    }
};

// host step functions (same math as the device chains, no rounding claims)
template <class T>
void shelf_step_h(const double *c, T *z, T &x, int neg, double gm1) {
    T y = z[0] + (T)c[0] * x;
    z[0] = (z[1] + x * (T)c[1]) - y * (T)c[4];
    z[1] = x * (T)c[2] - y * (T)c[5];
    x = neg ? y : x + (y - x) * (T)gm1;
}
template <class T>
T sos_step_h(const double *c, T *z, T x) {
    T y = (T)c[0] * x + z[0];
    z[0] = ((T)c[1] * x - (T)c[4] * y) + z[1];
    z[1] = (T)c[2] * x - (T)c[5] * y;
    return y;
}

void *align_up(size_t &off, size_t bytes) {
    size_t o = (off + 255) & ~(size_t)255;
    off = o + bytes;
    return reinterpret_cast<void *>(o);
}

}  // namespace

namespace amx {
// libswresample's resampler geometry and filter bank for the loudness measurement's
// 192 kHz stream (what ffmpeg inserts ahead of af_loudnorm in dynamic mode, :229).
// Restated from resample.c resample_init / build_filter with swresample's defaults:
// filter_size 32, phase_shift 10, exact_rational 1, cutoff 0.97, Kaiser beta 9, FLTP
// (float32 bank, scale 1).  Upsampling only (factor 1); L / M = out / in reduced (output j
// sits at input position j M / L).  The bank has L phases when L <= 1024 (exact_rational)
// and 1024 otherwise (22.05 / 11.025 kHz): the position then falls between two phases and
// libswresample's linear kernel interpolates (amx_dev.hpp swr_dot_lin).
int swr_geometry(int in_rate, int out_rate, int *L, int *M) {
    if (in_rate <= 0 || out_rate <= 0) return -1;
    int64_t a = in_rate, b = out_rate;
    while (b) { int64_t t = a % b; a = b; b = t; }
    *L = (int)(out_rate / a);
    *M = (int)(in_rate / a);
    return 0;
}

// resample_init: factor = min(out_rate * cutoff / in_rate, 1) (cutoff 0.97); filter_length
// = max(ceil(filter_size / factor), 1) rounded up to even; rows of filter_alloc =
// FFALIGN(filter_length, 8) floats.  An input above 192 kHz / 0.97 (352.8 / 384 / 705.6 /
// 768 kHz) is DOWNsampled with the longer, narrower filter.  Equal rates: no resampler
// (ffmpeg only converts the sample format), the 32-tap identity row.
int swr_filter(int in_rate, int out_rate, int *taps, int *alloc, double *factor) {
    if (in_rate <= 0 || out_rate <= 0) return -1;
    double f = out_rate * 0.97 / in_rate;
    if (f > 1.0 || in_rate == out_rate) f = 1.0;
    int t = (int)std::ceil(32 / f);
    if (t < 1) t = 1;
    if (t > 1) t = (t + 1) & ~1;
    const int al = (t + 7) & ~7;
    if (al > AMX_SWR_MAX_ALLOC) return -1;
    if (taps) *taps = t;
    if (alloc) *alloc = al;
    if (factor) *factor = f;
    return 0;
}

// resample_init: phase_count 1 << phase_shift (1024), replaced by the exact out / gcd
// when that is <= 1024 (exact_rational).  The interpolating (1024-phase) form is restated
// for the 32-tap filter only.
int swr_phases(int in_rate, int out_rate) {
    int L, M, t;
    if (swr_geometry(in_rate, out_rate, &L, &M) || swr_filter(in_rate, out_rate, &t, nullptr, nullptr)) return -1;
    if (L > 1024 && t != 32) return -1;
    return L <= 1024 ? L : 1024;
}

// resample_init: av_reduce(&src_incr, &dst_incr, out_rate, in_rate * phase_count), both
// doubled while below 2^20; output j sits at phase position j dst_incr / src_incr
int swr_incr(int in_rate, int out_rate, int64_t *src_incr, int64_t *dst_incr) {
    const int pc = swr_phases(in_rate, out_rate);
    if (pc < 0) return -1;
    int64_t a = out_rate, b = (int64_t)in_rate * pc, x = a, y = b;
    while (y) { int64_t t = x % y; x = y; y = t; }
    a /= x;
    b /= x;
    while (b < (1 << 20) && a < (1 << 20)) { a *= 2; b *= 2; }
    *src_incr = a;
    *dst_incr = b;
    return 0;
}

static double swr_bessel(double x) {
    double lastv = 0, t, v;
    double inv[100];
    for (int k = 0; k < 100; k++) inv[k] = 1.0 / ((double)(k + 1) * (double)(k + 1));
    x = x * x / 4;
    t = x;
    v = 1 + x;
    for (int i = 1; v != lastv && i < 98; i += 2) {
        t *= x * inv[i];
        v += t;
        lastv = v;
        t *= x * inv[i + 1];
        v += t;
    }
    return v;
}

// build_filter (Kaiser beta 9, FLTP, scale 1): pc rows of filter_alloc floats (zeros past
// filter_length); factor 1 forms sin(x) / x from an alternating sine table, factor < 1
// from sin(x) itself
int swr_bank(int in_rate, int out_rate, float *bank) {
    const int pc = swr_phases(in_rate, out_rate);
    int taps = 0, alloc = 0;
    double factor = 1.0;
    if (pc < 0 || swr_filter(in_rate, out_rate, &taps, &alloc, &factor)) return -1;
    const int center = (taps - 1) / 2;
    const int ph_nb = pc % 2 ? pc : pc / 2 + 1;
    std::vector<double> sin_lut(ph_nb), tab(taps);
    double norm = 0;
    std::fill(bank, bank + (size_t)pc * alloc, 0.0f);
    if (factor == 1.0)
        for (int ph = 0; ph < ph_nb; ph++) sin_lut[ph] = std::sin(M_PI * ph / pc) * (center & 1 ? 1 : -1);
    for (int ph = 0; ph < ph_nb; ph++) {
        double sv = factor == 1.0 ? sin_lut[ph] : 0.0;
        for (int i = 0; i < taps; i++) {
            const double x = M_PI * ((double)(i - center) - (double)ph / pc) * factor;
            double y = x == 0 ? 1.0 : (factor == 1.0 ? sv / x : std::sin(x) / x);
            const double w = 2.0 * x / (factor * taps * M_PI);
            y *= swr_bessel(9.0 * std::sqrt(std::max(1 - w * w, 0.0)));
            tab[i] = y;
            sv = -sv;
            if (!ph) norm += y;
        }
        for (int i = 0; i < taps; i++) bank[ph * alloc + i] = (float)(tab[i] * 1 / norm);
        if (pc % 2) continue;
        if (pc - ph < pc)
            for (int i = 0; i < taps; i++) bank[(pc - ph) * alloc + taps - 1 - i] = bank[ph * alloc + i];
    }
    return 0;
}
}  // namespace amx

struct amx_plan {
    amx_chain_desc desc;
    ChainDev cd;
    int L = 256, Lkw = 512, hop = 0;
    // loudness measurement stream: ffmpeg's pass 1 resamples to 192 kHz (L phases,
    // step M; Lin chain frames = Lout 192 kHz frames per K segment); resamp = 0 when
    // the track already is at 192 kHz (the measurement runs on d_out itself)
    int resamp = 0, upL = 1, upM = 1, upLin = 0, upLout = 0, up_static = 0, up_ok = 1;
    int meas_native = 0;    // no 192 kHz resampler for this rate: peaks only, no loudnorm
    const int32_t *gate = nullptr;   // amx_plan_set_gate: the per-sample kernels' mode word
    int32_t *publish = nullptr;      // amx_plan_set_publish: pinned host words k_decide also stores
    // libswresample's phase count (L, or 1024 when L > 1024), phase step dst / src per
    // output; up_lin: the step is not an integer, every output interpolates between rows
    // ph and ph + 1 (bank row pc = row 0 one tap later) with weight owt[n]
    int up_pc = 1, up_lin = 0;
    int up_taps = 32, up_alloc = 32;   // filter_length / filter_alloc (> 32: downsampling)
    int64_t up_src = 1, up_dst = 1;
    int32_t *d_obase = nullptr, *d_oph = nullptr;
    float *d_owt = nullptr;
    int32_t *d_slow = nullptr;   // K segments k_up_edge takes (static / poly path); n_slow of them
    int up_poly = 0;             // k_up_poly's form (AMX_UP_POLY) when the rate has one
    int32_t *d_fcnt = nullptr;   // k_up_poly: outputs per segment frame
    float *d_bankn = nullptr;    // k_up_poly: bank rows in output order
    int64_t n_slow = 0;
    double kdf_b[5] = {0, 0, 0, 0, 0}, kdf_a[5] = {0, 0, 0, 0, 0};   // K filter, fused direct form (192 kHz)
    hipStream_t up_aux = nullptr;            // k_up_edge's stream, forked from / joined to the caller's
    hipEvent_t up_fork = nullptr, up_join = nullptr;
    double *d_qh = nullptr, *d_qt = nullptr;
    float *d_bank = nullptr;
    int mask = 0, D = 0;
    int lev_eq = 0, lev_x = 0, lev_kw = 0;
    int mb = 0;
    int Le = 1024, warm = 2304, rounds = 2;   // compressor envelope segments (amx_dyn.hip)
    int Le_t[4] = {0, 0, 0, 0};               // segment length of the table for t active bands
    int env_wg = 1, env_pin = 0;              // k_env0 placement (amx_dyn.hip launch_env)
    int f1_mode = AMX_F1_SPLIT;               // pass-1 form for float32 stereo + analog
    int n_es = 0;
    std::vector<SegDev> esegs;
    std::vector<int> eseg0, neseg;
    int fuse_kw = 0;        // loudness pass-1 GEMV + peak run inside k_front2
    int kw_rest_states = 0;
    int kw_eb_ready = 0;     // the K scan's block sums (o_ebk) are those of the current e
    int kw_aligned = 0;     // K-filter hop pieces split only at 16-frame tile boundaries // the last amx_loudness_pass1 left the K-filter start states from rest
    int n_tracks = 0, n_chunks = 0, n_seg = 0, n_kseg = 0, n_blk = 0, n_kblk = 0;
    int64_t max_nkseg = 0;
    int64_t nloc = 0, out_frames = 0, max_chunk_out = 0, max_span = 0, max_chunk_n = 0;
    int64_t an_blocks = 0;      // k_analog_h's 4096-frame blocks over all chunks
    int an_vec = 1;             // k_analog_h<true>: every chunk at an even input frame, >= 4 frames
    int64_t in_frames = 0;  // input frames the chunks read (max in_offset + frames)
    int64_t max_hops = 1;   // 100 ms hops of the longest track's measurement stream
    int mono16 = 0;         // mono int16 input: duplicated to stereo into ws o_dup first
    std::vector<ChunkDev> chunks;
    std::vector<SegDev> segs;
    std::vector<KwSegDev> ksegs;
    std::vector<ScanBlk> blks, kblks;
    std::vector<SpanDev> spans;
    std::vector<int64_t> n1tab;
    Lti kw_model;
    std::vector<double> tail_pow;  // per span: A_kw^{len_last} (16 doubles)
    // device constant tables
    ChainDev *d_cd = nullptr;
    ChunkDev *d_chunks = nullptr;
    SegDev *d_segs = nullptr;
    KwSegDev *d_ksegs = nullptr;
    SpanDev *d_spans = nullptr;
    ScanBlk *d_blks = nullptr, *d_kblks = nullptr;
    SegDev *d_esegs = nullptr;
    int *d_eseg0 = nullptr, *d_neseg = nullptr;
    int64_t *d_n1 = nullptr;
    double *d_G = nullptr, *d_M = nullptr, *d_Mp = nullptr;
    double *d_Gx = nullptr, *d_Mx = nullptr, *d_Mpx = nullptr;
    double *d_Gkw = nullptr, *d_Mkw = nullptr, *d_Mpkw = nullptr;
    double *d_tabs = nullptr, *d_bounds = nullptr, *d_energies = nullptr;
    double *d_carryP = nullptr;
    int n_prev = 0;
    double *d_tailpow = nullptr;
    float *d_lut = nullptr;
    float *d_in_lut = nullptr;     // a stream chain's input table (amx_chain_desc.eq_in_lut), or NULL
    int sc = 0;                    // a stream chain (amx_chain_desc.stream_chain)
    double *lim_att = nullptr;     // amx_plan_set_limiter_trace
    float *d_lut_half = nullptr;   // the odd tanh table's half [0, 32768] (k_analog_h), or NULL
    unsigned int *d_pcnt = nullptr;   // k_peak_reduce's per-track block counter (self re-arming)
    int *d_ppart = nullptr;           // its per-block partial maxima
    int any_empty_span = 0;           // a span with no K segment: its peak is zeroed directly
    amx::LimScratch lim;              // general alimiter segments (amx_limiter_prepare)
    // workspace offsets
    size_t ws_bytes = 0;
    size_t o_a16, o_e, o_s, o_p16, o_ex, o_sx, o_bands, o_r, o_m, o_gain, o_esv, o_ee0, o_eflags, o_eact,
        o_ehead, o_elist, o_eprev, o_elist0;
    size_t o_ekw, o_skw, o_parts, o_phop, o_eterms = 0;
    size_t o_eb, o_ebx, o_ebk, o_pk, o_dup = 0;
    amx::ScanPlan scan_eq() const { return {D, n_blk, lev_eq, d_blks, d_M, d_Mp}; }
    amx::ScanPlan scan_xo() const { return {AMX_XO_DIM, mb ? n_blk : 0, lev_x, d_blks, d_Mx, d_Mpx}; }
    amx::ScanPlan scan_kw() const { return {AMX_KW_DIM, n_kblk, lev_kw, d_kblks, d_Mkw, d_Mpkw}; }
};

namespace {

template <class T>
int upload(T **dst, const T *src, size_t n) {
    if (n == 0) n = 1;
    HIPCHK(hipMalloc((void **)dst, n * sizeof(T)));
    if (src) HIPCHK(hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    return AMX_OK;
}
template <class T>
T *wsp(void *ws, size_t off) {
    return reinterpret_cast<T *>(reinterpret_cast<char *>(ws) + off);
}

// blocks of AMX_SCAN_S segments over each stream's run [j0, j0 + n) of segments
void add_blocks(std::vector<ScanBlk> &out, int32_t j0, int32_t n, int32_t stream) {
    const int32_t first = (int32_t)out.size();
    for (int32_t q = 0; q < n; q += AMX_SCAN_S) {
        ScanBlk b{};
        b.seg0 = j0 + q;
        b.nseg = (n - q) < AMX_SCAN_S ? (n - q) : AMX_SCAN_S;
        b.first = first;
        b.last = (q + AMX_SCAN_S >= n) ? 1 : 0;
        b.stream = stream;
        out.push_back(b);
    }
}

int64_t overlay_len(int64_t n, int fs) {
    // pydub: int(round(1000*(n/fs)) * (fs/1000.0)), Python round = half-to-even
    double ms = std::nearbyint(1000.0 * ((double)n / (double)fs));
    return (int64_t)(ms * (fs / 1000.0));
}

}  // namespace

extern "C" {

int amx_abi_version(void) { return AMX_ABI_VERSION; }
const char *amx_last_error(void) { return g_err.c_str(); }
#ifndef AMX_SRC_HASH
#define AMX_SRC_HASH "unstamped"
#endif
// "AMX_SRC_HASH=<hex>" in the binary: amx/build.py reads it from the file without
// loading the library (no HIP runtime before torch's)
static const char amx_stamp[] = "AMX_SRC_HASH=" AMX_SRC_HASH;
const char *amx_build_id(void) { return amx_stamp + 13; }

int amx_plan_create(const amx_chain_desc *desc, const amx_chunk *chunks, int32_t n_chunks,
                    const int64_t *track_frame0, const int64_t *track_total_frames,
                    int32_t seg_frames, amx_plan **out) {
    if (!desc || !out || (n_chunks > 0 && !chunks) || n_chunks < 0)
        return fail(AMX_EINVAL, "amx_plan_create: null argument");
    if (desc->sample_rate <= 0) return fail(AMX_EINVAL, "sample_rate must be > 0");
    if (desc->channels_in != 1 && desc->channels_in != 2)
        return fail(AMX_EINVAL, "channels_in must be 1 or 2");
    if (desc->analog_on && !desc->tanh_lut)
        return fail(AMX_EINVAL, "analog character needs the float32 tanh table (tanh_lut)");
    if (desc->stream_chain && (desc->analog_on || desc->width_on || !desc->input_s16 || desc->channels_in != 2))
        return fail(AMX_EINVAL, "a stream chain takes int16 pairs, without analog character or width");
    *out = nullptr;
    amx_plan *p = new (std::nothrow) amx_plan();
    if (!p) return fail(AMX_ENOMEM, "out of memory");
    p->desc = *desc;
    p->sc = desc->stream_chain ? 1 : 0;
    const int fs = desc->sample_rate;
    if (desc->env_warm_frames >= 0) p->warm = (desc->env_warm_frames + 127) / 128 * 128;   // whole ring of k_env0 tiles
    if (desc->env_rounds >= 0) p->rounds = desc->env_rounds;
    const char *env_le = std::getenv("AMX_ENV_LE");      // (measurements only)
    if (env_le) p->Le = std::max(128, std::atoi(env_le) / 128 * 128);
    if (p->rounds > AMX_ENV_MAX_ROUNDS) {
        delete p;
        return fail(AMX_EINVAL, "env_rounds %d > %d", desc->env_rounds, AMX_ENV_MAX_ROUNDS);
    }
    p->L = seg_frames > 0 ? seg_frames : 256;
    p->L = (p->L + AMX_TF_FRAMES - 1) / AMX_TF_FRAMES * AMX_TF_FRAMES;   // whole LDS tiles
    // the loudness measurement's rate: 192 kHz (af_loudnorm dynamic mode, :229)
    int kfs = AMX_MEAS_RATE;
    std::vector<float> bank;
    std::vector<int32_t> obase, oph, fcnt;
    std::vector<float> owt;
    std::vector<float> bankn;
    if (fs != kfs) {
        p->resamp = 1;
        if (amx::swr_geometry(fs, kfs, &p->upL, &p->upM) != 0 || amx::swr_phases(fs, kfs) < 0) {
            // a rate whose resampler is not restated (an interpolating downsampler: L >
            // 1024 with the longer filter): the plan measures at the track's own rate,
            // which gives the limiter its peaks (the only measurement lufs=None needs);
            // amx_loudness_decide refuses loudnorm on it.
            p->up_ok = 0;
            p->resamp = 0;
            p->meas_native = 1;
            p->upL = p->upM = 1;
            kfs = fs;
        } else {
            // ~384 192 kHz outputs per K segment, a divisor of the 100 ms hop (19200)
            // where one exists, so a segment lies inside one hop (no hop split)
            const int hop192 = (kfs + 5) / 10;
            int target = 480;                 // (AMX_UP_LOUT overrides, for measurements)
            if (const char *ev = std::getenv("AMX_UP_LOUT")) target = std::max(16, std::atoi(ev));
            p->up_pc = amx::swr_phases(fs, kfs);
            amx::swr_filter(fs, kfs, &p->up_taps, &p->up_alloc, nullptr);
            amx::swr_incr(fs, kfs, &p->up_src, &p->up_dst);
            p->up_lin = (p->up_dst % p->up_src) != 0;
            int kk = std::max(1, (target + p->upL / 2) / p->upL);
            for (int d = 0; d <= kk; d++) {
                if (kk - d >= 1 && hop192 % (p->upL * (kk - d)) == 0 && (p->upM * (kk - d)) % 8 == 0) { kk -= d; break; }
                if (hop192 % (p->upL * (kk + d)) == 0 && (p->upM * (kk + d)) % 8 == 0) { kk += d; break; }
            }
            p->upLin = p->upM * kk;
            p->upLout = p->upL * kk;
            const int al = p->up_alloc;
            bank.assign((size_t)(p->up_pc + 1) * al, 0.0f);
            amx::swr_bank(fs, kfs, bank.data());
            // resample_init's extra row pc: row 0 one tap later within the row (the
            // interpolation partner of the last phase)
            for (int i = 0; i < al; i++) bank[(size_t)p->up_pc * al + i] = bank[(i + al - 1) % al];
            // M == 1: the unrolled kernels (phase pattern static, phase 0 the identity)
            bool ident0 = p->up_taps == 32 && bank[15] == 1.0f;
            for (int i = 0; i < 32 && ident0; i++) ident0 = ident0 && (i == 15 || bank[i] == 0.0f);
            p->up_static = (p->upM == 1 && (p->upL == 1 || p->upL == 2 || p->upL == 4) && ident0 && !p->up_lin &&
                            p->upLin % 8 == 0) ? p->upL : 0;
        }
    } else {
        // already 192 kHz: ffmpeg inserts no resampler ahead of af_loudnorm, only the s16
        // -> dbl conversion x / 32768; a one-phase bank that is the unit impulse makes
        // k_ln_upsample produce exactly that (every other tap adds 0).  The measurement
        // takes the resampler path with that identity (L = M = 1, k_up<1>): one pass over
        // the samples -- K filter, peaks and the hop pieces' energy terms -- where the
        // native path ran the GEMV and then the filter again (k_kw1 + k_kw2).
        // AMX_K192_NATIVE=1 keeps the native path (measurements).
        bank.assign(32, 0.0f);
        bank[15] = 1.0f;
        if (std::getenv("AMX_K192_NATIVE") == nullptr) {
            p->resamp = 1;
            p->upL = p->upM = 1;
            p->up_pc = 1;
            p->up_taps = p->up_alloc = 32;
            p->up_src = p->up_dst = 1;
            p->up_lin = 0;
            p->upLin = p->upLout = 480;            // 40 K segments per 100 ms hop
            p->up_static = 1;
        }
    }
    p->hop = (kfs + 5) / 10;                   // libebur128 samples_in_100ms at 192 kHz
    {
        const int chain_hop = (fs + 5) / 10;
        p->Lkw = 128 < chain_hop ? 128 : chain_hop / AMX_TF_FRAMES * AMX_TF_FRAMES;
    }
    ChainDev &cd = p->cd;
    memset(&cd, 0, sizeof cd);
    cd.fs = fs;
    // mono int16 is duplicated to stereo on the device first (k_pcm_to_s16), so the
    // chain reads stereo int16 frames
    p->mono16 = (desc->input_s16 && desc->channels_in == 1) ? 1 : 0;
    cd.chin = p->mono16 ? 2 : desc->channels_in;
    cd.in_s16 = desc->input_s16 ? 1 : 0;
    cd.analog_on = desc->analog_on ? 1 : 0;
    cd.has_lut = desc->tanh_lut ? 1 : 0;
    cd.drive = desc->analog_drive;
    for (int k = 0; k < 6; k++) {
        cd.an_lo[k] = desc->analog_lo_ba[k];
        cd.an_hi[k] = desc->analog_hi_ba[k];
    }
    cd.an_glo1 = desc->analog_lo_gain - 1.0;
    cd.an_ghi1 = desc->analog_hi_gain - 1.0;
    // EQ stages and the compact state model
    int mask = 0, D = 0;
    for (int s = 0; s < 4; s++) {
        int kind = desc->eq_kind[s];
        int want = (s == 0 || s == 3) ? 1 : 2;
        if (kind != 0 && kind != want) {
            delete p;
            return fail(AMX_EINVAL, "eq stage %d: kind %d not supported at this position", s, kind);
        }
        EqStageDev &st = cd.st[s];
        st.kind = kind;
        if (!kind) continue;
        mask |= 1 << s;
        D += kind == 1 ? 2 : 8;
        st.neg = desc->eq_gain_db[s] < 0 ? 1 : 0;
        st.g = desc->eq_gain[s];
        st.gm1 = desc->eq_gain[s] - 1.0;
        st.gf = (float)desc->eq_gain[s];
        for (int k = 0; k < 24; k++) st.c[k] = desc->eq_coef[s][k];
    }
    {   // compact register-resident coefficients (amx_dev.hpp eq_chain)
        int c = 0;
        for (int s = 0; s < 4; s++) {
            const EqStageDev &st = cd.st[s];
            if (!st.kind) continue;
            const double *k = st.c;
            int nsec = st.kind == 1 ? 1 : 4;
            for (int q = 0; q < nsec; q++) {
                cd.eqc[c++] = k[6 * q + 0];
                cd.eqc[c++] = k[6 * q + 1];
                cd.eqc[c++] = k[6 * q + 2];
                cd.eqc[c++] = k[6 * q + 4];
                cd.eqc[c++] = k[6 * q + 5];
            }
            if (st.kind == 2) cd.eqc[c++] = st.gm1;
            else if (!st.neg) cd.eqc[c++] = st.gm1;
            else {
                const bool first = (mask & ((1 << s) - 1)) == 0;   // stage sees the float32 column
                cd.eqc[c++] = first ? (double)st.gf : st.g;
            }
        }
    }
    cd.eq_mask = mask;
    cd.eq_dim = D;
    p->mask = mask;
    p->D = D;
    cd.width_on = desc->width_on ? 1 : 0;
    cd.width = desc->width;
    cd.mb_on = p->mb = desc->multiband_on ? 1 : 0;
    for (int k = 0; k < 12; k++) {
        cd.xlo[k] = desc->xover_lo_sos[k];
        cd.xhi[k] = desc->xover_hi_sos[k];
    }
    cd.look = (int32_t)(5.0 * (fs / 1000.0));
    // K-weighting coefficients (libebur128 ebur128_init_filter)
    {
        double f0 = 1681.974450955533, G = 3.999843853973347, Q = 0.7071752369554196;
        double K = std::tan(M_PI * f0 / (double)kfs);
        double Vh = std::pow(10.0, G / 20.0);
        double Vb = std::pow(Vh, 0.4996667741545416);
        double pb[3] = {0.0, 0.0, 0.0}, pa[3] = {1.0, 0.0, 0.0};
        double rb[3] = {1.0, -2.0, 1.0}, ra[3] = {1.0, 0.0, 0.0};
        double a0 = 1.0 + K / Q + K * K;
        pb[0] = (Vh + Vb * K / Q + K * K) / a0;
        pb[1] = 2.0 * (K * K - Vh) / a0;
        pb[2] = (Vh - Vb * K / Q + K * K) / a0;
        pa[1] = 2.0 * (K * K - 1.0) / a0;
        pa[2] = (1.0 - K / Q + K * K) / a0;
        f0 = 38.13547087602444;
        Q = 0.5003270373238773;
        K = std::tan(M_PI * f0 / (double)kfs);
        ra[1] = 2.0 * (K * K - 1.0) / (1.0 + K / Q + K * K);
        ra[2] = (1.0 - K / Q + K * K) / (1.0 + K / Q + K * K);
        // libebur128 multiplies the two sections into one 4th-order direct form II;
        // its state (~1/(1-p)^2 ~ 1e5 x signal at 96 kHz) makes the A^L scan
        // ill-conditioned, so the GPU runs the same two sections as DF-II-T biquads.
        for (int k = 0; k < 3; k++) {
            cd.kw1[k] = pb[k];
            cd.kw1[3 + k] = pa[k];
            cd.kw2[k] = rb[k];
            cd.kw2[3 + k] = ra[k];
        }
        // the fused direct form itself, for the one place that runs libebur128's filter
        // sample by sample (loudnorm's r128_out, amx_loudnorm.hip)
        p->kdf_b[0] = pb[0] * rb[0];
        p->kdf_b[1] = pb[0] * rb[1] + pb[1] * rb[0];
        p->kdf_b[2] = pb[0] * rb[2] + pb[1] * rb[1] + pb[2] * rb[0];
        p->kdf_b[3] = pb[1] * rb[2] + pb[2] * rb[1];
        p->kdf_b[4] = pb[2] * rb[2];
        p->kdf_a[0] = pa[0] * ra[0];
        p->kdf_a[1] = pa[0] * ra[1] + pa[1] * ra[0];
        p->kdf_a[2] = pa[0] * ra[2] + pa[1] * ra[1] + pa[2] * ra[0];
        p->kdf_a[3] = pa[1] * ra[2] + pa[2] * ra[1];
        p->kdf_a[4] = pa[2] * ra[2];
    }
    // compressor tables (pydub compress_dynamic_range, exact C math == CPython math)
    std::vector<double> tabs;
    if (p->mb) {
        tabs.assign((size_t)3 * 3 * 32769, 0.0);
        const double A = 5.0 * (fs / 1000.0), R = 50.0 * (fs / 1000.0);
        for (int b = 0; b < 3; b++) {
            double thr = 32768.0 * std::pow(10.0, desc->comp_threshold_db[b] / 20.0);
            double ratio = desc->comp_ratio[b];
            if (ratio == 0.0) {
                delete p;
                return fail(AMX_EINVAL, "compressor ratio must be non-zero");
            }
            int rthr = 0;
            while (rthr <= 32768 && !((double)rthr > thr)) rthr++;
            cd.rthr[b] = rthr;
            double k = 1.0 - (1.0 / ratio);
            double ln10 = std::log(10.0);
            double *mt = &tabs[(size_t)b * 3 * 32769];
            for (int r = 0; r <= 32768; r++) {
                double m;
                if (desc->comp_m_table[b]) {
                    m = desc->comp_m_table[b][r];
                } else {
                    double over = 0.0;
                    if (r != 0) {
                        double db = 20 * (std::log((double)r / thr) / ln10);
                        over = (0 > db) ? 0.0 : db;
                    }
                    m = k * over;
                }
                mt[r] = m;
                mt[32769 + r] = m / A;
                mt[2 * 32769 + r] = m / R;
            }
            int rq = 0;
            while (rq <= 32768 && mt[rq] == 0.0) rq++;
            cd.rq[b] = rq;
        }
        // the device forms m / A as q = m (1/A), q + (m - q A) (1/A) (two FMAs, exact
        // to the IEEE quotient by Markstein's theorem for a correctly rounded 1/A);
        // checked here for every m the tables can produce
        {
            static const double exc[16] = {
                0x1.a934f0979a371p+1, -0x1.34413509f79ffp-2, 0x1.9dc1da994fd21p-59,
                -0x1.f48ad494ea3e9p-53, 0x1.26bb1bbb55516p+1, 0x1.ade156a5dcb37p-26,
                0x1.28af3fca7ab0cp-22, 0x1.71dee623fde64p-19, 0x1.a01997c89e6b0p-16,
                0x1.a01a014761f6ep-13, 0x1.6c16c1852b7b0p-10, 0x1.1111111122322p-7,
                0x1.55555555502a1p-5, 0x1.5555555555511p-3, 0x1.000000000000bp-1, 0.05};
            for (int i = 0; i < 16; i++) cd.exc[i] = exc[i];
        }
        cd.env_A = A;
        cd.env_R = R;
        cd.env_rA = 1.0 / A;
        cd.env_rR = 1.0 / R;
        cd.env_guess = 1;                                   // (measurements: AMX_ENV_GUESS=0)
        if (const char *ev = std::getenv("AMX_ENV_GUESS")) cd.env_guess = std::atoi(ev) != 0;
        cd.env_rcp = 1;
        for (size_t i = 0; i < (size_t)3 * 3 * 32769 && cd.env_rcp; i += 1) {
            if (i % (3 * 32769) >= 32769) continue;
            const double m = tabs[i];
            const double qa = m * cd.env_rA, qr = m * cd.env_rR;
            const double ca = std::fma(std::fma(-qa, A, m), cd.env_rA, qa);
            const double cr = std::fma(std::fma(-qr, R, m), cd.env_rR, qr);
            if (ca != m / A || cr != m / R) cd.env_rcp = 0;
        }
    }
    // ------------------------------------------------ chunks, tracks, segments
    int n_tracks = 0;
    for (int c = 0; c < n_chunks; c++) {
        if (chunks[c].frames < 0 || chunks[c].in_offset < 0 || chunks[c].track < 0) {
            delete p;
            return fail(AMX_EINVAL, "chunk %d: negative field", c);
        }
        if (c > 0 && chunks[c].track < chunks[c - 1].track) {
            delete p;
            return fail(AMX_EINVAL, "chunks must be ordered by track");
        }
        n_tracks = chunks[c].track + 1 > n_tracks ? chunks[c].track + 1 : n_tracks;
    }
    p->n_tracks = n_tracks;
    p->n_chunks = n_chunks;
    if (p->mb) {
        // k_env0 runs one resident wave set: env_wg waves per CU (one workgroup per CU),
        // Le the shortest multiple of 128 (>= 1024) whose segments fit it, so no CU runs
        // waves in turn and the warm-up share W / Le shrinks as the job grows
        // (AMX_ENV_WG = 0 is the single-wave-workgroup launch)
        int wg = 2;
        if (const char *ev = std::getenv("AMX_ENV_WG")) wg = std::atoi(ev);
        int64_t le_min = 1024;                                   // (measurements: AMX_ENV_LEMIN)
        if (const char *ev = std::getenv("AMX_ENV_LEMIN")) le_min = std::max(128, std::atoi(ev)) / 128 * 128;
        if (wg > 0) {
            p->env_wg = std::min(wg, 4);
            p->env_pin = 1;
            if (!env_le) {
                int dev = 0, ncu = 0;
                if (hipGetDevice(&dev) != hipSuccess ||
                    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 3)
                    ncu = 256;
                // segments per band: W waves of one band per CU, the CUs shared by the t
                // bands that are active (t = 3: every band; the tables for 1 and 2 active
                // bands have shorter segments, floor 512 frames; AMX_ENV_BANDTAB=0 keeps
                // the 3-band table for every count)
                int bandtab = 1;
                if (const char *ev = std::getenv("AMX_ENV_BANDTAB")) bandtab = std::atoi(ev);
                int64_t total = 0;
                for (int c = 0; c < n_chunks; c++) total += chunks[c].frames;
                for (int t = 3; t >= 1; t--) {
                    const int64_t fit = (int64_t)(ncu / t) * 64 * p->env_wg;
                    int64_t lo = (t == 3 || std::getenv("AMX_ENV_LEMIN")) ? le_min : 512;
                    if (const char *ev = std::getenv("AMX_ENV_LEMIN2"))           // (measurements)
                        if (t < 3) lo = std::max(128, std::atoi(ev)) / 128 * 128;
                    int64_t Le = std::max<int64_t>(lo, (total / fit + 127) / 128 * 128);
                    for (;; Le += 128) {
                        int64_t ne = 0;
                        for (int c = 0; c < n_chunks; c++) ne += (chunks[c].frames + Le - 1) / Le;
                        if (ne <= fit || Le >= (int64_t)1 << 24) break;
                    }
                    p->Le_t[t] = (t == 3 || bandtab) ? (int)Le : p->Le_t[3];
                }
                p->Le = p->Le_t[3];
            }
        }
        for (int t = 1; t <= 3; t++)
            if (p->Le_t[t] == 0) p->Le_t[t] = p->Le;
        // the warm-up: since the fix-up re-runs broken segments in parallel (round 5), a
        // shorter warm-up pays where it is most of a lane's frames (C3: Le 1 408 / 896,
        // C4: 8.5 k); a 60-min track's long segments keep 2 304
        if (desc->env_warm_frames < 0 && p->Le_t[3] <= 16384) p->warm = 1536;
    }
    int64_t loc = 0, outo = 0;
    p->spans.assign(n_tracks, SpanDev{});
    std::vector<int> track_seen(n_tracks, 0);
    for (int c = 0; c < n_chunks; c++) {
        ChunkDev ch{};
        ch.in_off = chunks[c].in_offset;
        ch.loc_off = loc;
        ch.out_off = outo;
        ch.n = chunks[c].frames;
        int64_t n1 = ch.n, n2 = ch.n;
        if (p->mb && ch.n > 0) {
            n1 = overlay_len(ch.n, fs);
            n2 = overlay_len(n1, fs);
        }
        ch.out_n = n2;
        ch.track = chunks[c].track;
        p->in_frames = std::max(p->in_frames, (int64_t)(chunks[c].in_offset + chunks[c].frames));
        ch.seg0 = (int32_t)p->segs.size();
        int64_t ns = (ch.n + p->L - 1) / p->L;
        ch.nseg = (int32_t)ns;
        add_blocks(p->blks, ch.seg0, (int32_t)ns, c);
        for (int64_t k = 0; k < ns; k++) {
            SegDev s{};
            s.pos = k * p->L;
            s.chunk = c;
            s.len = (int32_t)((ch.n - s.pos) < p->L ? (ch.n - s.pos) : p->L);
            s.first = ch.seg0;
            s.last = (k == ns - 1) ? 1 : 0;
            p->segs.push_back(s);
        }
        SpanDev &sp = p->spans[ch.track];
        if (!track_seen[ch.track]) {
            sp.out_off = outo;
            track_seen[ch.track] = 1;
        }
        sp.out_n += n2;
        p->chunks.push_back(ch);
        p->n1tab.push_back(n1);
        p->max_chunk_out = n2 > p->max_chunk_out ? n2 : p->max_chunk_out;
        p->max_chunk_n = ch.n > p->max_chunk_n ? ch.n : p->max_chunk_n;
        p->an_blocks += (ch.n + 4095) / 4096;
        if (ch.n > 0 && ((ch.in_off & 1) != 0 || ch.n < 4)) p->an_vec = 0;
        loc += (ch.n + 15) / 16 * 16;   // chunk rows of per-frame scratch start 16-frame aligned
        outo += n2;
    }
    if (loc >= ((int64_t)1 << 31) || outo >= ((int64_t)1 << 31)) {
        delete p;   // the chain kernels' row offsets are 32-bit (amx_chain.hip VRows)
        return fail(AMX_ERANGE, "a plan holds fewer than 2^31 frames (%lld): split the batch",
                    (long long)std::max(loc, outo));
    }
    p->nloc = loc;
    if (p->mb) {
        // envelope segment tables (ChainDev::etab): per table the chunks cut into Le_t-frame
        // segments; segment indices (SegDev::first, eseg0) are table-relative
        int ld = 0;
        for (int t = 3; t >= 1; t--) {
            if (t < 3 && p->Le_t[t] == p->Le_t[3]) {
                p->cd.etab[t] = p->cd.etab[3];
                continue;
            }
            const int Le = p->Le_t[t];
            const int es_off = (int)p->esegs.size(), ch_off = (int)p->eseg0.size();
            for (int c = 0; c < n_chunks; c++) {
                const int64_t n = p->chunks[c].n;
                const int64_t ne = (n + Le - 1) / Le;
                p->eseg0.push_back((int)p->esegs.size() - es_off);
                p->neseg.push_back((int)ne);
                for (int64_t k = 0; k < ne; k++) {
                    SegDev e{};
                    e.pos = k * Le;
                    e.chunk = c;
                    e.len = (int32_t)((n - e.pos) < Le ? (n - e.pos) : Le);
                    e.first = p->eseg0.back();
                    e.last = (k == ne - 1) ? 1 : 0;
                    p->esegs.push_back(e);
                }
            }
            const int n_es = (int)p->esegs.size() - es_off;
            p->cd.etab[t].es_off = es_off;
            p->cd.etab[t].n_es = n_es;
            p->cd.etab[t].ch_off = ch_off;
            p->cd.etab[t].Le = Le;
            ld = std::max(ld, n_es);
        }
        p->cd.etab[0] = p->cd.etab[3];
        p->cd.es_ld = ld;
        p->n_es = ld;
    }
    p->out_frames = outo;
    p->n_seg = (int)p->segs.size();
    // K-weighting segments per track span, on the measurement stream: output j of
    // the 192 kHz stream is made from the chain frames around floor(j M / L); a span
    // of chain frames [f0, f0 + n) of its track owns outputs [J(f0), J(f0 + n)),
    // J(f) = ceil(f L / M); segment q = chain frames f0 + q Lin + [0, Lin) = outputs
    // J(f0) + q Lout + [0, Lout)
    const int64_t uL = p->upL, uM = p->upM, uS = p->up_src, uD = p->up_dst, uP = p->up_pc;
    auto J = [&](int64_t f) { return (f * uL + uM - 1) / uM; };
    // (J(f0) dst - f0 pc src): the phase pattern -- output J(f0)'s position past frame f0
    // in units of 1 / (pc src) frame (exact rates: (J(f0) M - f0 L) src) -- equal for all spans
    int64_t pattern = -1;
    for (int t = 0; t < n_tracks; t++) {
        SpanDev &sp = p->spans[t];
        sp.tframe0 = track_frame0 ? track_frame0[t] : 0;
        sp.ttotal = track_total_frames ? track_total_frames[t] : sp.out_n;
        sp.kseg0 = (int32_t)p->ksegs.size();
        const int Lseg = p->resamp ? p->upLout : p->Lkw;
        const int Lsin = p->resamp ? p->upLin : p->Lkw;
        if (p->resamp && p->up_ok) {
            sp.m_tframe0 = J(sp.tframe0);
            sp.m_n = J(sp.tframe0 + sp.out_n) - sp.m_tframe0;
            sp.m_total = J(sp.ttotal);
            const int64_t pat = sp.m_tframe0 * uD - sp.tframe0 * uP * uS;
            if (sp.out_n > 0) {
                if (pattern >= 0 && pat != pattern) {
                    delete p;
                    return fail(AMX_EINVAL, "spans with different 192 kHz phase patterns in one plan");
                }
                pattern = pat;
            }
        } else {
            sp.m_tframe0 = sp.tframe0;
            sp.m_n = sp.out_n;
            sp.m_total = sp.ttotal;
        }
        sp.edge_lo = sp.tframe0 > 0 ? 1 : 0;
        sp.edge_hi = sp.tframe0 + sp.out_n < sp.ttotal ? 1 : 0;
        int64_t nk = (p->resamp && !p->up_ok) ? 0 : (sp.m_n + Lseg - 1) / Lseg;
        sp.nkseg = (int32_t)nk;
        add_blocks(p->kblks, sp.kseg0, (int32_t)nk, t);
        for (int64_t k = 0; k < nk; k++) {
            KwSegDev s{};
            s.out_pos = sp.out_off + k * Lsin;
            s.tframe = sp.m_tframe0 + k * Lseg;
            s.track = t;
            s.len = (int32_t)((sp.m_n - k * Lseg) < Lseg ? (sp.m_n - k * Lseg) : Lseg);
            s.first = sp.kseg0;
            s.last = (k == nk - 1) ? 1 : 0;
            p->ksegs.push_back(s);
        }
        p->max_span = sp.out_n > p->max_span ? sp.out_n : p->max_span;
        p->max_nkseg = sp.nkseg > p->max_nkseg ? sp.nkseg : p->max_nkseg;
        p->max_hops = std::max(p->max_hops, sp.m_total / p->hop + 1);
    }
    if (p->resamp && p->up_ok) {
        // per output n of a segment: the chain frame its window is centred on (relative
        // to the segment's first frame) and its phase
        if (pattern < 0) pattern = 0;
        obase.resize(p->upLout);
        oph.resize(p->upLout);
        owt.resize(p->upLout);
        const float inv = 1.0f / (float)uS;          // the float reciprocal resample.asm forms
        for (int64_t n = 0; n < p->upLout; n++) {
            const int64_t pos = pattern + n * uD;     // (J0 + n) dst - f0 pc src
            const int64_t idx = pos / uS;
            obase[n] = (int32_t)(idx / uP);
            oph[n] = (int32_t)(idx % uP);
            owt[n] = (float)(pos % uS) * inv;
        }
        if (p->up_static && pattern != 0) p->up_static = 0;
        if (!p->up_static && !p->up_lin && p->up_taps == 32) {
            // k_up_poly: frame f of a segment is the base of the outputs n with obase[n]
            // == f (consecutive n; every frame has one when L >= M); the form is (min,
            // max count, a block of TB frames dividing Lin)
            fcnt.assign((size_t)p->upLin, 0);
            bool ok = p->upL >= p->upM;
            for (int64_t n = 0; n < p->upLout && ok; n++) {
                ok = obase[n] >= 0 && obase[n] < p->upLin && (n == 0 || obase[n] >= obase[n - 1]);
                if (ok) fcnt[obase[n]]++;
            }
            int cmin = 1 << 30, cmax = 0;
            for (int32_t c : fcnt) { cmin = std::min(cmin, c); cmax = std::max(cmax, c); }
            const int tb = p->upLin % 8 == 0 ? 8 : (p->upLin % 7 == 0 ? 7 : 0);
            if (ok && cmin >= 1 && tb) p->up_poly = amx::up_poly_form(cmin, cmax, tb);
            if (const char *ev = std::getenv("AMX_UP_POLY")) p->up_poly = std::atoi(ev) ? p->up_poly : 0;
            if (p->up_poly) {
                bankn.resize((size_t)p->upLout * 32);
                for (int64_t n = 0; n < p->upLout; n++)
                    for (int k = 0; k < 32; k++) bankn[(size_t)n * 32 + k] = bank[(size_t)oph[n] * 32 + k];
            }
        }
    }
    p->n_kseg = (int)p->ksegs.size();
    // the segments the unrolled 192 kHz kernel leaves to the general one: windows that
    // reach past the span's frames, partial segments, segments holding a hop boundary
    // (the same test as up_fast_seg in amx_loud192.hip)
    std::vector<int32_t> slow;
    if (p->resamp && p->up_ok) {
        if (p->up_static || p->up_poly) {
            for (int32_t j = 0; j < p->n_kseg; j++) {
                const KwSegDev &sg = p->ksegs[j];
                const SpanDev &sp = p->spans[sg.track];
                const int64_t g0 = sg.out_pos - sp.out_off;
                const int64_t split = (sg.tframe / p->hop + 1) * p->hop - sg.tframe;
                const bool fast = g0 - 15 >= 0 && g0 + p->upLin + 17 <= sp.out_n &&
                                  sg.len == p->upLout && split >= p->upLout;
                if (!fast) slow.push_back(j);
            }
            p->n_slow = (int64_t)slow.size();
        } else {
            p->n_slow = p->n_kseg;       // every segment, d_slow NULL
        }
    }
    // hop splits on 16-frame tile boundaries (k_kw2 picks the hop piece per tile)
    p->kw_aligned = (!p->resamp && p->hop % AMX_TF_FRAMES == 0 && p->Lkw % AMX_TF_FRAMES == 0) ? 1 : 0;
    for (int t = 0; t < n_tracks; t++)
        if (p->spans[t].tframe0 % AMX_TF_FRAMES) p->kw_aligned = 0;
    // the K-filter segment grid equals the chain's when there is no multiband
    // (output frames == input frames) and every chunk but a span's last is whole
    // segments long: k_front2 then does loudness pass 1 on the output it writes
    p->fuse_kw = (!p->resamp && !p->mb && p->Lkw == p->L && p->n_kseg == p->n_seg && !desc->measure_only &&
                  !p->sc) ? 1 : 0;
    for (int c = 0; c < n_chunks && p->fuse_kw; c++) {
        const bool span_last = (c == n_chunks - 1) || (chunks[c + 1].track != chunks[c].track);
        if (!span_last && (p->chunks[c].n % p->L) != 0) p->fuse_kw = 0;
    }
    p->n_blk = (int)p->blks.size();
    p->n_kblk = (int)p->kblks.size();

    // ------------------------------------------------------- LTI models
    const double tol = 1e-22;
    std::vector<double> G, M, Mp, Gx, Mx, Mpx, Gkw, Mkw, Mpkw, qh, qt;
    if (D > 0) {
        Lti eq;
        eq.derive(D, [&](LD *z, LD x) {
            int o = 0;
            for (int s = 0; s < 4; s++) {
                const EqStageDev &st = cd.st[s];
                if (st.kind == 1) {
                    shelf_step_h(st.c, z + o, x, st.neg, st.gm1);
                    o += 2;
                } else if (st.kind == 2) {
                    LD b = x;
                    for (int k = 0; k < 4; k++) b = sos_step_h(st.c + 6 * k, z + o + 2 * k, b);
                    x = x + b * (LD)st.gm1;
                    o += 8;
                }
            }
        });
        G = eq.gemv_table(p->L);
        M = eq.pow(p->L);
        p->lev_eq = eq.window_powers((int64_t)p->L * AMX_SCAN_S, tol, 16, Mp);
        if (p->lev_eq < 0) {
            delete p;
            return fail(AMX_ERANGE, "EQ decays too slowly for %d-frame segments; raise seg_frames", p->L);
        }
    }
    if (p->mb) {
        Lti xo;
        xo.derive(AMX_XO_DIM, [&](LD *z, LD x) {
            LD l = sos_step_h(cd.xlo, z, x);
            sos_step_h(cd.xlo + 6, z + 2, l);
            LD h = sos_step_h(cd.xhi, z + 4, x);
            sos_step_h(cd.xhi + 6, z + 6, h);
        });
        Gx = xo.gemv_table(p->L);
        Mx = xo.pow(p->L);
        p->lev_x = xo.window_powers((int64_t)p->L * AMX_SCAN_S, tol, 16, Mpx);
        if (p->lev_x < 0) {
            delete p;
            return fail(AMX_ERANGE, "crossover decays too slowly for %d-frame segments", p->L);
        }
    }
    {
        Lti &kw = p->kw_model;
        kw.derive(AMX_KW_DIM, [&](LD *z, LD x) {
            LD y = sos_step_h(cd.kw1, z, x);
            sos_step_h(cd.kw2, z + 2, y);
        });
        const int Lseg = p->resamp ? std::max(1, p->upLout) : p->Lkw;
        if (p->resamp) {
            // the measurement kernels keep no GEMV table: their pass over the samples
            // runs the filter from rest and needs the free-response rows C A^n and
            // their Gram sums (amx_loud192.hip k_up / k_up_energy)
            LD Cr[AMX_KW_DIM];
            for (int k = 0; k < AMX_KW_DIM; k++) {
                LD z[AMX_KW_DIM] = {0.0L, 0.0L, 0.0L, 0.0L};
                z[k] = 1.0L;
                const LD y1 = sos_step_h(cd.kw1, z, 0.0L);
                Cr[k] = sos_step_h(cd.kw2, z + 2, y1);
            }
            Gkw.assign((size_t)Lseg * AMX_KW_DIM, 0.0);
            qh.assign((size_t)(Lseg + 1) * 16, 0.0);
            qt.assign((size_t)(Lseg + 1) * 16, 0.0);
            std::vector<LD> r(Cr, Cr + AMX_KW_DIM), t(AMX_KW_DIM), gl((size_t)Lseg * AMX_KW_DIM);
            std::vector<LD> qa(16, 0.0L);
            for (int n = 0; n < Lseg; n++) {
                for (int d = 0; d < AMX_KW_DIM; d++) {
                    gl[(size_t)n * AMX_KW_DIM + d] = r[d];
                    Gkw[(size_t)n * AMX_KW_DIM + d] = (double)r[d];
                }
                for (int u = 0; u < 4; u++)
                    for (int w = 0; w < 4; w++) {
                        qa[u * 4 + w] += r[u] * r[w];
                        qh[(size_t)(n + 1) * 16 + u * 4 + w] = (double)qa[u * 4 + w];
                    }
                for (int d = 0; d < AMX_KW_DIM; d++) {     // r <- r A
                    LD acc = 0.0L;
                    for (int k = 0; k < AMX_KW_DIM; k++) acc += r[k] * kw.A[(size_t)k * AMX_KW_DIM + d];
                    t[d] = acc;
                }
                r = t;
            }
            std::fill(qa.begin(), qa.end(), 0.0L);
            for (int n = Lseg - 1; n >= 0; n--) {
                const LD *g = &gl[(size_t)n * AMX_KW_DIM];
                for (int u = 0; u < 4; u++)
                    for (int w = 0; w < 4; w++) {
                        qa[u * 4 + w] += g[u] * g[w];
                        qt[(size_t)n * 16 + u * 4 + w] = (double)qa[u * 4 + w];
                    }
            }
        } else {
            Gkw = kw.gemv_table(Lseg);
        }
        Mkw = kw.pow(Lseg);
        // up to 32 block powers: a track measured at its own 192 kHz rate (loudnorm's
        // output) needs ~20 with 128-frame segments (the 38 Hz pole)
        p->lev_kw = kw.window_powers((int64_t)Lseg * AMX_SCAN_S, tol, 32, Mpkw);
        if (p->lev_kw < 0) {
            delete p;
            return fail(AMX_ERANGE, "K-weighting decays too slowly for %d-frame segments", Lseg);
        }
        p->tail_pow.assign((size_t)n_tracks * 16, 0.0);
        for (int t = 0; t < n_tracks; t++) {
            const SpanDev &sp = p->spans[t];
            if (sp.nkseg == 0) continue;
            int len_last = p->ksegs[sp.kseg0 + sp.nkseg - 1].len;
            Mat P = kw.pow(len_last);
            for (int k = 0; k < 16; k++) p->tail_pow[(size_t)t * 16 + k] = P[k];
        }
    }
    // histogram boundaries (libebur128 init_histogram)
    double bounds[1001], energies[1000];
    bounds[0] = std::pow(10.0, (-70.0 + 0.691) / 10.0);
    for (int i = 1; i < 1001; ++i) bounds[i] = std::pow(10.0, ((double)i / 10.0 - 70.0 + 0.691) / 10.0);
    for (int i = 0; i < 1000; ++i) energies[i] = std::pow(10.0, ((double)i / 10.0 - 69.95 + 0.691) / 10.0);

    // ------------------------------------------------------- upload
    int rc = AMX_OK;
#define UP(dst, src, n)                          \
    if ((rc = upload(&dst, src, n)) != AMX_OK) { \
        amx_plan_free(p);                        \
        return rc;                               \
    }
    UP(p->d_cd, &p->cd, 1);
    UP(p->d_chunks, p->chunks.data(), p->chunks.size());
    UP(p->d_segs, p->segs.data(), p->segs.size());
    UP(p->d_ksegs, p->ksegs.data(), p->ksegs.size());
    UP(p->d_spans, p->spans.data(), p->spans.size());
    UP(p->d_blks, p->blks.data(), p->blks.size());
    UP(p->d_kblks, p->kblks.data(), p->kblks.size());
    UP(p->d_n1, p->n1tab.data(), p->n1tab.size());
    UP(p->d_esegs, p->esegs.data(), p->esegs.size());
    UP(p->d_eseg0, p->eseg0.data(), p->eseg0.size());
    UP(p->d_neseg, p->neseg.data(), p->neseg.size());
    UP(p->d_G, G.data(), G.size());
    UP(p->d_M, M.data(), M.size());
    UP(p->d_Mp, Mp.data(), Mp.size());
    UP(p->d_Gx, Gx.data(), Gx.size());
    UP(p->d_Mx, Mx.data(), Mx.size());
    UP(p->d_Mpx, Mpx.data(), Mpx.size());
    UP(p->d_Gkw, Gkw.data(), Gkw.size());
    UP(p->d_Mkw, Mkw.data(), Mkw.size());
    UP(p->d_Mpkw, Mpkw.data(), Mpkw.size());
    UP(p->d_tabs, tabs.data(), tabs.size());
    UP(p->d_bounds, bounds, 1001);
    UP(p->d_energies, energies, 1000);
    UP(p->d_tailpow, p->tail_pow.data(), p->tail_pow.size());
    UP(p->d_obase, obase.data(), obase.size());
    UP(p->d_qh, qh.data(), qh.size());
    UP(p->d_qt, qt.data(), qt.size());
    UP(p->d_oph, oph.data(), oph.size());
    UP(p->d_owt, owt.data(), owt.size());
    if (!slow.empty()) UP(p->d_slow, slow.data(), slow.size());
    UP(p->d_bank, bank.data(), bank.size());
    if (p->up_poly) {
        UP(p->d_fcnt, fcnt.data(), fcnt.size());
        UP(p->d_bankn, bankn.data(), bankn.size());
    }
    {
        std::vector<unsigned int> zero((size_t)(p->n_tracks > 0 ? p->n_tracks : 1), 0u);
        UP(p->d_pcnt, zero.data(), zero.size());
        const size_t nb = (size_t)amx::peak_reduce_blocks(p->max_nkseg);
        UP(p->d_ppart, (const int *)nullptr, (size_t)(p->n_tracks > 0 ? p->n_tracks : 1) * (nb ? nb : 1) * 4);
        for (const SpanDev &sp : p->spans) p->any_empty_span |= sp.nkseg == 0 ? 1 : 0;
    }
    if (desc->tanh_lut) UP(p->d_lut, desc->tanh_lut, 65536);
    if (p->sc && desc->eq_in_lut) UP(p->d_in_lut, desc->eq_in_lut, 65536);
    if (desc->tanh_lut && desc->analog_on) {
        // numpy's float32 tanh is odd: lut[32768 - k] == -lut[32768 + k] bit for bit (sign
        // of zero included) for every k; then tanh(s) = sign(s) * half[|s|] with half[k] =
        // lut[32768 + k] and half[32768] = -lut[0].  Checked per table: any pair that
        // differs keeps the full table in global memory (k_front1s).
        const uint32_t *b = reinterpret_cast<const uint32_t *>(desc->tanh_lut);
        bool odd = true;
        for (int k = 1; k < 32768 && odd; k++) odd = b[32768 - k] == (b[32768 + k] ^ 0x80000000u);
        // (tests: AMX_F1 = 2 runs the full-table form k_front1s, the path a table that is
        // not odd takes)
        if (const char *ev = std::getenv("AMX_F1")) p->f1_mode = std::atoi(ev) == AMX_F1_FULL ? AMX_F1_FULL : AMX_F1_SPLIT;
        if (!odd) p->f1_mode = AMX_F1_FULL;
        if (p->f1_mode == AMX_F1_SPLIT) {
            std::vector<float> half(32769);
            for (int k = 0; k < 32768; k++) half[k] = desc->tanh_lut[32768 + k];
            half[32768] = -desc->tanh_lut[0];
            UP(p->d_lut_half, half.data(), half.size());
        }
    }
#undef UP
    // ------------------------------------------------------- workspace layout
    size_t off = 0;
    const size_t nseg = (size_t)p->n_seg, nl = (size_t)p->nloc, nk = (size_t)p->n_kseg;
    p->o_a16 = (size_t)align_up(off, nl * 4);
    p->o_e = (size_t)align_up(off, nseg * 2 * (D ? D : 1) * 8);
    p->o_s = (size_t)align_up(off, nseg * 2 * (D ? D : 1) * 8);
    if (p->mb) {
        p->o_p16 = (size_t)align_up(off, nl * 4);
        p->o_ex = (size_t)align_up(off, nseg * 2 * AMX_XO_DIM * 8);
        p->o_sx = (size_t)align_up(off, nseg * 2 * AMX_XO_DIM * 8);
        p->o_bands = (size_t)align_up(off, 3 * nl * 4);
        const size_t ne = (size_t)p->n_es;
        p->o_gain = (size_t)align_up(off, (3 * nl / 16 + 64) * 8);   // envelope checkpoints
        // m rows are read whole-tile by k_env0, from W frames before a chunk to the
        // 16-frame tile past its end: pad the buffer on both sides
        // (and k_gain_overlay reads whole 1024-frame wave tiles)
        // (k_env0's last tiles of a chunk-final segment read up to Le frames past it)
        const size_t mpad = (size_t)std::max(std::max(p->warm, p->Le), 1024) + 64;
        p->o_m = (size_t)align_up(off, (3 * nl + 2 * mpad) * 2) + mpad * 2;   // u16 r
        p->o_esv = (size_t)align_up(off, 3 * ne * 8);
        p->o_ee0 = (size_t)align_up(off, 3 * ne * 8);
        p->o_eflags = (size_t)align_up(off, (AMX_ENV_LIST + 3) * 4);   // + band words, list lengths, flag
        p->o_eact = (size_t)align_up(off, 3 * ne * 4);
        p->o_ehead = (size_t)align_up(off, 3 * ne * 4);   // chain-head marks
        p->o_elist = (size_t)align_up(off, 3 * ne * 4);   // chain-head list
        p->o_eprev = (size_t)align_up(off, 3 * ne * 4);   // nearest earlier active segment
        p->o_elist0 = (size_t)align_up(off, 3 * ne * 4);  // the optimistic re-run list
    }
    if (p->mono16) p->o_dup = (size_t)align_up(off, (size_t)p->in_frames * 4);
    const size_t nb = (size_t)p->n_blk, nkb = (size_t)p->n_kblk;
    p->o_eb = (size_t)align_up(off, nb * 2 * (D ? D : 1) * 8);
    if (p->mb) {
        p->o_ebx = (size_t)align_up(off, nb * 2 * AMX_XO_DIM * 8);
    }
    p->o_ebk = (size_t)align_up(off, nkb * 2 * AMX_KW_DIM * 8);
    p->o_ekw = (size_t)align_up(off, nk * 2 * AMX_KW_DIM * 8);
    p->o_pk = (size_t)align_up(off, nk * 4 * 4);
    p->o_skw = (size_t)align_up(off, nk * 2 * AMX_KW_DIM * 8);
    p->o_parts = (size_t)align_up(off, nk * 4 * 8);
    if (p->resamp) p->o_eterms = (size_t)align_up(off, nk * 2 * 10 * 8);
    p->o_phop = (size_t)align_up(off, nk * 8);
    p->ws_bytes = (off + 255) & ~(size_t)255;
    if (p->resamp && (p->up_static || p->up_poly) && p->n_slow > 0) {
        if (hipStreamCreateWithFlags(&p->up_aux, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&p->up_fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&p->up_join, hipEventDisableTiming) != hipSuccess) {
            amx_plan_free(p);
            return fail(AMX_EHIP, "stream / event creation failed");
        }
    }
    *out = p;
    return AMX_OK;
}

void amx_plan_free(amx_plan *p) {
    if (!p) return;
    void *ptrs[] = {p->d_cd,  p->d_chunks, p->d_segs, p->d_ksegs, p->d_spans,  p->d_blks,
                    p->d_kblks, p->d_n1,   p->d_G,    p->d_M,     p->d_Mp,     p->d_Gx,
                    p->d_Mx,  p->d_Mpx,    p->d_Gkw,  p->d_Mkw,   p->d_Mpkw,   p->d_tabs,
                    p->d_bounds, p->d_tailpow, p->d_lut, p->d_energies, p->d_carryP,
                    p->d_esegs, p->d_eseg0, p->d_neseg, p->d_pcnt, p->d_ppart,
                    p->lim.seg_state, p->lim.cnt, p->d_obase, p->d_oph, p->d_bank,
                    p->d_qh, p->d_qt, p->d_slow, p->d_lut_half, p->d_fcnt, p->d_bankn, p->d_owt,
                    p->d_in_lut};
    for (void *q : ptrs)
        if (q) (void)hipFree(q);
    if (p->up_fork) (void)hipEventDestroy(p->up_fork);
    if (p->up_join) (void)hipEventDestroy(p->up_join);
    if (p->up_aux) (void)hipStreamDestroy(p->up_aux);
    delete p;
}

int amx_plan_get_info(const amx_plan *p, amx_plan_info *info) {
    if (!p || !info) return fail(AMX_EINVAL, "null argument");
    memset(info, 0, sizeof *info);
    info->workspace_bytes = (int64_t)p->ws_bytes;
    info->out_frames = p->out_frames;
    info->n_tracks = p->n_tracks;
    info->n_chunks = p->n_chunks;
    info->n_segments = p->n_seg;
    info->seg_frames = p->L;
    info->scan_levels_eq = p->lev_eq;
    info->scan_levels_xover = p->lev_x;
    info->scan_levels_kw = p->lev_kw;
    info->eq_dim = p->D;
    info->hop_frames = p->hop;
    info->meas_rate = p->meas_native ? p->cd.fs : AMX_MEAS_RATE;
    info->max_hops = p->max_hops;
    return AMX_OK;
}

int amx_plan_track_span(const amx_plan *p, int32_t track, amx_track_span *span) {
    if (!p || !span || track < 0 || track >= p->n_tracks) return fail(AMX_EINVAL, "bad track");
    const SpanDev &s = p->spans[track];
    span->out_offset = s.out_off;
    span->out_frames = s.out_n;
    span->track_frame0 = s.tframe0;
    span->track_frames_total = s.ttotal;
    return AMX_OK;
}

int amx_run_stage(amx_plan *p, int32_t stage, const float *d_in, int16_t *d_out, void *d_ws,
                  void *stream) {
    if (!p || (p->nloc > 0 && (!d_in || !d_out || !d_ws))) return fail(AMX_EINVAL, "null argument");
    if (stage < 0 || stage >= AMX_STAGE_COUNT) return fail(AMX_EINVAL, "bad stage %d", stage);
    if (p->n_seg == 0) return AMX_OK;
    hipStream_t st = (hipStream_t)stream;
    amx::Launch l{p->d_cd, p->d_chunks, p->d_segs, p->n_chunks, p->n_seg, p->L, st, p->d_lut_half,
                  p->f1_mode, p->max_chunk_n, p->an_blocks, p->an_vec};
    int16_t *a16 = wsp<int16_t>(d_ws, p->o_a16);
    double *e = wsp<double>(d_ws, p->o_e), *s = wsp<double>(d_ws, p->o_s);
    int16_t *p16 = p->mb ? wsp<int16_t>(d_ws, p->o_p16) : nullptr;
    double *ex = p->mb ? wsp<double>(d_ws, p->o_ex) : nullptr;
    double *sx = p->mb ? wsp<double>(d_ws, p->o_sx) : nullptr;
    int16_t *bands = p->mb ? wsp<int16_t>(d_ws, p->o_bands) : nullptr;
    double *ck = p->mb ? wsp<double>(d_ws, p->o_gain) : nullptr;
    uint16_t *mframe = p->mb ? wsp<uint16_t>(d_ws, p->o_m) : nullptr;
    double *esv = p->mb ? wsp<double>(d_ws, p->o_esv) : nullptr;
    double *ee0 = p->mb ? wsp<double>(d_ws, p->o_ee0) : nullptr;
    int *eflags = p->mb ? wsp<int>(d_ws, p->o_eflags) : nullptr;
    int *eact = p->mb ? wsp<int>(d_ws, p->o_eact) : nullptr;
    int *ehead = p->mb ? wsp<int>(d_ws, p->o_ehead) : nullptr;
    int *elist = p->mb ? wsp<int>(d_ws, p->o_elist) : nullptr;
    int *eprev = p->mb ? wsp<int>(d_ws, p->o_eprev) : nullptr;
    int *elist0 = p->mb ? wsp<int>(d_ws, p->o_elist0) : nullptr;
    amx::DynLaunch dl{p->d_cd,    p->d_chunks, p->n_chunks, p->d_esegs, p->n_es,
                      p->d_eseg0, p->d_neseg,  p->nloc,     p->max_chunk_n, p->cd.look,
                      p->warm,    p->Le,       p->cd.env_rcp, p->d_tabs, st,
                      p->env_wg,  p->env_pin};
    switch (stage) {
    case AMX_STAGE_FRONT1:
        if (p->mono16) {
            int16_t *dup = wsp<int16_t>(d_ws, p->o_dup);
            HIPCHK(amx::launch_pcm_to_s16(d_in, p->in_frames, 1, AMX_PCM_S16, dup, st));
            d_in = reinterpret_cast<const float *>(dup);
        }
        HIPCHK(amx::launch_front1(l, p->D, (p->cd.chin == 2 && !p->cd.in_s16) ? 2 : 1,
                                  p->cd.analog_on != 0, d_in, p->sc ? p->d_in_lut : p->d_lut, a16, p->d_G, e,
                                  p->sc != 0));
        break;
    case AMX_STAGE_SCAN_EQ:
        if (p->D > 0)
            HIPCHK(amx::launch_scan(p->scan_eq(), e, s, nullptr, wsp<double>(d_ws, p->o_eb), st));
        break;
    case AMX_STAGE_FRONT2:
        if (p->mb)
            HIPCHK(amx::launch_front2(l, p->mask, a16, s, p16, 0, p->d_Gx, ex, nullptr, nullptr,
                                      nullptr, p->sc != 0, p->d_in_lut));
        else if (p->sc)
            HIPCHK(amx::launch_front2(l, p->mask, a16, s, d_out, 1, nullptr, nullptr, nullptr,
                                      nullptr, nullptr, true, p->d_in_lut));
        else if (p->fuse_kw)
            HIPCHK(amx::launch_front2(l, p->mask, a16, s, d_out, 1, nullptr, nullptr, p->d_Gkw,
                                      wsp<double>(d_ws, p->o_ekw), wsp<uint32_t>(d_ws, p->o_pk)));
        else
            HIPCHK(amx::launch_front2(l, p->mask, a16, s, d_out, 1, nullptr, nullptr, nullptr,
                                      nullptr, nullptr));
        break;
    case AMX_STAGE_SCAN_XO:
        if (p->mb)
            HIPCHK(amx::launch_scan(p->scan_xo(), ex, sx, nullptr, wsp<double>(d_ws, p->o_ebx), st));
        break;
    case AMX_STAGE_XOVER:
        if (p->mb) HIPCHK(amx::launch_xover2(l, p16, sx, bands, p->nloc, eflags + AMX_ENV_BACT));
        break;
    case AMX_STAGE_RMS:
        if (p->mb) HIPCHK(amx::launch_rms(dl, bands, mframe, eflags + AMX_ENV_BACT));
        break;
    case AMX_STAGE_ENV:
        if (p->mb)
            HIPCHK(amx::launch_env(dl, mframe, ck, esv, ee0, eact, elist, ehead, eprev, elist0, eflags, p->rounds, 0));
        break;
    case AMX_STAGE_FIX:
        if (p->mb) {
            HIPCHK(amx::launch_env(dl, mframe, ck, esv, ee0, eact, elist, ehead, eprev, elist0, eflags, p->rounds, 1));
            HIPCHK(amx::launch_envseq(dl, mframe, ck, esv, ee0, eact, eflags, p->rounds));
        }
        break;
    case AMX_STAGE_APPLY:
        if (p->mb)
            HIPCHK(amx::launch_gain_overlay(dl, mframe, ck, bands, d_out, p->max_chunk_out, p->d_n1, eact,
                                            eflags + AMX_ENV_BACT));
        break;
    }
    return AMX_OK;
}

int amx_run_chunks(amx_plan *p, const float *d_in, int16_t *d_out, void *d_ws, void *stream) {
    for (int s = 0; s < AMX_STAGE_COUNT; s++) {
        int rc = amx_run_stage(p, s, d_in, d_out, d_ws, stream);
        if (rc) return rc;
    }
    return AMX_OK;
}

}  // extern "C"

namespace {
amx::UpArgs up_args(const amx_plan *p, const int16_t *d_out, const int16_t *d_edge, void *d_ws) {
    amx::UpArgs a{};
    a.cd = p->d_cd;
    a.ks = p->d_ksegs;
    a.n_kseg = p->n_kseg;
    a.spans = p->d_spans;
    a.Lin = p->upLin;
    a.Lout = p->upLout;
    a.static_l = p->up_static;
    a.poly = p->up_poly;
    a.fcnt = p->d_fcnt;
    a.bankn = p->d_bankn;
    a.hop = p->hop;
    a.obase = p->d_obase;
    a.oph = p->d_oph;
    a.owt = p->d_owt;
    a.lin = p->up_lin;
    a.slow = p->d_slow;
    a.n_slow = p->n_slow;
    a.bank = p->d_bank;
    a.taps = p->up_taps;
    a.alloc = p->up_alloc;
    a.x = reinterpret_cast<const uint32_t *>(d_out);
    a.edge = reinterpret_cast<const uint32_t *>(d_edge);
    a.G = p->d_Gkw;
    a.qh = p->d_qh;
    a.qt = p->d_qt;
    a.eterms = wsp<double>(d_ws, p->o_eterms);
    a.e = wsp<double>(d_ws, p->o_ekw);
    a.s = wsp<double>(d_ws, p->o_skw);
    a.parts = wsp<double>(d_ws, p->o_parts);
    a.part_hop = wsp<int64_t>(d_ws, p->o_phop);
    a.pk = wsp<uint32_t>(d_ws, p->o_pk);
    return a;
}
// ---- loudnorm's 192 kHz modes: scratch layout (amx_loudnorm.hip)
#define LN_FIRST_FRAMES 576000     // frame_size(192000, 3000)
struct LnLayout {
    int T = 0, nb_last = 0, Fs = 4, Wf = 3, J = 0, M = 0, K = 0, P = 0;
    int64_t o_u = 0, o_ring = 0, o_ctl = 0, o_dctl = 0, o_v = 0, o_hold = 0, o_D = 0, o_G = 0, o_ramp = 0;
    int64_t o_recG = 0, o_recE = 0, o_wrec = 0, o_cnt = 0, o_match = 0, o_rings = 0, o_wring = 0, o_bm = 0;
    int64_t o_bmF = 0;
    int64_t total = 0;
};
// INNER frames, segments of Fs frames each warmed up Wf frames (AMX_LN_WARM, default 2)
// before its start, at most P persistent k_lp_seg workgroups of AMX_LP_NT lanes (AMX_LN_P;
// default 3072 waves: three per SIMD, k_lp_seg's register budget).  Fs (AMX_LN_SEG overrides) is the smallest >= 2 whose segments fit the P waves: a
// wave then runs one segment, Fs + Wf frames (r04m: a 5-min track 11.9 -> 9.1 ms per
// dynamic step from Fs 4 / Wf 3 / 1024 waves); a longer track takes longer segments, so
// the warm-up share Wf / Fs shrinks instead of waves running several segments each.
LnLayout ln_layout(int64_t n192, int64_t u_frames = -1, int p_cap = -1) {
    LnLayout l;
    l.Wf = 2;
    int pmax = 3072 / (AMX_LP_NT / 64);
    if (const char *ev = std::getenv("AMX_LN_P")) pmax = std::max(64, std::atoi(ev));
    if (n192 >= LN_FIRST_FRAMES) {
        l.T = (int)((n192 - LN_FIRST_FRAMES + 19199) / 19200);
        l.nb_last = l.T > 0 ? (int)(n192 - LN_FIRST_FRAMES - 19200LL * (l.T - 1)) : 0;
    }
    l.Fs = std::max(2, (l.T + (pmax - 32) - 1) / (pmax - 32));
    if (const char *ev = std::getenv("AMX_LN_SEG")) l.Fs = std::max(1, std::atoi(ev));
    if (const char *ev = std::getenv("AMX_LN_WARM")) l.Wf = std::max(0, std::atoi(ev));
    // boundaries only at full INNER frames (a partial last frame's wrap reads reach the
    // frame before it), at FINAL's start and inside FINAL
    const int t_ok = (l.T > 0 && l.nb_last == 19200) ? l.T : l.T - 1;
    l.J = t_ok >= 1 + l.Fs ? (t_ok - 1) / l.Fs : 0;
    l.M = (29 + l.Fs - 1) / l.Fs;
    l.K = 1 + l.J + l.M;
    l.P = std::min(l.K, pmax);
    if (p_cap > 0) l.P = std::min(l.P, p_cap);     // a window's segments need no more waves
    int64_t o = 0;
    auto take = [&](int64_t bytes) { const int64_t at = o; o += ((bytes + 255) / 256) * 256; return at; };
    l.o_u = take((u_frames < 0 ? n192 : u_frames) * 2 * (int64_t)sizeof(float));
    l.o_ring = take((2 * 40320 + 64) * (int64_t)sizeof(double));
    l.o_ctl = take(16 * sizeof(int));
    l.o_dctl = take(8 * sizeof(double));
    l.o_v = take((int64_t)l.T * sizeof(double));
    l.o_hold = take((int64_t)l.T * sizeof(int));
    l.o_D = take((int64_t)l.T * sizeof(double));
    l.o_G = take((int64_t)(l.T + 1) * sizeof(double));
    l.o_ramp = take(19200 * sizeof(double));
    l.o_recG = take((int64_t)l.K * AMX_LN_REC * sizeof(double));
    l.o_recE = take((int64_t)l.K * AMX_LN_REC * sizeof(double));
    l.o_wrec = take(2 * AMX_LN_REC * sizeof(double));
    l.o_cnt = take((int64_t)(l.K + 1) * sizeof(int));
    l.o_match = take((int64_t)(l.K + 1) * sizeof(int));
    l.o_rings = take((int64_t)l.P * AMX_LN_RING * 2 * sizeof(double));
    l.o_wring = take((int64_t)AMX_LN_RING * 2 * sizeof(double));
    l.o_bm = take((n192 / 64 + 2) * (int64_t)sizeof(double));
    l.o_bmF = take((n192 / 64 + 2) * (int64_t)sizeof(double));
    l.total = o;
    return l;
}
// the 192 kHz stream's frames of a whole track (the resampler's output, or the track
// itself when it already is 192 kHz)
int ln_frames(const amx_plan *p, int32_t track, int64_t *n192) {
    if (p->meas_native || (p->resamp && !p->up_ok))
        return fail(AMX_ERANGE, "loudnorm's 192 kHz modes need a 192 kHz upsampler (input above 192 kHz)");
    const SpanDev &sp = p->spans[track];
    *n192 = p->resamp ? (sp.out_n * p->upL + p->upM - 1) / p->upM : sp.out_n;
    return AMX_OK;
}
// the first output position of segment k: its frame (k_lp_*'s lp_seg_start) and that
// frame's base (lp_frame: INNER frames from 0, FINAL's from S0)
int64_t ln_seg_base(const LnLayout &lo, int64_t n192, int k) {
    const int phi = k == 0 ? 0 : (k <= lo.J ? 1 + k * lo.Fs : lo.T + 1 + (k - lo.J - 1) * lo.Fs);
    const int64_t S0 = n192 - (LN_FIRST_FRAMES - 19200);
    return phi <= lo.T ? (int64_t)19200 * phi : S0 + (int64_t)19200 * (phi - lo.T - 1);
}
int check_edges(const amx_plan *p, const int16_t *d_edge) {
    if (!p->resamp || d_edge) return AMX_OK;
    for (const SpanDev &sp : p->spans)
        if (sp.out_n > 0 && (sp.edge_lo || sp.edge_hi))
            return fail(AMX_EINVAL, "a span inside its track needs the neighbour frames (d_edge)");
    return AMX_OK;
}
}  // namespace

extern "C" {

int amx_loudness_pass1_part(amx_plan *p, int32_t part, const int16_t *d_out, const int16_t *d_edge,
                            double *d_kw_tail, double *d_peak, void *d_ws, void *stream) {
    if (!p || !d_peak || (p->n_kseg > 0 && (!d_out || !d_ws)))
        return fail(AMX_EINVAL, "null argument");
    if (part != 0 && part != 1) return fail(AMX_EINVAL, "bad part %d", part);
    if (p->resamp && !p->up_ok)
        return fail(AMX_ERANGE, "%d Hz has no 192 kHz upsampler (loudnorm pass 1)",
                    p->cd.fs);
    if (int rc = check_edges(p, d_edge)) return rc;
    hipStream_t st = (hipStream_t)stream;
    double *e = wsp<double>(d_ws, p->o_ekw), *s = wsp<double>(d_ws, p->o_skw);
    uint32_t *pk = wsp<uint32_t>(d_ws, p->o_pk);
    if (part == 0) {
        // the pass over the samples: per K segment the zero-state end state (and, at
        // 192 kHz, the peaks and energy terms; amx_loud192.hip)
        p->kw_rest_states = 0;
        p->kw_eb_ready = 0;
        if (p->n_kseg == 0) return AMX_OK;
        if (p->resamp)
            HIPCHK(amx::launch_up1(up_args(p, d_out, d_edge, d_ws), st, p->up_aux, p->up_fork, p->up_join));
        else if (!p->fuse_kw)  // else the GEMV + per-segment peaks were made by k_front2 (amx_run_chunks)
            HIPCHK(amx::launch_kw1(p->d_cd, p->d_ksegs, p->n_kseg, p->Lkw, d_out, p->d_Gkw, e, pk, p->gate, st));
        return AMX_OK;
    }
    // k_peak_reduce writes every track's peak; only tracks without a K segment (empty
    // spans) need the zero written here
    if (p->any_empty_span || p->n_kseg == 0)
        HIPCHK(amx::launch_zero(d_peak, sizeof(double) * 4 * (size_t)p->n_tracks, st));
    if (p->n_kseg == 0) {
        if (d_kw_tail) HIPCHK(amx::launch_zero(d_kw_tail, sizeof(double) * 8 * (size_t)p->n_tracks, st));
        return AMX_OK;
    }
    HIPCHK(amx::launch_peak_reduce(p->d_spans, p->n_tracks, p->max_nkseg, pk, d_peak, p->d_pcnt,
                                   p->d_ppart, p->d_ksegs, p->Lkw, d_out, p->d_Gkw, e, p->fuse_kw,
                                   p->resamp, st));
    // the span tails from the scan's own down sweep unless a span is empty (its tail is 0:
    // k_kw_tail writes it)
    const bool tail_fused = d_kw_tail && !p->any_empty_span;
    HIPCHK(amx::launch_scan(p->scan_kw(), e, s, nullptr, wsp<double>(d_ws, p->o_ebk), st, true,
                            tail_fused ? p->d_tailpow : nullptr, tail_fused ? d_kw_tail : nullptr));
    p->kw_rest_states = 1;   // s = the start states from rest: pass 2 without a carry reuses them
    p->kw_eb_ready = 1;      // and the block sums: pass 2 with a carry runs the down sweep only
    if (d_kw_tail && !tail_fused)
        HIPCHK(amx::launch_kw_tail(p->d_spans, p->n_tracks, s, e, p->d_tailpow, d_kw_tail, st));
    return AMX_OK;
}

int amx_loudness_pass1(amx_plan *p, const int16_t *d_out, const int16_t *d_edge, double *d_kw_tail,
                       double *d_peak, void *d_ws, void *stream) {
    int rc = amx_loudness_pass1_part(p, 0, d_out, d_edge, d_kw_tail, d_peak, d_ws, stream);
    if (rc) return rc;
    return amx_loudness_pass1_part(p, 1, d_out, d_edge, d_kw_tail, d_peak, d_ws, stream);
}

int amx_loudnorm_192k_size(const amx_plan *p, int32_t track, int64_t *frames, int64_t *ws_bytes) {
    if (!p || !frames || !ws_bytes || track < 0 || track >= p->n_tracks) return fail(AMX_EINVAL, "bad argument");
    int64_t n192 = 0;
    if (int rc = ln_frames(p, track, &n192)) return rc;
    *frames = n192;
    *ws_bytes = ln_layout(n192).total;
    return AMX_OK;
}

}  // extern "C"

namespace {
// the kernels' arguments of one filter run of track `track` (amx_loudnorm_192k_ex / _shard)
int ln_args(amx_plan *p, int32_t track, const amx_loudnorm_desc *d, const double *d_measured,
            const double *d_offset_i, const int32_t *d_gate, const int16_t *d_out, const double *d_hops,
            int64_t max_hops, const double *d_peak, int16_t *d_y192, double *d_summary, void *d_ws2,
            amx::LnArgs &a, amx::LpArgs &q, int64_t &n192, int64_t u_lo = 0, int64_t u_frames = -1,
            int64_t y_lo = 0, int p_cap = -1) {
    if (!p || track < 0 || track >= p->n_tracks) return fail(AMX_EINVAL, "bad argument");
    n192 = 0;
    if (int rc = ln_frames(p, track, &n192)) return rc;
    if (!d || !d_out || !d_hops || !d_peak || !d_y192 || !d_summary || !d_ws2)
        return fail(AMX_EINVAL, "null argument");
    const SpanDev &sp = p->spans[track];
    if (sp.tframe0 != 0 || sp.ttotal != sp.out_n)
        return fail(AMX_EINVAL, "loudnorm's 192 kHz modes run on whole tracks (one plan holds the track)");
    if (max_hops < n192 / 19200 + 1) return fail(AMX_EINVAL, "d_hops holds %lld hops", (long long)max_hops);
    const LnLayout lo = ln_layout(n192, u_frames, p_cap);
    char *w = reinterpret_cast<char *>(d_ws2);
    a = amx::LnArgs{};
    a.n192 = n192;
    // a window (amx_ln_shard.windowed): u holds positions [u_lo, ..) and d_y192 starts at
    // position y_lo; the kernels index whole-track positions, so the bases move back
    // (only positions inside the windows are ever touched)
    a.u = reinterpret_cast<float *>(reinterpret_cast<uintptr_t>(w + lo.o_u) - (uintptr_t)u_lo * 2 * sizeof(float));
    a.ring = reinterpret_cast<double *>(w + lo.o_ring);
    a.y = reinterpret_cast<int16_t *>(reinterpret_cast<uintptr_t>(d_y192) - (uintptr_t)y_lo * 2 * sizeof(int16_t));
    a.summary = d_summary;
    a.hops = d_hops + (int64_t)track * max_hops * 2;
    a.peak = d_peak + (int64_t)track * 4;
    a.energies = p->d_energies;
    a.bounds = p->d_bounds;
    // af_loudnorm init / config_input: dB options to the linear factors it keeps
    a.target_i = d->target_i;
    a.target_lra = d->target_lra;
    a.target_tp = std::pow(10., d->target_tp / 20.);
    a.measured_i = d->measured_i;
    a.measured_thresh = d->measured_thresh;
    a.offset = std::pow(10., d->offset / 20.);
    {   // init_gaussian_filter
        double total = 0.0;
        const double sigma = 3.5;
        const int off = 21 / 2;
        const double c1 = 1.0 / (sigma * std::sqrt(2.0 * M_PI));
        const double c2 = 2.0 * std::pow(sigma, 2.0);
        for (int i = 0; i < 21; i++) {
            const int x = i - off;
            a.weights[i] = c1 * std::exp(-(std::pow(x, 2.0) / c2));
            total += a.weights[i];
        }
        const double adjust = 1.0 / total;
        for (int i = 0; i < 21; i++) a.weights[i] *= adjust;
    }
    for (int k = 0; k < 5; k++) { a.kb[k] = p->kdf_b[k]; a.ka[k] = p->kdf_a[k]; }
    q = amx::LpArgs{};
    q.n = n192;
    q.S0 = n192 - (LN_FIRST_FRAMES - 19200);
    q.T = lo.T;
    q.nb_last = lo.nb_last;
    q.Fs = lo.Fs;
    q.Wf = lo.Wf;
    q.J = lo.J;
    q.M = lo.M;
    q.K = lo.K;
    q.P = lo.P;
    q.u = a.u;
    q.hops = a.hops;
    q.energies = a.energies;
    q.bounds = a.bounds;
    q.target_i = a.target_i;
    q.target_lra = a.target_lra;
    q.ceiling = a.target_tp;
    q.measured_i = a.measured_i;
    q.measured_thresh = a.measured_thresh;
    q.offset = a.offset;
    q.measured_src = d_measured;
    q.offset_src = d_offset_i;
    q.gate = d_gate;
    for (int i = 0; i < 21; i++) q.weights[i] = a.weights[i];
    q.v = reinterpret_cast<double *>(w + lo.o_v);
    q.hold = reinterpret_cast<int *>(w + lo.o_hold);
    q.D = reinterpret_cast<double *>(w + lo.o_D);
    q.G = reinterpret_cast<double *>(w + lo.o_G);
    q.ramp = reinterpret_cast<double *>(w + lo.o_ramp);
    q.recG = reinterpret_cast<double *>(w + lo.o_recG);
    q.recE = reinterpret_cast<double *>(w + lo.o_recE);
    q.wrec = reinterpret_cast<double *>(w + lo.o_wrec);
    q.cnt = reinterpret_cast<int *>(w + lo.o_cnt);
    q.match = reinterpret_cast<int *>(w + lo.o_match);
    q.rings = reinterpret_cast<double *>(w + lo.o_rings);
    q.wring = reinterpret_cast<double *>(w + lo.o_wring);
    q.ctl = reinterpret_cast<int *>(w + lo.o_ctl);
    q.dctl = reinterpret_cast<double *>(w + lo.o_dctl);
    q.y = a.y;
    q.summary = d_summary;
    a.lp_ctl = q.ctl;
    a.lp_dctl = q.dctl;
    a.lp_D = q.D;
    a.lp_recG = q.recG;
    a.lp_Fs = q.Fs;
    a.lp_J = q.J;
    a.lp_tstop = INT_MAX;
    q.kb = 0;
    q.ke = q.K;
    // k_lp_fill + the skipping scan + the sparse emit (AMX_LP_FILL=0: the dense form, for
    // A/B measurements)
    const char *fe = std::getenv("AMX_LP_FILL");
    q.bm = (fe && std::atoi(fe) == 0) ? nullptr : reinterpret_cast<double *>(w + lo.o_bm);
    // FINAL's bound (AMX_LP_FINAL_SKIP=0: FINAL's frames scan every group, for A/B)
    const char *fs = std::getenv("AMX_LP_FINAL_SKIP");
    q.bmF = (q.bm && !(fs && std::atoi(fs) == 0)) ? reinterpret_cast<double *>(w + lo.o_bmF) : nullptr;
    return AMX_OK;
}
}  // namespace

extern "C" {

int amx_loudnorm_192k_ex(amx_plan *p, int32_t track, const amx_loudnorm_desc *d, const double *d_measured,
                         const double *d_offset_i, const int32_t *d_gate, const int16_t *d_out, const double *d_hops,
                         int64_t max_hops, const double *d_peak, int16_t *d_y192, double *d_summary,
                         void *d_ws2, void *stream) {
    amx::LnArgs a;
    amx::LpArgs q;
    int64_t n192 = 0;
    if (int rc = ln_args(p, track, d, d_measured, d_offset_i, d_gate, d_out, d_hops, max_hops, d_peak, d_y192,
                         d_summary, d_ws2, a, q, n192))
        return rc;
    const SpanDev &sp = p->spans[track];
    amx::SwrDev r{p->up_pc, p->up_lin, p->up_src, p->up_dst, p->d_bank, p->up_taps, p->up_alloc};
    HIPCHK(amx::launch_loudnorm(a, q, reinterpret_cast<const uint32_t *>(d_out) + sp.out_off, sp.out_n, r,
                                d->reuse_stream == 0, (hipStream_t)stream));
    return AMX_OK;
}

int amx_loudnorm_192k_shard(amx_plan *p, int32_t track, const amx_loudnorm_desc *d, const double *d_measured,
                            const double *d_offset_i, const amx_ln_shard *sh, const int16_t *d_out,
                            const double *d_hops, int64_t max_hops, const double *d_peak, int16_t *d_y192,
                            double *d_summary, void *d_ws2, void *stream) {
    if (!sh || sh->part < 0 || sh->part > 3) return fail(AMX_EINVAL, "bad shard");
    if (sh->part == 3 && sh->kb != 0) return fail(AMX_EINVAL, "part 3 (a quiet start) runs on the first segments' rank");
    amx::LnArgs a;
    amx::LpArgs q;
    int64_t n192 = 0;
    if (!p || track < 0 || track >= p->n_tracks) return fail(AMX_EINVAL, "bad argument");
    if (int rc = ln_frames(p, track, &n192)) return rc;
    int64_t win[9] = {0, 0, sh->u_lo, sh->u_hi, 0, 0, 0, 0, 0};
    if (sh->windowed || sh->u_lo < 0) {
        int64_t wsb = 0;
        if (int rc = amx_loudnorm_192k_shard_window(p, track, sh->kb, sh->ke, win, &wsb)) return rc;
    }
    const int64_t u_lo = win[2], u_hi = win[3];
    if (int rc = ln_args(p, track, d, d_measured, d_offset_i, nullptr, d_out, d_hops, max_hops, d_peak, d_y192,
                         d_summary, d_ws2, a, q, n192, sh->windowed ? u_lo : 0, sh->windowed ? u_hi - u_lo : -1,
                         sh->windowed ? win[4] : 0, sh->windowed ? sh->ke - sh->kb : -1))
        return rc;
    if (sh->kb < 0 || sh->ke > q.K || sh->kb > sh->ke) return fail(AMX_EINVAL, "segments [%d, %d) of %d", sh->kb, sh->ke, q.K);
    if (u_hi > n192 || u_lo > u_hi) return fail(AMX_EINVAL, "bad 192 kHz range");
    if (sh->part == 2 && sh->kb > 0 && !sh->d_rec_in) return fail(AMX_EINVAL, "segment %d needs the true state", sh->kb);
    q.kb = sh->kb;
    q.ke = sh->ke;
    // part 3: a hand-over at segment k needs the INNER frames < k Fs; the last segment this
    // rank may hand over at is ke - 1 (a later lift: the replicated form)
    if (sh->part == 3) a.lp_tstop = sh->ke - 1 > 0 ? (sh->ke - 1) * q.Fs : 0;
    q.rec_in = sh->kb > 0 ? sh->d_rec_in : nullptr;
    q.rec_out = sh->ke < q.K ? sh->d_rec_out : nullptr;
    const SpanDev &sp = p->spans[track];
    amx::SwrDev r{p->up_pc, p->up_lin, p->up_src, p->up_dst, p->d_bank, p->up_taps, p->up_alloc};
    // the positions segments [kb, ke) emit
    const LnLayout lo = ln_layout(n192);
    const int64_t y_lo = ln_seg_base(lo, n192, sh->kb), y_hi = sh->ke < lo.K ? ln_seg_base(lo, n192, sh->ke) : n192;
    // windowed: d_out holds track frames [x_lo, x_hi) (the base moves back to frame 0)
    const uint32_t *x = sh->windowed
                            ? reinterpret_cast<const uint32_t *>(reinterpret_cast<uintptr_t>(d_out) -
                                                                 (uintptr_t)win[0] * sizeof(uint32_t))
                            : reinterpret_cast<const uint32_t *>(d_out) + sp.out_off;
    HIPCHK(amx::launch_loudnorm_shard(a, q, x, sp.out_n, r, u_lo, u_hi, y_lo, y_hi, sh->part, d->reuse_stream == 0,
                                      (hipStream_t)stream));
    return AMX_OK;
}

int amx_loudnorm_192k_shard_window(const amx_plan *p, int32_t track, int32_t kb, int32_t ke, int64_t *win,
                                   int64_t *ws_bytes) {
    if (!p || track < 0 || track >= p->n_tracks || !win || !ws_bytes) return fail(AMX_EINVAL, "bad argument");
    int64_t n192 = 0;
    if (int rc = ln_frames(p, track, &n192)) return rc;
    const LnLayout lo = ln_layout(n192);
    if (kb < 0 || ke > lo.K || kb >= ke) return fail(AMX_EINVAL, "segments [%d, %d) of %d", kb, ke, lo.K);
    // what segments [kb, ke) read: from Wf + 2 frames before the first one's start (its
    // warm-up) to a ring and two frames past the last one's end
    const int64_t u_lo = std::max<int64_t>(0, ln_seg_base(lo, n192, kb) - (int64_t)19200 * (lo.Wf + 2));
    const int64_t u_hi = ke < lo.K ? std::min<int64_t>(n192, ln_seg_base(lo, n192, ke) + AMX_LN_RING + 2 * 19200) : n192;
    // the chain frames the resampler reads for them: output j's window starts at frame
    // floor(j M / L) - 15 (32 taps), with a margin; 192 kHz input: the positions themselves
    const SpanDev &sp = p->spans[track];
    int64_t x_lo = u_lo, x_hi = u_hi;
    if (p->resamp) {
        const int64_t m = p->up_alloc + 8;       // the window's reach (center + the row)
        x_lo = std::max<int64_t>(0, (int64_t)((__int128)u_lo * p->upM / p->upL) - m);
        x_hi = std::min<int64_t>(sp.out_n, (int64_t)(((__int128)u_hi * p->upM + p->upL - 1) / p->upL) + m);
    }
    win[0] = x_lo;
    win[1] = x_hi;
    win[2] = u_lo;
    win[3] = u_hi;
    win[4] = ln_seg_base(lo, n192, kb);
    win[5] = ke < lo.K ? ln_seg_base(lo, n192, ke) : n192;
    const LnLayout lw = ln_layout(n192, u_hi - u_lo, ke - kb);
    win[6] = lw.o_ctl;
    win[7] = lw.o_D;       // (ABI 4) the INNER frames' deltas, T doubles (a quiet start's hand-over)
    win[8] = lw.T;
    *ws_bytes = lw.total;
    return AMX_OK;
}

int amx_loudnorm_192k_segments(const amx_plan *p, int32_t track, int64_t *starts, int32_t cap, int32_t *K,
                               int32_t *k_fin, int32_t *rec_doubles, int64_t *ctl_offset) {
    if (!p || track < 0 || track >= p->n_tracks || !K) return fail(AMX_EINVAL, "bad argument");
    int64_t n192 = 0;
    if (int rc = ln_frames(p, track, &n192)) return rc;
    const LnLayout lo = ln_layout(n192);
    *K = lo.K;
    if (k_fin) *k_fin = lo.J + 1;
    if (rec_doubles) *rec_doubles = AMX_LN_REC;
    if (ctl_offset) *ctl_offset = lo.o_ctl;
    if (starts) {
        if (cap < lo.K + 1) return fail(AMX_EINVAL, "starts holds %d, needs %d", cap, lo.K + 1);
        for (int k = 0; k < lo.K; k++) starts[k] = ln_seg_base(lo, n192, k);
        starts[lo.K] = n192;
    }
    return AMX_OK;
}

int amx_loudnorm_192k(amx_plan *p, int32_t track, const amx_loudnorm_desc *d, const int16_t *d_out,
                      const double *d_hops, int64_t max_hops, const double *d_peak, int16_t *d_y192,
                      double *d_summary, void *d_ws2, void *stream) {
    return amx_loudnorm_192k_ex(p, track, d, nullptr, nullptr, nullptr, d_out, d_hops, max_hops, d_peak, d_y192,
                                d_summary, d_ws2, stream);
}

int amx_pcm_to_s16(const void *d_raw, int64_t frames, int32_t channels, int32_t format,
                   int16_t *d_out, void *stream) {
    if (frames < 0 || (frames > 0 && (!d_raw || !d_out))) return fail(AMX_EINVAL, "null argument");
    if (channels < 1 || channels > 8) return fail(AMX_EINVAL, "channels must be 1..8");
    if (format < AMX_PCM_U8 || format > AMX_PCM_F64BE) return fail(AMX_EINVAL, "bad PCM format %d", format);
    HIPCHK(amx::launch_pcm_to_s16(d_raw, frames, channels, format, d_out, (hipStream_t)stream));
    return AMX_OK;
}

int amx_plan_set_gate(amx_plan *p, const int32_t *d_gate) {
    if (!p) return fail(AMX_EINVAL, "null plan");
    p->gate = d_gate;
    return AMX_OK;
}

int amx_plan_set_limiter_trace(amx_plan *p, double *d_att) {
    if (!p) return fail(AMX_EINVAL, "null plan");
    p->lim_att = d_att;
    return AMX_OK;
}

int amx_plan_set_publish(amx_plan *p, int32_t *h_ctl) {
    if (!p) return fail(AMX_EINVAL, "null plan");
    p->publish = h_ctl;
    return AMX_OK;
}

int amx_env_counters(const amx_plan *p, const void *d_ws, int32_t *out, int32_t n) {
    if (!p || !out || n < 0) return fail(AMX_EINVAL, "null argument");
    const int32_t have = AMX_ENV_MAX_ROUNDS * AMX_ENV_NCTR;
    for (int32_t i = 0; i < n; i++) out[i] = 0;
    if (!p->mb || p->n_es == 0) return AMX_OK;
    if (!d_ws) return fail(AMX_EINVAL, "null workspace");
    const int32_t k = n < have ? n : have;
    HIPCHK(hipMemcpy(out, reinterpret_cast<const char *>(d_ws) + p->o_eflags + AMX_ENV_MAX_ROUNDS * 4,
                     (size_t)k * 4, hipMemcpyDeviceToHost));
    return AMX_OK;
}

int amx_kw_propagate(const amx_plan *p, int64_t frames, const double *in8, double *out8) {
    if (!p || !in8 || !out8 || frames < 0) return fail(AMX_EINVAL, "bad argument");
    Mat P = p->kw_model.pow(frames);
    for (int c = 0; c < 2; c++)
        for (int i = 0; i < AMX_KW_DIM; i++) {
            double acc = 0.0;
            for (int k = 0; k < AMX_KW_DIM; k++) acc += P[(size_t)i * AMX_KW_DIM + k] * in8[c * 4 + k];
            out8[c * 4 + i] = acc;
        }
    return AMX_OK;
}

int amx_loudness_pass2(amx_plan *p, const int16_t *d_out, const int16_t *d_edge,
                       const double *d_kw_carry, double *d_hops, int64_t max_hops, void *d_ws,
                       void *stream) {
    if (!p || !d_hops || max_hops <= 0 || (p->n_kseg > 0 && (!d_out || !d_ws)))
        return fail(AMX_EINVAL, "null argument");
    if (p->resamp && !p->up_ok)
        return fail(AMX_ERANGE, "%d Hz has no 192 kHz upsampler (loudnorm pass 1)",
                    p->cd.fs);
    if (max_hops < p->max_hops) return fail(AMX_EINVAL, "max_hops %lld < %lld", (long long)max_hops,
                                            (long long)p->max_hops);
    if (int rc = check_edges(p, d_edge)) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (p->n_kseg == 0) {
        HIPCHK(amx::launch_zero(d_hops, sizeof(double) * 2 * (size_t)max_hops * p->n_tracks, st));
        return AMX_OK;
    }
    double *e = wsp<double>(d_ws, p->o_ekw), *s = wsp<double>(d_ws, p->o_skw);
    double *parts = wsp<double>(d_ws, p->o_parts);
    int64_t *phop = wsp<int64_t>(d_ws, p->o_phop);
    if (d_kw_carry || !p->kw_rest_states) {
        // the block sums do not depend on the carry: after pass 1 only the down sweep runs
        HIPCHK(amx::launch_scan(p->scan_kw(), e, s, d_kw_carry, wsp<double>(d_ws, p->o_ebk), st, !p->kw_eb_ready));
        p->kw_eb_ready = 1;
        p->kw_rest_states = d_kw_carry ? 0 : 1;
    }
    if (p->resamp)
        HIPCHK(amx::launch_up2(up_args(p, d_out, d_edge, d_ws), st));
    else
        HIPCHK(amx::launch_kw2(p->d_cd, p->d_ksegs, p->n_kseg, p->Lkw, p->hop, d_out, s, parts, phop,
                               p->kw_aligned, p->gate, st));
    HIPCHK(amx::launch_hops(p->d_spans, p->n_tracks, p->d_ksegs, p->resamp ? p->upLout : p->Lkw,
                            p->hop, parts, phop, d_hops, max_hops, st));
    return AMX_OK;
}

int amx_loudness_histograms(amx_plan *p, const double *d_hops, int64_t max_hops, uint64_t *d_hist,
                            uint64_t *d_st_hist, void *d_ws, void *stream) {
    (void)d_ws;
    if (!p || !d_hops || !d_hist || !d_st_hist || max_hops <= 0)
        return fail(AMX_EINVAL, "null argument");
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(amx::launch_hist(p->d_spans, p->n_tracks, p->hop, d_hops, max_hops, p->d_bounds,
                            reinterpret_cast<unsigned long long *>(d_hist),
                            reinterpret_cast<unsigned long long *>(d_st_hist), st));
    return AMX_OK;
}

int amx_limiter_geometry(const amx_plan *p, const amx_final_desc *fd, int32_t *buffer_size,
                         int32_t *halo_frames, int64_t *state_doubles) {
    if (!p || !fd) return fail(AMX_EINVAL, "null argument");
    const int channels = 2;
    double attack = fd->attack_ms / 1000.0;
    int bs = (int)(p->cd.fs * attack * channels);   // af_alimiter config_input
    bs -= bs % channels;
    if (bs <= 0) return fail(AMX_EINVAL, "Attack is too small.");
    if (buffer_size) *buffer_size = bs;
    if (halo_frames) *halo_frames = bs / channels - 1;
    if (state_doubles) *state_doubles = 8 + 3 * (int64_t)bs;
    return AMX_OK;
}

int amx_limiter_prepare(amx_plan *p, const amx_final_desc *fd, int32_t seg_frames,
                        int32_t warm_frames) {
    if (!p || !fd) return fail(AMX_EINVAL, "null argument");
    int32_t bs = 0, halo = 0;
    int64_t sd = 0;
    int rc = amx_limiter_geometry(p, fd, &bs, &halo, &sd);
    if (rc) return rc;
    if (seg_frames <= 0) seg_frames = p->lim.seg_frames > 0 ? p->lim.seg_frames : AMX_LIM_SEG_DEFAULT;
    if (seg_frames < 64 || seg_frames < bs / 2)
        return fail(AMX_EINVAL, "limiter segments of %d frames: need >= 64 and >= the ring (%d frames)",
                    seg_frames, bs / 2);
    if (amx::limiter_lds_bytes(bs) > AMX_LIM_LDS_MAX)
        return fail(AMX_ERANGE, "Attack is too large: the alimiter's %d-sample look-ahead ring does not fit "
                    "a CU's LDS (inputs above ~670 kHz)", bs);
    if (amx::limiter_lds_bytes(bs) > 64 * 1024) HIPCHK(amx::limiter_allow_lds(amx::limiter_lds_bytes(bs)));
    const int64_t max_segs64 = p->max_span > 0 ? (p->max_span + seg_frames - 1) / seg_frames : 1;
    if (max_segs64 > INT32_MAX / 2) return fail(AMX_EINVAL, "limiter: too many segments");
    const int max_segs = (int)max_segs64;
    if (warm_frames < 0) {
        // three releases plus the ring: a limiter that rested anywhere in the
        // warm-up has forgotten everything before it
        const double rel = p->cd.fs * (fd->release_ms / 1000.0);
        warm_frames = (int)std::min(1e9, std::ceil(3.0 * rel)) + bs / 2;
    }
    p->lim.warm_frames = warm_frames;
    // warm-ups reach back over active stretches up to 10 s (longer ones are left to
    // the in-order repair); warm_frames 0 disables the search (tests)
    p->lim.warm_cap = warm_frames > 0 ? (int64_t)p->cd.fs * 10 : 0;
    if (p->lim.seg_state && p->lim.buffer_size == bs && p->lim.seg_frames == seg_frames &&
        p->lim.max_segs == max_segs)
        return AMX_OK;
    const int T = p->n_tracks > 0 ? p->n_tracks : 1;
    // the new scratch is allocated before the old is released, so a failed
    // allocation leaves the plan's previous (consistent) limiter scratch in place
    double *seg_state = nullptr;
    unsigned *cnt = nullptr;
    if (hipMalloc(&seg_state, (size_t)T * max_segs * 2 * sd * sizeof(double)) != hipSuccess ||
        hipMalloc(&cnt, (size_t)T * sizeof(unsigned)) != hipSuccess ||
        hipMemset(cnt, 0, (size_t)T * sizeof(unsigned)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        if (seg_state) (void)hipFree(seg_state);
        if (cnt) (void)hipFree(cnt);
        return fail(AMX_EHIP, "limiter scratch allocation failed");
    }
    if (p->lim.seg_state) (void)hipFree(p->lim.seg_state);
    if (p->lim.cnt) (void)hipFree(p->lim.cnt);
    const int64_t cap = p->lim.warm_cap;
    p->lim = amx::LimScratch{};
    p->lim.warm_frames = warm_frames;
    p->lim.warm_cap = cap;
    p->lim.seg_state = seg_state;
    p->lim.cnt = cnt;
    p->lim.seg_frames = seg_frames;
    p->lim.max_segs = max_segs;
    p->lim.buffer_size = bs;
    return AMX_OK;
}

int amx_publish_ctl(const int32_t *d_ctl, int32_t *h_ctl, int32_t n, void *stream) {
    if (n < 0 || (n > 0 && (!d_ctl || !h_ctl))) return fail(AMX_EINVAL, "null argument");
    HIPCHK(amx::launch_publish(d_ctl, h_ctl, n, (hipStream_t)stream));
    return AMX_OK;
}

int amx_loudness_decide(amx_plan *p, const amx_decide_desc *dd, const amx_final_desc *fd,
                        const uint64_t *d_hist, const uint64_t *d_st_hist, const double *d_peak,
                        double *d_stats, double *d_gains, int32_t *d_ctl, void *stream) {
    if (!p || !dd || !fd || !d_peak || !d_stats || !d_gains || !d_ctl ||
        (dd->lufs_on && (!d_hist || !d_st_hist)))
        return fail(AMX_EINVAL, "null argument");
    if (dd->lufs_on && p->meas_native)
        return fail(AMX_ERANGE, "%d Hz: loudnorm measures the track resampled to 192 kHz with an "
                    "interpolating downsampler (not restated); lufs=None works", p->cd.fs);
    amx::DecideArgs a{};
    a.n_tracks = p->n_tracks;
    a.lufs_on = dd->lufs_on ? 1 : 0;
    a.hist = reinterpret_cast<const unsigned long long *>(d_hist);
    a.st_hist = reinterpret_cast<const unsigned long long *>(d_st_hist);
    a.peak = d_peak;
    a.energies = p->d_energies;
    a.bounds = p->d_bounds;
    a.target_i = dd->target_i;
    a.target_tp = dd->target_tp;
    a.target_lra = dd->target_lra;
    a.level_in = fd->level_in;
    a.limit = fd->limit;
    a.stats = d_stats;
    a.gains = d_gains;
    a.ctl = d_ctl;
    a.host_ctl = p->publish;
    HIPCHK(amx::launch_decide(a, (hipStream_t)stream));
    return AMX_OK;
}

int amx_kw_carry_setup(amx_plan *p, int32_t n_prev, const int64_t *frames_after) {
    if (!p || n_prev < 0 || (n_prev > 0 && !frames_after)) return fail(AMX_EINVAL, "bad argument");
    std::vector<double> P((size_t)(n_prev > 0 ? n_prev : 1) * 16, 0.0);
    for (int q = 0; q < n_prev; q++) {
        if (frames_after[q] < 0) return fail(AMX_EINVAL, "frames_after[%d] < 0", q);
        // the gap on the measurement stream: J(f0) - J(f0 - frames_after), J(f) = ceil(f L / M)
        int64_t gap = frames_after[q];
        if (p->resamp && p->n_tracks > 0) {
            const int64_t f0 = p->spans[0].tframe0, L = p->upL, M = p->upM;
            auto J = [&](int64_t f) { return (f * L + M - 1) / M; };
            gap = J(f0) - J(f0 - frames_after[q]);
        }
        Mat m = p->kw_model.pow(gap);
        for (int k = 0; k < 16; k++) P[(size_t)q * 16 + k] = m[k];
    }
    if (p->d_carryP) (void)hipFree(p->d_carryP);
    p->d_carryP = nullptr;
    int rc = upload(&p->d_carryP, P.data(), P.size());
    if (rc) return rc;
    p->n_prev = n_prev;
    return AMX_OK;
}

int amx_kw_carry(amx_plan *p, const double *d_tails, double *d_carry, void *stream) {
    if (!p || !d_carry || (p->n_prev > 0 && !d_tails)) return fail(AMX_EINVAL, "null argument");
    if (!p->d_carryP) return fail(AMX_EINVAL, "amx_kw_carry: call amx_kw_carry_setup first");
    HIPCHK(amx::launch_kw_carry(d_tails, p->d_carryP, p->n_prev, d_carry, (hipStream_t)stream));
    return AMX_OK;
}

int amx_kw_carry_rows(amx_plan *p, const double *d_rows, int32_t world, int32_t ld, double *d_carry,
                      double *d_peak, void *stream) {
    if (!p || !d_rows || !d_carry || !d_peak) return fail(AMX_EINVAL, "null argument");
    if (!p->d_carryP) return fail(AMX_EINVAL, "amx_kw_carry_rows: call amx_kw_carry_setup first");
    if (world < 1 || ld < 12 || p->n_prev >= world)
        return fail(AMX_EINVAL, "amx_kw_carry_rows: %d rows of %d doubles for %d previous spans", world, ld,
                    p->n_prev);
    HIPCHK(amx::launch_kw_carry_rows(d_rows, world, ld, p->d_carryP, p->n_prev, d_carry, d_peak,
                                     (hipStream_t)stream));
    return AMX_OK;
}

int amx_finalize(amx_plan *p, const amx_final_desc *fd, const int16_t *d_x,
                 const double *d_gains, const int32_t *d_ctl, int32_t fast,
                 const int16_t *d_halo, int16_t *d_y, double *d_lim_state, void *d_ws,
                 void *stream) {
    (void)d_ws;
    if (!p || !fd || !d_gains || (p->out_frames > 0 && (!d_x || !d_y)))
        return fail(AMX_EINVAL, "null argument");
    if (p->out_frames == 0) return AMX_OK;
    int32_t bs = 0, halo = 0;
    int64_t sd = 0;
    int rc = amx_limiter_geometry(p, fd, &bs, &halo, &sd);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    const double level = fd->auto_level ? 1 / fd->limit : 1;
    if ((d_ctl || !fast) && !d_lim_state) return fail(AMX_EINVAL, "general limiter needs d_lim_state");
    if ((d_ctl || !fast) && (!p->lim.seg_state || p->lim.buffer_size != bs)) {
        // amx_limiter_prepare allocates: not while the stream is being captured into a
        // graph (callers that capture call it first)
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIPCHK(hipStreamIsCapturing(st, &cs));
        if (cs != hipStreamCaptureStatusNone)
            return fail(AMX_EINVAL, "amx_finalize: call amx_limiter_prepare before capturing the stream");
        rc = amx_limiter_prepare(p, fd, 0, -1);
        if (rc) return rc;
    }
    p->lim.gate = p->gate;
    p->lim.att = p->lim_att;
    HIPCHK(amx::launch_final(p->d_spans, p->n_tracks, p->max_span, d_x, d_halo, halo, d_gains, d_ctl,
                             fast ? 1 : 0, p->cd.fs, fd->level_in, level, fd->level_out, fd->limit,
                             fd->release_ms / 1000.0, bs, d_lim_state, sd, fd->from_rest, p->lim, d_y, st));
    return AMX_OK;
}

}  // extern "C"

// ==================================================================================
// More than two channels (round 6).  audio_segment_to_float_array only reshapes a
// stereo chunk (:252), so a 3..8-channel chunk goes through the chain as ONE
// interleaved 1-D stream: analog character (its shelves along the stream, :264-265),
// EQ (:274, float64 result), no width (:268), the crossover along the stream (:303);
// pydub's compressor and overlay then work on frames of C samples (:306-309).
//   pa (analog on): a stream chain (stream in L of int16 pairs) whose "EQ" is the
//      analog character's two shelves, the input through the float32 tanh table;
//   pb: the stream chain of the EQ (and the crossover bands when multiband);
//   pc (multiband): a stereo plan over the chunks' real frames whose envelope kernels
//      (k_env0 + fix-up) run on the C-sample r that k_mc_rms forms from pb's bands;
//      k_mc_gain_overlay writes the C-channel output.
struct amx_mc_plan {
    int C = 0, mb = 0, in_s16 = 0;
    amx_plan *pa = nullptr, *pb = nullptr, *pc = nullptr;
    int64_t M = 0;                 // stream samples the pack covers
    int64_t out_frames = 0;
    size_t o_pack = 0, o_outa = 0, o_outb = 0, o_wa = 0, o_wb = 0, o_wc = 0, ws_bytes = 0;
};

extern "C" {

void amx_mc_plan_free(amx_mc_plan *m) {
    if (!m) return;
    amx_plan_free(m->pa);
    amx_plan_free(m->pb);
    amx_plan_free(m->pc);
    delete m;
}

int amx_mc_plan_create(const amx_chain_desc *desc, const amx_chunk *chunks, int32_t n_chunks, int32_t seg_frames,
                       amx_mc_plan **out) {
    if (!desc || !out || n_chunks < 0 || (n_chunks > 0 && !chunks)) return fail(AMX_EINVAL, "null argument");
    *out = nullptr;
    const int C = desc->channels_in;
    if (C < 3 || C > 8) return fail(AMX_EINVAL, "amx_mc_plan_create: %d channels (3..8; 1 or 2: amx_plan_create)", C);
    if (desc->analog_on && !desc->tanh_lut)
        return fail(AMX_EINVAL, "analog character needs the float32 tanh table (tanh_lut)");
    amx_mc_plan *m = new (std::nothrow) amx_mc_plan();
    if (!m) return fail(AMX_ENOMEM, "out of memory");
    m->C = C;
    m->mb = desc->multiband_on ? 1 : 0;
    m->in_s16 = desc->input_s16 ? 1 : 0;
    std::vector<amx_chunk> sch((size_t)n_chunks), ach((size_t)n_chunks);
    int64_t in_end = 0, acc = 0, sum_n = 0;
    for (int32_t k = 0; k < n_chunks; k++) {
        if (chunks[k].frames < 0 || chunks[k].in_offset < 0) {
            delete m;
            return fail(AMX_EINVAL, "chunk %d: negative offset or length", k);
        }
        sch[k] = chunks[k];
        sch[k].in_offset = chunks[k].in_offset * C;
        sch[k].frames = chunks[k].frames * C;
        ach[k] = sch[k];
        ach[k].in_offset = acc;                       // pb reads pa's output, chunks back to back
        acc += sch[k].frames;
        in_end = std::max(in_end, chunks[k].in_offset + chunks[k].frames);
        sum_n += chunks[k].frames;
    }
    m->M = in_end * C;
    // the stream chains: int16 pairs, the stream in L
    amx_chain_desc ds = *desc;
    ds.channels_in = 2;
    ds.input_s16 = 1;
    ds.analog_on = 0;
    ds.tanh_lut = nullptr;
    ds.width_on = 0;
    ds.measure_only = 0;
    ds.stream_chain = 1;
    ds.eq_in_lut = nullptr;
    int rc = AMX_OK;
    if (desc->analog_on) {
        // x = tanh(float32 s / 32768 * drive) (the table), then low shelf 120 Hz with g =
        // 10^(cf/20) and high shelf 12 kHz with 10^(1.5 cf/20), both gains > 0: the EQ's
        // positive-gain shelf form x + (y - x)(g - 1) at stages 0 and 3 (:264-265, :288)
        amx_chain_desc da = ds;
        da.multiband_on = 0;
        for (int s = 0; s < 4; s++) { da.eq_kind[s] = 0; da.eq_gain_db[s] = 0.0; da.eq_gain[s] = 1.0; }
        da.eq_kind[0] = 1;
        da.eq_gain[0] = desc->analog_lo_gain;
        da.eq_gain_db[0] = 20.0 * std::log10(desc->analog_lo_gain);
        da.eq_kind[3] = 1;
        da.eq_gain[3] = desc->analog_hi_gain;
        da.eq_gain_db[3] = 20.0 * std::log10(desc->analog_hi_gain);
        for (int k = 0; k < 6; k++) {
            da.eq_coef[0][k] = desc->analog_lo_ba[k];
            da.eq_coef[3][k] = desc->analog_hi_ba[k];
        }
        if (!(da.eq_gain_db[0] > 0.0 && da.eq_gain_db[3] > 0.0)) {
            delete m;
            return fail(AMX_EINVAL, "analog character gains must be > 1");
        }
        da.eq_in_lut = desc->tanh_lut;
        rc = amx_plan_create(&da, sch.data(), n_chunks, nullptr, nullptr, seg_frames, &m->pa);
        if (rc) { amx_mc_plan_free(m); return rc; }
    }
    rc = amx_plan_create(&ds, desc->analog_on ? ach.data() : sch.data(), n_chunks, nullptr, nullptr, seg_frames,
                         &m->pb);
    if (rc) { amx_mc_plan_free(m); return rc; }
    if (m->mb) {
        amx_chain_desc dc = *desc;
        dc.channels_in = 2;
        dc.input_s16 = 1;
        dc.analog_on = 0;
        dc.tanh_lut = nullptr;
        dc.width_on = 0;
        dc.measure_only = 0;
        dc.stream_chain = 0;
        dc.eq_in_lut = nullptr;
        for (int s = 0; s < 4; s++) { dc.eq_kind[s] = 0; dc.eq_gain_db[s] = 0.0; dc.eq_gain[s] = 1.0; }
        rc = amx_plan_create(&dc, chunks, n_chunks, nullptr, nullptr, seg_frames, &m->pc);
        if (rc) { amx_mc_plan_free(m); return rc; }
        m->out_frames = m->pc->out_frames;
    } else {
        m->out_frames = sum_n;
    }
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t at = off; off += (bytes + 255) / 256 * 256; return at; };
    m->o_pack = take((size_t)std::max<int64_t>(m->M, 1) * 4);
    if (m->pa) m->o_outa = take((size_t)std::max<int64_t>(m->pa->out_frames, 1) * 4);
    if (!m->mb) m->o_outb = take((size_t)std::max<int64_t>(m->pb->out_frames, 1) * 4);
    if (m->pa) m->o_wa = take(m->pa->ws_bytes);
    m->o_wb = take(m->pb->ws_bytes);
    if (m->pc) m->o_wc = take(m->pc->ws_bytes);
    m->ws_bytes = off;
    *out = m;
    return AMX_OK;
}

int amx_mc_plan_get_info(const amx_mc_plan *m, int64_t *workspace_bytes, int64_t *out_frames) {
    if (!m || !workspace_bytes || !out_frames) return fail(AMX_EINVAL, "null argument");
    *workspace_bytes = (int64_t)m->ws_bytes;
    *out_frames = m->out_frames;
    return AMX_OK;
}

int amx_mc_run_chunks(amx_mc_plan *m, const void *d_in, int16_t *d_out, void *d_ws, void *stream) {
    if (!m || (m->M > 0 && (!d_in || !d_out || !d_ws))) return fail(AMX_EINVAL, "null argument");
    if (m->M == 0) return AMX_OK;
    hipStream_t st = (hipStream_t)stream;
    char *w = reinterpret_cast<char *>(d_ws);
    uint32_t *pack = reinterpret_cast<uint32_t *>(w + m->o_pack);
    HIPCHK(amx::launch_mc_pack(d_in, m->M, m->in_s16, pack, st));
    const float *src = reinterpret_cast<const float *>(pack);
    if (m->pa) {
        int16_t *outa = reinterpret_cast<int16_t *>(w + m->o_outa);
        int rc = amx_run_chunks(m->pa, src, outa, w + m->o_wa, stream);
        if (rc) return rc;
        src = reinterpret_cast<const float *>(outa);
    }
    amx_plan *pb = m->pb;
    void *wb = w + m->o_wb;
    if (!m->mb) {
        int16_t *outb = reinterpret_cast<int16_t *>(w + m->o_outb);
        int rc = amx_run_chunks(pb, src, outb, wb, stream);
        if (rc) return rc;
        HIPCHK(amx::launch_mc_unpack(reinterpret_cast<const uint32_t *>(outb), m->out_frames * m->C, d_out, st));
        return AMX_OK;
    }
    // the stream's EQ and crossover bands (pb), then the compressor on C-sample frames
    for (int s = AMX_STAGE_FRONT1; s <= AMX_STAGE_XOVER; s++) {
        int rc = amx_run_stage(pb, s, src, d_out, wb, stream);
        if (rc) return rc;
    }
    amx_plan *pc = m->pc;
    void *wc = w + m->o_wc;
    amx::DynLaunch dl{pc->d_cd,    pc->d_chunks, pc->n_chunks, pc->d_esegs, pc->n_es,
                      pc->d_eseg0, pc->d_neseg,  pc->nloc,     pc->max_chunk_n, pc->cd.look,
                      pc->warm,    pc->Le,       pc->cd.env_rcp, pc->d_tabs, st,
                      pc->env_wg,  pc->env_pin};
    const int16_t *bands = wsp<int16_t>(wb, pb->o_bands);
    uint16_t *mframe = wsp<uint16_t>(wc, pc->o_m);
    int *bact = wsp<int>(wc, pc->o_eflags) + AMX_ENV_BACT;
    HIPCHK(amx::launch_mc_rms(dl, pb->d_chunks, bands, pb->nloc, m->C, mframe, bact));
    for (int s : {AMX_STAGE_ENV, AMX_STAGE_FIX}) {
        int rc = amx_run_stage(pc, s, reinterpret_cast<const float *>(d_in), d_out, wc, stream);
        if (rc) return rc;
    }
    HIPCHK(amx::launch_mc_gain_overlay(dl, pb->d_chunks, mframe, wsp<double>(wc, pc->o_gain), bands, pb->nloc,
                                       m->C, pc->max_chunk_out, pc->d_n1, bact, d_out));
    return AMX_OK;
}

int amx_mc_split_pairs(const int16_t *d_y, int64_t frames, int32_t channels, int16_t *d_pairs, void *stream) {
    if (frames > 0 && (!d_y || !d_pairs)) return fail(AMX_EINVAL, "null argument");
    HIPCHK(amx::launch_mc_split_pairs(d_y, frames, channels, d_pairs, (hipStream_t)stream));
    return AMX_OK;
}

int amx_mc_loudness_combine(const double *d_hops, int64_t max_hops, const double *d_peak, int32_t channels,
                            double *d_hops1, double *d_peak1, void *stream) {
    if (!d_hops || !d_peak || !d_hops1 || !d_peak1 || max_hops <= 0) return fail(AMX_EINVAL, "null argument");
    HIPCHK(amx::launch_mc_loudness_combine(d_hops, max_hops, d_peak, channels, d_hops1, d_peak1,
                                           (hipStream_t)stream));
    return AMX_OK;
}

int amx_mc_peak_pick(const int16_t *d_y, int64_t frames, int32_t channels, const double *d_gain, int16_t *d_syn,
                     void *stream) {
    if (frames > 0 && (!d_y || !d_gain || !d_syn)) return fail(AMX_EINVAL, "null argument");
    if (channels < 1 || channels > 8) return fail(AMX_EINVAL, "%d channels", channels);
    HIPCHK(amx::launch_mc_peak_pick(d_y, frames, channels, d_gain, d_syn, (hipStream_t)stream));
    return AMX_OK;
}

int amx_mc_limiter_out(const amx_plan *p, const amx_final_desc *fd, const int16_t *d_y, int32_t channels,
                       const double *d_gains, const int32_t *d_ctl, const double *d_att, int16_t *d_out,
                       void *stream) {
    if (!p || !fd || !d_gains || !d_ctl || (p->out_frames > 0 && (!d_y || !d_att || !d_out)))
        return fail(AMX_EINVAL, "null argument");
    if (channels < 1 || channels > 8) return fail(AMX_EINVAL, "%d channels", channels);
    if (p->n_tracks != 1 || p->spans[0].tframe0 != 0) return fail(AMX_EINVAL, "one whole track per plan");
    int32_t bs = 0, halo = 0;
    int64_t sd = 0;
    if (int rc = amx_limiter_geometry(p, fd, &bs, &halo, &sd)) return rc;
    const double level = fd->auto_level ? 1 / fd->limit : 1;
    HIPCHK(amx::launch_mc_limiter_out(d_y, p->out_frames, channels, halo, d_gains, d_ctl, d_att, fd->level_in,
                                      level, fd->level_out, fd->limit, d_out, (hipStream_t)stream));
    return AMX_OK;
}

}  // extern "C"
