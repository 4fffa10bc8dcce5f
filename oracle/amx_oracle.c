/*
 * amx_oracle.c -- CPU restatement of the reference's mastering hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle: it may be linked,
 * loaded or executed only by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, as the checker.  The product path (libamx.so + amx/) never
 * calls it.
 *
 * Pinning: the per-chunk stages (analog, EQ, width, int16 conversions, crossover,
 * compressor, overlay) are checked bit-for-bit against golden vectors produced by
 * running the reference's own audio_mastering_engine.py (tests/golden/, generator
 * tests/golden/make_golden.py).  The ffmpeg stages (loudnorm measurement/linear
 * gain, alimiter) have NO reference code or fixtures in /root/reference and no
 * ffmpeg binary exists here: their restatement below follows the published
 * libebur128 / FFmpeg af_loudnorm.c / af_alimiter.c algorithms and is
 * "parity unpinned" beyond the EBU Tech 3341/3342 known answers in the tests.
 *
 * Floating-point operation ORDER follows the reference exactly (scipy's
 * _linear_filter / _sosfilt inner loops, numpy dtype promotion, CPython audioop).
 * Build with -ffp-contract=off so no FMA contraction changes rounding.
 * All citations are audio_mastering_engine.py:<line> unless noted.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

#define EXPORT __attribute__((visibility("default")))

/* ---------------------------------------------------------------- filters */

/* scipy.signal.lfilter DF-II-transposed inner loop for a 2nd-order ba filter,
 * zero initial state, a[0] == 1 (butter output).  Order of operations is
 * scipy's _linear_filter:  y = Z0 + b0*x;  Z0 = Z1 + x*b1 - y*a1;  Z1 = x*b2 - y*a2.
 * Used by apply_shelf_filter (:286). */
typedef struct { double z0, z1; } lf_state;

static inline double lf_step(const double *b, const double *a, lf_state *s, double x) {
    double y = s->z0 + b[0] * x;
    s->z0 = (s->z1 + x * b[1]) - y * a[1];
    s->z1 = x * b[2] - y * a[2];
    return y;
}

/* scipy.signal.sosfilt (_sosfilt) inner loop, one section:
 *   x_new = b0*x + zi0;  zi0 = b1*x - a1*x_new + zi1;  zi1 = b2*x - a2*x_new.
 * sos rows are [b0 b1 b2 a0 a1 a2] with a0 == 1.  Used at :296 and :303. */
static inline double sos_step(const double *sec, double *zi, double x) {
    double xn = sec[0] * x + zi[0];
    zi[0] = (sec[1] * x - sec[4] * xn) + zi[1];
    zi[1] = sec[2] * x - sec[5] * xn;
    return xn;
}

/* float_array_to_audio_segment (:254-257) for float32 arrays:
 * np.clip(x,-1,1) * 32767 in float32, .astype(int16) truncates toward zero. */
static inline int16_t f32_to_s16(float x) {
    float v = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
    v = v * 32767.0f;
    return (int16_t)v;
}
/* same for float64 arrays (analog character :266, crossover bands :305) */
static inline int16_t f64_to_s16(double x) {
    double v = x < -1.0 ? -1.0 : (x > 1.0 ? 1.0 : x);
    v = v * 32767.0;
    return (int16_t)v;
}

/* ------------------------------------------------------- analog character */
/* apply_analog_character (:258-266).  x = s16/32768 (f32, :253); tanh(x*drive)
 * in float32 -- taken from `tanh_lut` (65536 float32 values indexed by s16+32768,
 * built from numpy's own float32 tanh by the caller); then two shelf filters
 * whose lfilter runs along axis -1, i.e. ACROSS THE TWO CHANNELS of each frame
 * (:264-265): a length-2 sequence per frame, zero state per frame.
 * Both shelves have gain_db > 0, so :288 applies:  x + (y - x)*(g - 1). */
EXPORT void orc_analog(const int16_t *in, int64_t n, const float *tanh_lut,
                       const double *b_lo, const double *a_lo, double g_lo,
                       const double *b_hi, const double *a_hi, double g_hi,
                       int16_t *out) {
    const double glo1 = g_lo - 1.0, ghi1 = g_hi - 1.0;
    for (int64_t i = 0; i < n; i++) {
        double x0 = (double)tanh_lut[(int)in[2 * i] + 32768];
        double x1 = (double)tanh_lut[(int)in[2 * i + 1] + 32768];
        lf_state s = {0.0, 0.0};
        double y0 = lf_step(b_lo, a_lo, &s, x0);
        double y1 = lf_step(b_lo, a_lo, &s, x1);
        double u0 = x0 + (y0 - x0) * glo1;
        double u1 = x1 + (y1 - x1) * glo1;
        lf_state t = {0.0, 0.0};
        double v0 = lf_step(b_hi, a_hi, &t, u0);
        double v1 = lf_step(b_hi, a_hi, &t, u1);
        double w0 = u0 + (v0 - u0) * ghi1;
        double w1 = u1 + (v1 - u1) * ghi1;
        out[2 * i] = f64_to_s16(w0);
        out[2 * i + 1] = f64_to_s16(w1);
    }
}

/* ------------------------------------------------------------------- EQ */
/* _apply_eq_to_channel (:277-282): four stages in order, each skipped when its
 * gain is 0 (:284, :291).  kind: 0 = skipped, 1 = shelf (ba, lfilter, :283-289),
 * 2 = peak (4 SOS band-pass, sosfilt, :290-298).
 * coef layout per stage: kind 1 -> b[3], a[3];  kind 2 -> sos[4][6].
 * Numpy dtype promotion: the channel enters as float32; the first ACTIVE stage
 * sees a float32 input, later stages float64.  That matters only for the
 * negative-gain shelf, where `samples * gain` (:289) is a float32 product when
 * `samples` is float32 (NEP 50: the Python float is cast to float32).
 * The final float64 result is stored back into the float32 column (:274). */
typedef struct {
    int kind[4];
    double gain_db[4];
    double g[4];          /* 10**(gain_db/20) as computed by Python */
    double coef[4][24];
} orc_eq_t;

EXPORT void orc_eq_channel(const float *in, int64_t n, int stride, const orc_eq_t *eq,
                           float *out) {
    lf_state ls[4];
    double zs[4][4][2];
    memset(ls, 0, sizeof(ls));
    memset(zs, 0, sizeof(zs));
    for (int64_t i = 0; i < n; i++) {
        float xf = in[i * stride];
        double x = (double)xf;
        int first = 1;
        for (int st = 0; st < 4; st++) {
            int k = eq->kind[st];
            if (k == 0) continue;
            const double *c = eq->coef[st];
            if (k == 1) {
                double y = lf_step(c, c + 3, &ls[st], x);
                double g = eq->g[st];
                if (eq->gain_db[st] > 0) {
                    x = x + (y - x) * (g - 1.0);
                } else {
                    double xg = first ? (double)(xf * (float)g) : x * g;
                    x = xg + (y - xg);
                }
            } else {
                double y = x;
                for (int s = 0; s < 4; s++) y = sos_step(c + 6 * s, zs[st][s], y);
                x = x + y * (eq->g[st] - 1.0);
            }
            first = 0;
        }
        out[i * stride] = first ? xf : (float)x;
    }
}

/* apply_stereo_width (:267-271), float32 M/S with clip. */
EXPORT void orc_width(float *lr, int64_t n, float w) {
    for (int64_t i = 0; i < n; i++) {
        float l = lr[2 * i], r = lr[2 * i + 1];
        float mid = (l + r) / 2.0f, side = (l - r) / 2.0f;
        side = side * w;
        float nl = mid + side, nr = mid - side;
        lr[2 * i] = nl < -1.0f ? -1.0f : (nl > 1.0f ? 1.0f : nl);
        lr[2 * i + 1] = nr < -1.0f ? -1.0f : (nr > 1.0f ? 1.0f : nr);
    }
}

EXPORT void orc_f32_to_s16(const float *x, int64_t n, int16_t *out) {
    for (int64_t i = 0; i < n; i++) out[i] = f32_to_s16(x[i]);
}

/* ------------------------------------------------------------ crossover */
/* apply_multiband_compressor (:300-305): x = s16/32768 (float32, :253);
 * low = sosfilt(butter(4,250,'lowpass',sos), x, axis=0); high likewise at 4 kHz
 * 'highpass' (2 SOS each, float64); mid = x - low - high; each band -> int16. */
EXPORT void orc_crossover(const int16_t *p16, int64_t n, const double *lo_sos,
                          const double *hi_sos, int16_t *lo, int16_t *mid, int16_t *hi) {
    for (int c = 0; c < 2; c++) {
        double zl[2][2] = {{0, 0}, {0, 0}}, zh[2][2] = {{0, 0}, {0, 0}};
        for (int64_t i = 0; i < n; i++) {
            float xf = (float)p16[2 * i + c] / 32768.0f;
            double x = (double)xf;
            double l = x, h = x;
            for (int s = 0; s < 2; s++) l = sos_step(lo_sos + 6 * s, zl[s], l);
            for (int s = 0; s < 2; s++) h = sos_step(hi_sos + 6 * s, zh[s], h);
            double m = (x - l) - h;
            lo[2 * i + c] = f64_to_s16(l);
            mid[2 * i + c] = f64_to_s16(m);
            hi[2 * i + c] = f64_to_s16(h);
        }
    }
}

/* ----------------------------------------------------------- compressor */
/* CPython audioop.mul's clamp (Modules/audioop.c fbound): > max -> max,
 * < min+1 -> min, then floor. */
static inline int16_t audioop_mul16(int v, double factor) {
    double val = (double)v * factor;
    if (val > 32767.0) val = 32767.0;
    else if (val < -32768.0 + 1.0) val = -32768.0;
    return (int16_t)(int)floor(val);
}

/* pydub.effects.compress_dynamic_range (pydub 0.25.1, called at :306-308),
 * restated:  thresh_rms = 32768 * 10**(T/20); look_frames = int(5*(fs/1000.0));
 * per frame i: rms of frames [max(i-L,0), i) via audioop.rms (double sum of
 * squares -- exact integer here -- / sample count, sqrt, truncating (unsigned)),
 * over = max(20*log(rms/thr,10), 0) (0 if rms==0; math.log(x,10) = log(x)/log(10)),
 * max_att = (1 - 1/ratio)*over; inc = max_att/(5*fs/1000.0), dec = max_att/(50*fs/1000.0);
 * attack if rms > thr and att <= max_att (capped at max_att) else release (floored at 0);
 * if att != 0 the frame is audioop.mul'ed by 10**(-att/20).
 * If att_trace != NULL the per-frame attenuation is written there. */
EXPORT void orc_compress(const int16_t *in, int64_t n, int fs, double threshold, double ratio,
                         int16_t *out, double *att_trace) {
    const double thr = 32768.0 * pow(10.0, threshold / 20.0);
    const int64_t L = (int64_t)(5.0 * (fs / 1000.0));
    const double A = 5.0 * (fs / 1000.0), R = 50.0 * (fs / 1000.0);
    const double k = 1.0 - (1.0 / ratio);
    const double ln10 = log(10.0);
    int64_t S = 0;   /* exact sum of squares of the window */
    double att = 0.0;
    for (int64_t i = 0; i < n; i++) {
        if (i > 0) {
            int64_t a = in[2 * (i - 1)], b = in[2 * (i - 1) + 1];
            S += a * a + b * b;
        }
        if (i - L - 1 >= 0) {
            int64_t a = in[2 * (i - L - 1)], b = in[2 * (i - L - 1) + 1];
            S -= a * a + b * b;
        }
        int64_t lo = i - L < 0 ? 0 : i - L;
        int64_t cnt = 2 * (i - lo);
        unsigned int rms = cnt ? (unsigned int)sqrt((double)S / (double)cnt) : 0u;
        double over = 0.0;
        if (rms != 0) {
            double db = 20 * (log((double)rms / thr) / ln10);
            over = db > 0 ? db : (db == 0 ? db : 0.0);
        }
        double m = k * over;
        double inc = m / A, dec = m / R;
        if ((double)rms > thr && att <= m) {
            att += inc;
            att = att < m ? att : m;
        } else {
            att -= dec;
            att = att > 0 ? att : 0.0;
        }
        if (att_trace) att_trace[i] = att;
        if (att != 0.0) {
            double f = pow(10.0, (-att) / 20.0);
            out[2 * i] = audioop_mul16(in[2 * i], f);
            out[2 * i + 1] = audioop_mul16(in[2 * i + 1], f);
        } else {
            out[2 * i] = in[2 * i];
            out[2 * i + 1] = in[2 * i + 1];
        }
    }
}

/* --------------------------------------------------------------- overlay */
/* pydub AudioSegment.__len__ / __getitem__ ms rounding used by overlay (:309):
 * int(round(1000*(n/fs)) * (fs/1000.0)) frames (round = half-to-even). */
EXPORT int64_t orc_overlay_len(int64_t n, int fs) {
    double ms = nearbyint(1000.0 * ((double)n / (double)fs));
    return (int64_t)(ms * (fs / 1000.0));
}

static inline int16_t sat16(int v) { return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }

/* low.overlay(mid).overlay(high) (:309): audioop.add (saturating) over the common
 * length; seg1 is first ms-rounded (zero-padded or truncated).  Returns out frames. */
EXPORT int64_t orc_overlay3(const int16_t *lo, const int16_t *mid, const int16_t *hi,
                            int64_t n, int fs, int16_t *out) {
    int64_t n1 = orc_overlay_len(n, fs);
    int64_t n2 = orc_overlay_len(n1, fs);
    int64_t nn = n1 < n ? n1 : n;
    for (int64_t i = 0; i < 2 * nn; i++) out[i] = sat16((int)lo[i] + (int)mid[i]);
    for (int64_t i = 2 * nn; i < 2 * n1; i++) out[i] = 0;
    /* second overlay on the n1-frame intermediate (ms-rounded again to n2) */
    for (int64_t i = 2 * n1; i < 2 * n2; i++) out[i] = 0;
    int64_t m = n2 < n ? n2 : n;
    for (int64_t i = 0; i < 2 * m; i++) out[i] = sat16((int)out[i] + (int)hi[i]);
    return n2;
}

/* ------------------------------------------------------- chunk composition */
typedef struct {
    int fs;
    int analog_on;
    double an_b_lo[3], an_a_lo[3], an_g_lo, an_b_hi[3], an_a_hi[3], an_g_hi;
    const float *tanh_lut;
    orc_eq_t eq;
    int width_on;
    float width;
    int mb_on;
    double xlo[12], xhi[12];
    double thr_db[3], ratio[3];
} orc_chunk_t;

/* the chunk body, audio_mastering_engine.py:189-197, on an s16 stereo chunk.
 * `out` must hold max(n, overlay_len(n)) + 8 frames.  Returns output frames. */
EXPORT int64_t orc_chunk(const orc_chunk_t *p, const int16_t *in16, int64_t n, int16_t *out) {
    int16_t *a16 = (int16_t *)malloc(sizeof(int16_t) * 2 * (n + 1));
    float *f = (float *)malloc(sizeof(float) * 2 * (n + 1));
    const int16_t *src = in16;
    if (p->analog_on) {
        orc_analog(in16, n, p->tanh_lut, p->an_b_lo, p->an_a_lo, p->an_g_lo,
                   p->an_b_hi, p->an_a_hi, p->an_g_hi, a16);
        src = a16;
    }
    for (int64_t i = 0; i < 2 * n; i++) f[i] = (float)src[i] / 32768.0f;
    orc_eq_channel(f, n, 2, &p->eq, f);
    orc_eq_channel(f + 1, n, 2, &p->eq, f + 1);
    if (p->width_on) orc_width(f, n, p->width);
    int64_t nout = n;
    if (!p->mb_on) {
        orc_f32_to_s16(f, 2 * n, out);
    } else {
        int16_t *p16 = a16;
        orc_f32_to_s16(f, 2 * n, p16);
        int16_t *b = (int16_t *)malloc(sizeof(int16_t) * 12 * (n + 1));
        int16_t *lo = b, *mi = b + 2 * (n + 1), *hi = b + 4 * (n + 1);
        int16_t *loc = b + 6 * (n + 1), *mic = b + 8 * (n + 1), *hic = b + 10 * (n + 1);
        orc_crossover(p16, n, p->xlo, p->xhi, lo, mi, hi);
        orc_compress(lo, n, p->fs, p->thr_db[0], p->ratio[0], loc, NULL);
        orc_compress(mi, n, p->fs, p->thr_db[1], p->ratio[1], mic, NULL);
        orc_compress(hi, n, p->fs, p->thr_db[2], p->ratio[2], hic, NULL);
        nout = orc_overlay3(loc, mic, hic, n, p->fs, out);
        free(b);
    }
    free(a16);
    free(f);
    return nout;
}

/* ------------------------------------------- more than two channels (round 6) */
/* A chunk with C > 2 channels (the file's own layout after the ffmpeg split; :190
 * duplicates only mono).  audio_segment_to_float_array reshapes only when channels == 2
 * (:252), so every array stage runs on ONE interleaved 1-D stream of n*C samples:
 *  - analog character (:258-266): tanh, then both shelves' lfilter along the stream
 *    (axis -1 of a 1-D array), f64 -> int16;
 *  - EQ (:272-276): _apply_eq_to_channel on the whole stream; its result is NOT stored
 *    back into a float32 column (the 1-D branch rebinds `samples`), so it stays float64
 *    when a stage ran -- float_array_to_audio_segment then clips and scales in float64;
 *    with every stage skipped it is the float32 input;
 *  - width (:268) returns a 1-D array unchanged;
 *  - the crossover (:303) sosfilt's axis 0 of the 1-D stream;
 *  - pydub's compressor and overlay work on frames of C samples. */
EXPORT void orc_analog_stream(const int16_t *in, int64_t m, const float *tanh_lut,
                              const double *b_lo, const double *a_lo, double g_lo,
                              const double *b_hi, const double *a_hi, double g_hi,
                              int16_t *out) {
    const double glo1 = g_lo - 1.0, ghi1 = g_hi - 1.0;
    lf_state s = {0.0, 0.0}, t = {0.0, 0.0};
    for (int64_t i = 0; i < m; i++) {
        const double x = (double)tanh_lut[(int)in[i] + 32768];
        const double y = lf_step(b_lo, a_lo, &s, x);
        const double u = x + (y - x) * glo1;
        const double v = lf_step(b_hi, a_hi, &t, u);
        out[i] = f64_to_s16(u + (v - u) * ghi1);
    }
}

/* the EQ over the stream; returns 1 if a stage ran (out = its float64 result), else 0
 * (out = the float32 input, widened) */
EXPORT int orc_eq_stream(const float *in, int64_t m, const orc_eq_t *eq, double *out) {
    lf_state ls[4];
    double zs[4][4][2];
    memset(ls, 0, sizeof(ls));
    memset(zs, 0, sizeof(zs));
    int any = 0;
    for (int st = 0; st < 4; st++) any |= eq->kind[st] != 0;
    for (int64_t i = 0; i < m; i++) {
        const float xf = in[i];
        double x = (double)xf;
        int first = 1;
        for (int st = 0; st < 4; st++) {
            const int k = eq->kind[st];
            if (k == 0) continue;
            const double *c = eq->coef[st];
            if (k == 1) {
                const double y = lf_step(c, c + 3, &ls[st], x);
                const double g = eq->g[st];
                if (eq->gain_db[st] > 0) {
                    x = x + (y - x) * (g - 1.0);
                } else {
                    const double xg = first ? (double)(xf * (float)g) : x * g;
                    x = xg + (y - xg);
                }
            } else {
                double y = x;
                for (int q = 0; q < 4; q++) y = sos_step(c + 6 * q, zs[st][q], y);
                x = x + y * (eq->g[st] - 1.0);
            }
            first = 0;
        }
        out[i] = x;
    }
    return any;
}

/* pydub compress_dynamic_range on frames of C samples: audioop.rms over the window's
 * C (i - lo) samples, the gain on all C samples of the frame (orc_compress is C = 2) */
EXPORT void orc_compress_mc(const int16_t *in, int64_t n, int C, int fs, double threshold,
                            double ratio, int16_t *out, double *att_trace) {
    const double thr = 32768.0 * pow(10.0, threshold / 20.0);
    const int64_t L = (int64_t)(5.0 * (fs / 1000.0));
    const double A = 5.0 * (fs / 1000.0), R = 50.0 * (fs / 1000.0);
    const double k = 1.0 - (1.0 / ratio);
    const double ln10 = log(10.0);
    int64_t S = 0;
    double att = 0.0;
    for (int64_t i = 0; i < n; i++) {
        if (i > 0)
            for (int c = 0; c < C; c++) { const int64_t a = in[C * (i - 1) + c]; S += a * a; }
        if (i - L - 1 >= 0)
            for (int c = 0; c < C; c++) { const int64_t a = in[C * (i - L - 1) + c]; S -= a * a; }
        const int64_t lo = i - L < 0 ? 0 : i - L;
        const int64_t cnt = (int64_t)C * (i - lo);
        const unsigned int rms = cnt ? (unsigned int)sqrt((double)S / (double)cnt) : 0u;
        double over = 0.0;
        if (rms != 0) {
            const double db = 20 * (log((double)rms / thr) / ln10);
            over = db > 0 ? db : (db == 0 ? db : 0.0);
        }
        const double m = k * over;
        const double inc = m / A, dec = m / R;
        if ((double)rms > thr && att <= m) {
            att += inc;
            att = att < m ? att : m;
        } else {
            att -= dec;
            att = att > 0 ? att : 0.0;
        }
        if (att_trace) att_trace[i] = att;
        if (att != 0.0) {
            const double f = pow(10.0, (-att) / 20.0);
            for (int c = 0; c < C; c++) out[C * i + c] = audioop_mul16(in[C * i + c], f);
        } else {
            for (int c = 0; c < C; c++) out[C * i + c] = in[C * i + c];
        }
    }
}

/* orc_overlay3 on frames of C samples */
EXPORT int64_t orc_overlay3_mc(const int16_t *lo, const int16_t *mid, const int16_t *hi,
                               int64_t n, int C, int fs, int16_t *out) {
    const int64_t n1 = orc_overlay_len(n, fs);
    const int64_t n2 = orc_overlay_len(n1, fs);
    const int64_t nn = n1 < n ? n1 : n;
    for (int64_t i = 0; i < C * nn; i++) out[i] = sat16((int)lo[i] + (int)mid[i]);
    for (int64_t i = C * nn; i < C * n1; i++) out[i] = 0;
    for (int64_t i = C * n1; i < C * n2; i++) out[i] = 0;
    const int64_t mm = n2 < n ? n2 : n;
    for (int64_t i = 0; i < C * mm; i++) out[i] = sat16((int)out[i] + (int)hi[i]);
    return n2;
}

/* the chunk body (:189-197) on an s16 chunk of C > 2 channels [n][C]; `out` holds
 * C (max(n, overlay_len(n)) + 8) samples.  Returns output frames.  p->width_on is
 * ignored (:268). */
EXPORT int64_t orc_chunk_mc(const orc_chunk_t *p, const int16_t *in16, int64_t n, int C, int16_t *out) {
    const int64_t m = n * (int64_t)C;
    int16_t *a16 = (int16_t *)malloc(sizeof(int16_t) * (m + 1));
    float *f = (float *)malloc(sizeof(float) * (m + 1));
    double *y = (double *)malloc(sizeof(double) * (m + 1));
    const int16_t *src = in16;
    if (p->analog_on) {
        orc_analog_stream(in16, m, p->tanh_lut, p->an_b_lo, p->an_a_lo, p->an_g_lo,
                          p->an_b_hi, p->an_a_hi, p->an_g_hi, a16);
        src = a16;
    }
    for (int64_t i = 0; i < m; i++) f[i] = (float)src[i] / 32768.0f;
    const int any = orc_eq_stream(f, m, &p->eq, y);
    int16_t *p16 = p->mb_on ? a16 : out;
    for (int64_t i = 0; i < m; i++) p16[i] = any ? f64_to_s16(y[i]) : f32_to_s16(f[i]);
    int64_t nout = n;
    if (p->mb_on) {
        int16_t *b = (int16_t *)malloc(sizeof(int16_t) * 6 * (m + 1));
        int16_t *lo = b, *mi = b + (m + 1), *hi = b + 2 * (m + 1);
        int16_t *loc = b + 3 * (m + 1), *mic = b + 4 * (m + 1), *hic = b + 5 * (m + 1);
        double zl[2][2] = {{0, 0}, {0, 0}}, zh[2][2] = {{0, 0}, {0, 0}};
        for (int64_t i = 0; i < m; i++) {
            const float xf = (float)p16[i] / 32768.0f;
            const double x = (double)xf;
            double l = x, h = x;
            for (int q = 0; q < 2; q++) l = sos_step(p->xlo + 6 * q, zl[q], l);
            for (int q = 0; q < 2; q++) h = sos_step(p->xhi + 6 * q, zh[q], h);
            const double md = (x - l) - h;
            lo[i] = f64_to_s16(l);
            mi[i] = f64_to_s16(md);
            hi[i] = f64_to_s16(h);
        }
        orc_compress_mc(lo, n, C, p->fs, p->thr_db[0], p->ratio[0], loc, NULL);
        orc_compress_mc(mi, n, C, p->fs, p->thr_db[1], p->ratio[1], mic, NULL);
        orc_compress_mc(hi, n, C, p->fs, p->thr_db[2], p->ratio[2], hic, NULL);
        nout = orc_overlay3_mc(loc, mic, hic, n, C, p->fs, out);
        free(b);
    }
    free(a16);
    free(f);
    free(y);
    return nout;
}

/* ========================================================================
 * ffmpeg stages -- restated from the published FFmpeg sources (not in the
 * container).  PARITY UNPINNED: no ffmpeg binary and no reference fixtures.
 * ======================================================================== */

/* ---------------------------------------------------- libebur128 (ffmpeg) */
static double hist_energies[1000], hist_bounds[1001];
static int hist_init_done = 0;
EXPORT void orc_ebur128_tables(double *energies, double *bounds) {
    if (!hist_init_done) {
        hist_bounds[0] = pow(10.0, (-70.0 + 0.691) / 10.0);
        for (int i = 0; i < 1000; ++i)
            hist_energies[i] = pow(10.0, ((double)i / 10.0 - 69.95 + 0.691) / 10.0);
        for (int i = 1; i < 1001; ++i)
            hist_bounds[i] = pow(10.0, ((double)i / 10.0 - 70.0 + 0.691) / 10.0);
        hist_init_done = 1;
    }
    if (energies) memcpy(energies, hist_energies, sizeof(hist_energies));
    if (bounds) memcpy(bounds, hist_bounds, sizeof(hist_bounds));
}

static size_t find_hist_index(double energy) {
    size_t lo = 0, hi = 1000, mid;
    do {
        mid = (lo + hi) / 2;
        if (energy >= hist_bounds[mid]) lo = mid; else hi = mid;
    } while (hi - lo != 1);
    return lo;
}

/* K-weighting coefficients (libebur128 ebur128_init_filter): b[5], a[5]. */
EXPORT void orc_kweight_coefs(int fs, double *b, double *a) {
    double f0 = 1681.974450955533, G = 3.999843853973347, Q = 0.7071752369554196;
    double K = tan(M_PI * f0 / (double)fs);
    double Vh = pow(10.0, G / 20.0);
    double Vb = pow(Vh, 0.4996667741545416);
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
    K = tan(M_PI * f0 / (double)fs);
    ra[1] = 2.0 * (K * K - 1.0) / (1.0 + K / Q + K * K);
    ra[2] = (1.0 - K / Q + K * K) / (1.0 + K / Q + K * K);
    b[0] = pb[0] * rb[0];
    b[1] = pb[0] * rb[1] + pb[1] * rb[0];
    b[2] = pb[0] * rb[2] + pb[1] * rb[1] + pb[2] * rb[0];
    b[3] = pb[1] * rb[2] + pb[2] * rb[1];
    b[4] = pb[2] * rb[2];
    a[0] = pa[0] * ra[0];
    a[1] = pa[0] * ra[1] + pa[1] * ra[0];
    a[2] = pa[0] * ra[2] + pa[1] * ra[1] + pa[2] * ra[0];
    a[3] = pa[1] * ra[2] + pa[2] * ra[1];
    a[4] = pa[2] * ra[2];
}

/* Streaming libebur128 state (MODE_I | MODE_LRA | MODE_SAMPLE_PEAK), FFmpeg's
 * libavfilter/ebur128.c: ff_ebur128_add_frames_double() -> ebur128_filter (sample
 * peak, 4th-order DF-II K filter, DBL_MIN flush at the end of every filter call),
 * ebur128_calc_gating_block (400 ms blocks every 100 ms, 3 s short-term blocks
 * every 1 s) into the 1000-bin histograms. */
typedef struct {
    int channels;
    double b[5], a[5];
    size_t h100, ring_frames, idx, needed, st_counter;
    double *ring;
    double v[8][5];
    uint64_t *hist, *st_hist;
    double peak[8];
    double w[8];          /* channel weights of libebur128's default channel map */
    int64_t nb;
} Ebur;

/* libebur128 ebur128_init_channel_map (FFmpeg's copy; af_loudnorm sets no map of its
 * own): 4 channels L R Ls Rs, 5 channels L R C Ls Rs, otherwise L R C unused Ls Rs and
 * every later channel unused.  A block's energy skips unused channels and weights the
 * surrounds (Mp110 / Mm110) by 1.41 (ebur128_calc_gating_block).  Stereo: 1, 1. */
EXPORT void orc_ebur128_weights(int channels, double *w) {
    for (int c = 0; c < channels && c < 8; c++) {
        double v;
        if (channels == 4) v = c < 2 ? 1.0 : 1.41;
        else if (channels == 5) v = c < 3 ? 1.0 : 1.41;
        else v = c < 3 ? 1.0 : (c == 3 ? 0.0 : (c < 6 ? 1.41 : 0.0));
        w[c] = v;
    }
}

static void ebur_init(Ebur *e, int fs, int channels, uint64_t *hist, uint64_t *st_hist) {
    orc_ebur128_tables(NULL, NULL);
    memset(e, 0, sizeof *e);
    e->channels = channels;
    orc_ebur128_weights(channels, e->w);
    orc_kweight_coefs(fs, e->b, e->a);
    e->h100 = (size_t)((fs + 5) / 10);
    e->ring_frames = (size_t)fs * 3000 / 1000;
    if (e->ring_frames % e->h100) e->ring_frames = (e->ring_frames + e->h100) - (e->ring_frames % e->h100);
    e->ring = (double *)calloc(e->ring_frames * channels, sizeof(double));
    e->hist = hist;
    e->st_hist = st_hist;
    memset(hist, 0, 1000 * sizeof(uint64_t));
    memset(st_hist, 0, 1000 * sizeof(uint64_t));
    e->needed = e->h100 * 4;
}

/* ebur128_filter_double on `take` interleaved frames */
static void ebur_filter(Ebur *e, const double *x, size_t take) {
    const int ch = e->channels;
    for (int c = 0; c < ch; c++) {
        double mx = 0.0;
        for (size_t i = 0; i < take; i++) {
            double s = x[i * ch + c];
            if (s > mx) mx = s; else if (-s > mx) mx = -1.0 * s;
        }
        if (mx > e->peak[c]) e->peak[c] = mx;
    }
    const double *a = e->a, *b = e->b;
    for (int c = 0; c < ch; c++) {
        double *v = e->v[c];
        for (size_t i = 0; i < take; i++) {
            v[0] = x[i * ch + c] - a[1] * v[1] - a[2] * v[2] - a[3] * v[3] - a[4] * v[4];
            e->ring[e->idx + i * ch + c] = b[0] * v[0] + b[1] * v[1] + b[2] * v[2] + b[3] * v[3] + b[4] * v[4];
            v[4] = v[3]; v[3] = v[2]; v[2] = v[1]; v[1] = v[0];
        }
        for (int k = 1; k < 5; k++) v[k] = fabs(v[k]) < DBL_MIN ? 0.0 : v[k];
    }
}

static double ebur_block_energy(const Ebur *e, size_t fpb) {
    const int ch = e->channels;
    double sum = 0.0;
    for (int c = 0; c < ch; c++) {
        if (e->w[c] == 0.0) continue;                 /* FF_EBUR128_UNUSED */
        double cs = 0.0;
        if (e->idx < fpb * ch) {
            for (size_t i = 0; i < e->idx / ch; ++i) cs += e->ring[i * ch + c] * e->ring[i * ch + c];
            for (size_t i = e->ring_frames - (fpb - e->idx / ch); i < e->ring_frames; ++i)
                cs += e->ring[i * ch + c] * e->ring[i * ch + c];
        } else {
            for (size_t i = e->idx / ch - fpb; i < e->idx / ch; ++i) cs += e->ring[i * ch + c] * e->ring[i * ch + c];
        }
        if (e->w[c] != 1.0) cs *= e->w[c];            /* the surrounds' 1.41 */
        sum += cs;
    }
    return sum / (double)fpb;
}

/* ff_ebur128_add_frames_double: one call, split at the block boundaries */
static void ebur_add(Ebur *e, const double *x, size_t frames) {
    const int ch = e->channels;
    size_t src = 0;
    while (frames > 0) {
        if (frames >= e->needed) {
            ebur_filter(e, x + src * ch, e->needed);
            src += e->needed;
            frames -= e->needed;
            e->idx += e->needed * ch;
            double en = ebur_block_energy(e, e->h100 * 4);       /* gating block */
            e->nb++;
            if (en >= hist_bounds[0]) ++e->hist[find_hist_index(en)];
            e->st_counter += e->needed;
            if (e->st_counter == e->h100 * 30) {
                double st = ebur_block_energy(e, e->h100 * 30);
                if (st >= hist_bounds[0]) ++e->st_hist[find_hist_index(st)];
                e->st_counter = e->h100 * 20;
            }
            e->needed = e->h100;
            if (e->idx == e->ring_frames * ch) e->idx = 0;
        } else {
            ebur_filter(e, x + src * ch, frames);
            e->idx += frames * ch;
            e->st_counter += frames;
            e->needed -= frames;
            frames = 0;
        }
    }
}

/* libebur128 over an s16 track fed as doubles x/32768 at its own rate, as ONE
 * add_frames call (kept for the EBU Tech 3341/3342 known answers; ffmpeg's
 * loudnorm pass 1 measures at 192 kHz, orc_ebur128_192k below). */
EXPORT void orc_ebur128(const int16_t *x, int64_t n, int fs, int channels,
                        uint64_t *hist, uint64_t *st_hist, double *peak,
                        int64_t *n_blocks) {
    Ebur e;
    ebur_init(&e, fs, channels, hist, st_hist);
    double *buf = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1) * channels);
    for (int64_t i = 0; i < n * channels; i++) buf[i] = (double)x[i] * (1.0 / 32768.0);
    ebur_add(&e, buf, (size_t)n);
    for (int c = 0; c < channels; c++) peak[c] = e.peak[c];
    *n_blocks = e.nb;
    free(buf);
    free(e.ring);
}

/* ------------------------------------- libswresample: s16 -> 192 kHz float
 * ffmpeg's loudnorm pass 1 (:229) gets no measured_* values, so af_loudnorm is in
 * dynamic mode and asks for 192 kHz input (query_formats); ffmpeg auto-inserts a
 * resampler: libswresample with its defaults (swresample options.c): filter_size
 * 32, phase_shift 10, linear_interp 1, exact_rational 1, cutoff 0 -> 0.97, Kaiser
 * window beta 9.  s16 in / dbl out picks the FLTP internal format (swr_init), so
 * the filter bank is float32 and every output sample is a float32 dot product.
 * Restated from resample.c (build_filter, bessel, resample_init,
 * invert_initial_buffer, resample_flush) and the float kernel's order of operations
 * on an x86-64 host with FMA3 (resample.asm, ymm: 8 fused chains over taps
 * k, k+8, k+16, k+24, then (a0+a4 + a2+a6) + (a1+a5 + a3+a7)).  With exact_rational
 * the phase step is an integer (frac stays 0), so linear interpolation adds 0.
 * PARITY UNPINNED: no ffmpeg binary or fixture exists here; a host without FMA3
 * sums in another order (differences of float32 rounding in the measured values). */
#define SWR_TAPS 32              /* filter_size; the filter of an upsampling rate */
#define SWR_CENTER 15            /* (taps - 1) / 2 */
#define SWR_MAX_ALLOC 256        /* the widest bank row restated (factor >= 1 / 8) */

static double swr_bessel(double x) {
    double lastv = 0, t, v;
    double inv[100];
    for (int k = 0; k < 100; k++) inv[k] = 1.0 / ((double)(k + 1) * (double)(k + 1));
    x = x * x / 4;
    t = x;
    v = 1 + x;
    for (int i = 1; v != lastv; i += 2) {
        t *= x * inv[i];
        v += t;
        lastv = v;
        t *= x * inv[i + 1];
        v += t;
    }
    return v;
}

static int64_t gcd64(int64_t a, int64_t b) { while (b) { int64_t t = a % b; a = b; b = t; } return a; }

/* L / M = out_rate / in_rate reduced (output j sits at input position j M / L); 0 =
 * supported, else -1.  The filter bank has orc_swr_phases() rows: L when L <= 1024
 * (exact_rational: phase_count = L), else 1024 (libswresample's default phase_shift 10;
 * the position then falls between phases and the linear path interpolates, see
 * swr_block).  Inputs above 192 kHz / 0.97 (the loudnorm pass-1 resampler then
 * DOWNsamples: 352.8 / 384 / 705.6 / 768 kHz) take the longer, narrower filter of
 * orc_swr_filter; the interpolating path is restated for the 32-tap filter only. */
EXPORT int orc_swr_geometry(int in_rate, int out_rate, int *L, int *M) {
    if (in_rate <= 0 || out_rate <= 0) return -1;
    int64_t g = gcd64(in_rate, out_rate);
    int64_t l = out_rate / g, m = in_rate / g;
    *L = (int)l;
    *M = (int)m;
    return 0;
}

/* resample_init: factor = min(out_rate * cutoff / in_rate, 1) (cutoff 0.97);
 * filter_length = max(ceil(filter_size / factor), 1) rounded up to even; the bank rows
 * are filter_alloc = FFALIGN(filter_length, 8) floats (zeros past filter_length) */
EXPORT int orc_swr_filter(int in_rate, int out_rate, int *taps, int *alloc, double *factor) {
    if (in_rate <= 0 || out_rate <= 0) return -1;
    double f = out_rate * 0.97 / in_rate;
    if (f > 1.0 || in_rate == out_rate) f = 1.0;   /* equal rates: no resampling (the identity row) */
    int t = (int)ceil(SWR_TAPS / f);
    if (t < 1) t = 1;
    if (t > 1) t = (t + 1) & ~1;
    const int al = (t + 7) & ~7;
    if (al > SWR_MAX_ALLOC) return -1;
    if (taps) *taps = t;
    if (alloc) *alloc = al;
    if (factor) *factor = f;
    return 0;
}

/* resample_init: phase_count = 1 << phase_shift (1024), replaced by the exact
 * out / gcd when that is <= 1024 */
EXPORT int orc_swr_phases(int in_rate, int out_rate) {
    int L, M, t, al;
    if (orc_swr_geometry(in_rate, out_rate, &L, &M)) return -1;
    if (orc_swr_filter(in_rate, out_rate, &t, &al, NULL)) return -1;
    if (L > 1024 && t != SWR_TAPS) return -1;    /* interpolating downsampler: not restated */
    return L <= 1024 ? L : 1024;
}

/* resample_init: av_reduce(&src_incr, &dst_incr, out_rate, in_rate * phase_count,
 * INT32_MAX / 2), both doubled while below 2^20.  Per output the phase index moves by
 * dst_incr / src_incr (integer part dst_incr_div, fraction frac in units of 1/src_incr) */
EXPORT int orc_swr_incr(int in_rate, int out_rate, int64_t *src_incr, int64_t *dst_incr) {
    const int pc = orc_swr_phases(in_rate, out_rate);
    if (pc < 0) return -1;
    int64_t a = out_rate, b = (int64_t)in_rate * pc;
    const int64_t g = gcd64(a, b);
    a /= g;
    b /= g;
    while (b < (1 << 20) && a < (1 << 20)) { a *= 2; b *= 2; }
    *src_incr = a;
    *dst_incr = b;
    return 0;
}

/* build_filter (Kaiser, FLTP, scale 1): bank[ph][i] (rows of filter_alloc floats,
 * zeros past filter_length), ph < pc.  factor 1 (upsampling) forms sin(x) / x from a
 * sine table alternating in sign; factor < 1 (downsampling) from sin(x) itself */
EXPORT int orc_swr_bank(int in_rate, int out_rate, float *bank) {
    const int pc = orc_swr_phases(in_rate, out_rate);
    int tap_count, alloc;
    double factor;
    if (pc < 0 || orc_swr_filter(in_rate, out_rate, &tap_count, &alloc, &factor)) return -1;
    const int center = (tap_count - 1) / 2;
    const int ph_nb = pc % 2 ? pc : pc / 2 + 1;
    const double beta = 9.0;
    double tab[SWR_MAX_ALLOC];
    double *sin_lut = (double *)malloc(sizeof(double) * ph_nb);
    double norm = 0;
    memset(bank, 0, sizeof(float) * (size_t)pc * alloc);
    if (factor == 1.0)
        for (int ph = 0; ph < ph_nb; ph++) sin_lut[ph] = sin(M_PI * ph / pc) * (center & 1 ? 1 : -1);
    for (int ph = 0; ph < ph_nb; ph++) {
        double s = factor == 1.0 ? sin_lut[ph] : 0.0;
        for (int i = 0; i < tap_count; i++) {
            double x = M_PI * ((double)(i - center) - (double)ph / pc) * factor;
            double y;
            if (x == 0) y = 1.0;
            else if (factor == 1.0) y = s / x;
            else y = sin(x) / x;
            double w = 2.0 * x / (factor * tap_count * M_PI);
            y *= swr_bessel(beta * sqrt(fmax(1 - w * w, 0)));
            tab[i] = y;
            s = -s;
            if (!ph) norm += y;
        }
        for (int i = 0; i < tap_count; i++) bank[ph * alloc + i] = (float)(tab[i] * 1 / norm);
        if (pc % 2) continue;
        for (int i = 0; i < tap_count; i++)
            if (pc - ph < pc) bank[(pc - ph) * alloc + tap_count - 1 - i] = bank[ph * alloc + i];
    }
    free(sin_lut);
    return 0;
}

EXPORT int64_t orc_swr_out_frames(int64_t n, int in_rate, int out_rate) {
    int L, M;
    if (orc_swr_geometry(in_rate, out_rate, &L, &M)) return -1;
    return (n * L + M - 1) / M;
}

/* input sample k of the stream the resampler sees: mirrored at both ends
 * (invert_initial_buffer: x[-k] = x[k]; resample_flush: x[n+j] = x[n-1-j]) */
static inline int64_t swr_reflect(int64_t k, int64_t n) {
    for (;;) {
        if (k < 0) k = -k;
        else if (k >= n) k = 2 * n - 1 - k;
        else return k;
    }
}

/* the float kernel's order (see above): the ymm loop runs over filter_alloc taps (the
 * row's zero padding multiplies the samples that follow the window) */
static inline float swr_dot(const float *w, const float *h, int alloc) {
    float a[8];
    for (int k = 0; k < 8; k++) {
        float acc = fmaf(w[k], h[k], 0.0f);
        for (int q = 8; q < alloc; q += 8) acc = fmaf(w[k + q], h[k + q], acc);
        a[k] = acc;
    }
    const float b0 = a[0] + a[4], b1 = a[1] + a[5], b2 = a[2] + a[6], b3 = a[3] + a[7];
    return (b0 + b2) + (b1 + b3);
}

/* resample_linear_float (resample.asm, FMA3): the dot products with rows ph (h) and
 * ph + 1 (h2) run as two sets of 8 fused chains in the same loop; each set is folded
 * to 4 lanes (a[k] + a[k + 4]); per lane val += (v2 - val) * wf as one FMA, wf =
 * (float)frac * (1.0f / src_incr) (cvtsi2ss, a float reciprocal formed once); then
 * the horizontal sum of the common kernel.  PARITY UNPINNED: our reading of the
 * published assembly, no ffmpeg here to check it against */
static inline float swr_dot_lin(const float *w, const float *h, const float *h2, float wf) {
    float a[8], c[8];
    for (int k = 0; k < 8; k++) {
        float acc = fmaf(w[k], h[k], 0.0f), acc2 = fmaf(w[k], h2[k], 0.0f);
        for (int q = 8; q < 32; q += 8) {
            acc = fmaf(w[k + q], h[k + q], acc);
            acc2 = fmaf(w[k + q], h2[k + q], acc2);
        }
        a[k] = acc;
        c[k] = acc2;
    }
    float e[4];
    for (int k = 0; k < 4; k++) {
        const float b = a[k] + a[k + 4], d = (c[k] + c[k + 4]) - b;
        e[k] = fmaf(d, wf, b);
    }
    return (e[0] + e[2]) + (e[1] + e[3]);
}

/* Resampler geometry for one rate: the bank has pc + 1 rows (row pc = row 0 one tap
 * later, build_filter's extra row for the interpolation at the last phase) */
typedef struct {
    int L, M, pc, lin;
    int taps, alloc, center;      /* filter_length, filter_alloc, (taps - 1) / 2 */
    int64_t src_incr, dst_incr;
    float inv;                    /* 1.0f / (float)src_incr */
    float *bank;
} Swr;

static int swr_open(Swr *r, int in_rate, int out_rate) {
    if (orc_swr_geometry(in_rate, out_rate, &r->L, &r->M)) return -1;
    r->pc = orc_swr_phases(in_rate, out_rate);
    if (r->pc < 0 || orc_swr_filter(in_rate, out_rate, &r->taps, &r->alloc, NULL)) return -1;
    r->center = (r->taps - 1) / 2;
    orc_swr_incr(in_rate, out_rate, &r->src_incr, &r->dst_incr);
    /* swri_resample: the linear kernel whenever frac or dst_incr_mod is non-zero, i.e.
     * for every output when the phase step is not an integer; else the common one */
    r->lin = (r->dst_incr % r->src_incr) != 0;
    r->inv = 1.0f / (float)r->src_incr;
    r->bank = (float *)malloc(sizeof(float) * (size_t)(r->pc + 1) * r->alloc);
    orc_swr_bank(in_rate, out_rate, r->bank);
    /* resample_init's extra row pc: row 0 one tap later within the row (filter_alloc) */
    float *ex = r->bank + (size_t)r->pc * r->alloc, *r0 = r->bank;
    for (int i = 0; i < r->alloc; i++) ex[i] = r0[(i + r->alloc - 1) % r->alloc];
    return 0;
}

/* output frames [j0, j1) of the 192 kHz stream, interleaved doubles.  Output j sits at
 * phase position p = j dst_incr / src_incr (units of 1/pc input sample; exact in
 * int64): base = floor(p) / pc, phase floor(p) % pc, frac = the remainder */
static void swr_block(const int16_t *x, int64_t n, int channels, const Swr *r,
                      int64_t j0, int64_t j1, double *out) {
    float w[SWR_MAX_ALLOC];
    for (int64_t j = j0; j < j1; j++) {
        const int64_t pos = j * r->dst_incr, idx = pos / r->src_incr, frac = pos % r->src_incr;
        const int64_t base = idx / r->pc;
        const int ph = (int)(idx % r->pc);
        const float wf = (float)frac * r->inv;
        for (int c = 0; c < channels; c++) {
            for (int i = 0; i < r->alloc; i++)
                w[i] = (float)x[swr_reflect(base - r->center + i, n) * channels + c] * (1.0f / 32768.0f);
            const float *h = r->bank + (size_t)ph * r->alloc;
            out[(j - j0) * channels + c] =
                (double)(r->lin ? swr_dot_lin(w, h, h + SWR_TAPS, wf) : swr_dot(w, h, r->alloc));
        }
    }
}

/* per-output tables of one period of L outputs (M input frames), for the GPU plan's
 * checks: base frame, phase row and interpolation weight of output n */
EXPORT int orc_swr_table(int in_rate, int out_rate, int32_t *obase, int32_t *oph, float *owt) {
    Swr r;
    if (swr_open(&r, in_rate, out_rate)) return -1;
    for (int64_t n = 0; n < r.L; n++) {
        const int64_t pos = n * r.dst_incr, idx = pos / r.src_incr, frac = pos % r.src_incr;
        obase[n] = (int32_t)(idx / r.pc);
        oph[n] = (int32_t)(idx % r.pc);
        owt[n] = (float)frac * r.inv;
    }
    free(r.bank);
    return r.lin;
}

/* the upsampled stream itself (tests: small inputs) */
EXPORT int orc_upsample(const int16_t *x, int64_t n, int channels, int in_rate, int out_rate,
                        double *out) {
    Swr r;
    if (swr_open(&r, in_rate, out_rate)) return -1;
    swr_block(x, n, channels, &r, 0, orc_swr_out_frames(n, in_rate, out_rate), out);
    free(r.bank);
    return 0;
}

/* loudnorm pass 1 as ffmpeg runs it: the s16 track resampled to 192 kHz and fed to
 * libebur128 in af_loudnorm's dynamic-mode frames (first min(3 s, all), then
 * 100 ms at a time: these calls set where the K filter's DBL_MIN flush happens). */
EXPORT int orc_ebur128_192k(const int16_t *x, int64_t n, int fs, int channels,
                            uint64_t *hist, uint64_t *st_hist, double *peak, int64_t *n_blocks) {
    const int out_rate = 192000;
    Swr r;
    if (swr_open(&r, fs, out_rate)) return -1;
    const int64_t n_out = n > 0 ? orc_swr_out_frames(n, fs, out_rate) : 0;
    const int64_t first = (int64_t)out_rate * 3, step = (int64_t)out_rate / 10;
    double *buf = (double *)malloc(sizeof(double) * (size_t)first * channels);
    Ebur e;
    ebur_init(&e, out_rate, channels, hist, st_hist);
    for (int64_t j = 0; j < n_out;) {
        const int64_t take = (j == 0 ? first : step) < n_out - j ? (j == 0 ? first : step) : n_out - j;
        swr_block(x, n, channels, &r, j, j + take, buf);
        ebur_add(&e, buf, (size_t)take);
        j += take;
    }
    for (int c = 0; c < channels; c++) peak[c] = e.peak[c];
    *n_blocks = e.nb;
    free(buf);
    free(r.bank);
    free(e.ring);
    return 0;
}

/* ------------------------------------------------------------ alimiter */
/* FFmpeg af_alimiter.c filter_frame(), restated for interleaved doubles with
 * asc (auto release) off -- the reference passes only
 * level_in=1:level_out=1:limit=0.98:attack=5:release=50 (:223), so
 * asc=0, level (auto level)=1, latency=0.  Input s16 -> double x/32768,
 * output double -> s16 llrint(x*32768) clipped.  Output is the input delayed
 * by buffer_size/channels - 1 frames (no latency compensation). */
EXPORT void orc_alimiter(const int16_t *x, int64_t n, int fs, int channels,
                         double level_in, double level_out, double limit,
                         double attack_ms, double release_ms, int auto_level,
                         int16_t *out) {
    double attack = attack_ms / 1000.0, release = release_ms / 1000.0;
    int buffer_size = (int)(fs * attack * channels);
    buffer_size -= buffer_size % channels;
    int max_size = (int)((int64_t)fs * 100 / 1000) * channels; /* av_rescale(sr,100,1000)*ch */
    if (max_size < buffer_size + channels) max_size = buffer_size + channels;
    double *buffer = (double *)calloc((size_t)max_size, sizeof(double));
    double *nextdelta = (double *)calloc((size_t)max_size, sizeof(double));
    int *nextpos = (int *)malloc(sizeof(int) * (size_t)max_size);
    for (int i = 0; i < max_size; i++) nextpos[i] = -1;
    double att = 1.0, delta = 0.0;
    int pos = 0, nextiter = 0, nextlen = 0;
    double level = auto_level ? 1 / limit : 1;
    for (int64_t nn = 0; nn < n; nn++) {
        const int16_t *src = x + nn * channels;
        double dst[8];
        double peak = 0;
        for (int c = 0; c < channels; c++) {
            double sample = ((double)src[c] * (1.0 / 32768.0)) * level_in;
            buffer[pos + c] = sample;
            peak = fmax(peak, fabs(sample));
        }
        if (peak > limit) {
            double patt = fmin(limit / peak, 1.);
            double rdelta = (1.0 - patt) / (fs * release);
            double d = (limit / peak - att) / buffer_size * channels;
            int found = 0, i;
            if (d < delta) {
                delta = d;
                nextpos[0] = pos;
                nextpos[1] = -1;
                nextdelta[0] = rdelta;
                nextlen = 1;
                nextiter = 0;
            } else {
                for (i = nextiter; i < nextiter + nextlen; i++) {
                    int j = i % buffer_size;
                    double ppeak = 0, pdelta;
                    for (int c = 0; c < channels; c++) ppeak = fmax(ppeak, fabs(buffer[nextpos[j] + c]));
                    pdelta = (limit / peak - limit / ppeak) /
                             (((buffer_size - nextpos[j] + pos) % buffer_size) / channels);
                    if (pdelta < nextdelta[j]) {
                        nextdelta[j] = pdelta;
                        found = 1;
                        break;
                    }
                }
                if (found) {
                    nextlen = i - nextiter + 1;
                    nextpos[(nextiter + nextlen) % buffer_size] = pos;
                    nextdelta[(nextiter + nextlen) % buffer_size] = rdelta;
                    nextpos[(nextiter + nextlen + 1) % buffer_size] = -1;
                    nextlen++;
                }
            }
        }
        double *buf = &buffer[(pos + channels) % buffer_size];
        peak = 0;
        for (int c = 0; c < channels; c++) peak = fmax(peak, fabs(buf[c]));
        att += delta;
        for (int c = 0; c < channels; c++) dst[c] = buf[c] * att;
        if ((pos + channels) % buffer_size == nextpos[nextiter]) {
            delta = nextdelta[nextiter];
            att = limit / peak;
            nextlen -= 1;
            nextpos[nextiter] = -1;
            nextiter = (nextiter + 1) % buffer_size;
        }
        if (att > 1.) {
            att = 1.;
            delta = 0.;
            nextiter = 0;
            nextlen = 0;
            nextpos[0] = -1;
        }
        if (att <= 0.) {
            att = 0.0000000000001;
            delta = (1.0 - att) / (fs * release);
        }
        if (att != 1. && (1. - att) < 0.0000000000001) att = 1.;
        if (delta != 0. && fabs(delta) < 0.00000000000001) delta = 0.;
        for (int c = 0; c < channels; c++) {
            double v = dst[c];
            v = v < -limit ? -limit : (v > limit ? limit : v);
            v = v * level * level_out;
            double q = (double)llrint(v * 32768.0);
            out[nn * channels + c] = (int16_t)(q > 32767 ? 32767 : (q < -32768 ? -32768 : q));
        }
        pos = (pos + channels) % buffer_size;
    }
    free(buffer);
    free(nextdelta);
    free(nextpos);
}

/* loudnorm LINEAR mode (af_loudnorm.c, pass 2 at :240 when the measured values
 * allow it): dst = src * 10^((I_target - I_measured)/20) on doubles x/32768,
 * then s16 via llrint(x*32768) clipped. */
EXPORT void orc_linear_gain(const int16_t *x, int64_t n_samples, double gain, int16_t *out) {
    for (int64_t i = 0; i < n_samples; i++) {
        double v = ((double)x[i] * (1.0 / 32768.0)) * gain;
        double q = (double)llrint(v * 32768.0);
        out[i] = (int16_t)(q > 32767 ? 32767 : (q < -32768 ? -32768 : q));
    }
}

/* A.1: ffmpeg's f32 -> s16 conversion, clip(lrintf(x*32768)); mono duplicated. */
EXPORT void orc_quantize(const float *x, int64_t n, int channels, int16_t *out) {
    for (int64_t i = 0; i < n; i++) {
        for (int c = 0; c < 2; c++) {
            float v = x[i * channels + (channels == 1 ? 0 : c)] * 32768.0f;
            long q = lrintf(v);
            out[2 * i + c] = (int16_t)(q > 32767 ? 32767 : (q < -32768 ? -32768 : q));
        }
    }
}

/* A.1 for every sample of a C > 2 channel file (no duplication): n_samples values */
EXPORT void orc_quantize_flat(const float *x, int64_t n_samples, int16_t *out) {
    for (int64_t i = 0; i < n_samples; i++) {
        long q = lrintf(x[i] * 32768.0f);
        out[i] = (int16_t)(q > 32767 ? 32767 : (q < -32768 ? -32768 : q));
    }
}

/* libebur128 gated loudness / relative threshold / loudness range from
 * histograms (ebur128_gated_loudness, ff_ebur128_relative_threshold,
 * ff_ebur128_loudness_range_multiple), single state.  out[0]=I, out[1]=LRA,
 * out[2]=threshold (LUFS). */
EXPORT void orc_loudness_stats(const uint64_t *hist, const uint64_t *st_hist, double *out) {
    orc_ebur128_tables(NULL, NULL);
    const double gate = pow(10.0, -10.0 / 10.0);
    double rel = 0.0;
    uint64_t cnt = 0;
    for (int j = 0; j < 1000; ++j) { rel += hist[j] * hist_energies[j]; cnt += hist[j]; }
    double I = -HUGE_VAL, thr = -70.0;
    if (cnt) {
        rel /= (double)cnt;
        rel *= gate;
        thr = 10 * log10(rel) - 0.691;
        size_t start;
        if (rel < hist_bounds[0]) start = 0;
        else { start = find_hist_index(rel); if (rel > hist_energies[start]) ++start; }
        double g = 0.0;
        uint64_t above = 0;
        for (size_t j = start; j < 1000; ++j) { g += hist[j] * hist_energies[j]; above += hist[j]; }
        if (above) I = 10 * log10(g / (double)above) - 0.691;
    }
    /* LRA */
    double lra = 0.0, stl_size = 0.0, stl_power = 0.0;
    for (int j = 0; j < 1000; ++j) { stl_size += st_hist[j]; stl_power += st_hist[j] * hist_energies[j]; }
    if (stl_size) {
        stl_power /= stl_size;
        double stl_int = pow(10.0, -20.0 / 10.0) * stl_power;
        size_t index;
        if (stl_int < hist_bounds[0]) index = 0;
        else { index = find_hist_index(stl_int); if (stl_int > hist_energies[index]) ++index; }
        stl_size = 0;
        for (size_t j = index; j < 1000; ++j) stl_size += st_hist[j];
        if (stl_size) {
            size_t plo = (size_t)((stl_size - 1) * 0.1 + 0.5);
            size_t phi = (size_t)((stl_size - 1) * 0.95 + 0.5);
            stl_size = 0;
            size_t j = index;
            while (stl_size <= plo) stl_size += st_hist[j++];
            double l_en = hist_energies[j - 1];
            while (stl_size <= phi) stl_size += st_hist[j++];
            double h_en = hist_energies[j - 1];
            lra = (10 * log10(h_en) - 0.691) - (10 * log10(l_en) - 0.691);
        }
    }
    out[0] = I;
    out[1] = lra;
    out[2] = thr;
}

/* ------------------------------------------------ loudnorm: the whole filter
 * FFmpeg af_loudnorm.c restated (config_input, init_gaussian_filter,
 * gaussian_filter, detect_peak, true_peak_limiter, filter_frame, flush_frame and
 * activate's framing: a first frame of 3 s, then 100 ms frames, a flush frame at
 * EOF) on the s16 track resampled to 192 kHz (swr_block above; the 192 kHz input
 * format is what makes ffmpeg insert the resampler, whichever mode is taken).
 * Options as the reference passes them: pass 1 (:229) I/TP/LRA only (measured_*
 * defaults: I 0, LRA 0, TP 99, thresh -70, offset 0), pass 2 (:240) all measured
 * values and offset = pass 1's target_offset.  linear=1 (default): with valid
 * measured values that meet TP and LRA, init picks LINEAR_MODE and the filter keeps
 * the input rate (no resampler) -- orc_linear_gain covers that case; here the
 * 192 kHz modes: dynamic (FIRST / INNER / FINAL frames) and the LINEAR_MODE a
 * first frame shorter than 3 s falls back to.
 * PARITY UNPINNED: restated from the published source, no ffmpeg here.  Open
 * point: the flush frame goes through filter_frame, whose first statement feeds
 * r128_in; if ffmpeg does that, pass 1's input_* also count the last 2.9 s twice.
 * This restatement (and the GPU measurement) feed r128_in once. */
enum { LN_FIRST, LN_INNER, LN_FINAL, LN_LINEAR };
enum { LIM_OUT, LIM_ATTACK, LIM_SUSTAIN, LIM_RELEASE };

typedef struct {
    double target_i, target_lra, target_tp;          /* dB (TP in dBTP) */
    double measured_i, measured_lra, measured_tp, measured_thresh, offset;
} orc_loudnorm_opts;

typedef struct {
    int ch, fs;
    double target_i, target_lra, target_tp, measured_i, measured_lra, measured_tp,
        measured_thresh, offset;
    double *buf;
    int buf_size, buf_index, prev_buf_index;
    double delta[30], weights[21], prev_delta;
    int index;
    double gain_reduction[2];
    double *limiter_buf;
    double prev_smp[8];
    int limiter_buf_index, limiter_buf_size, limiter_state, peak_index, env_index, env_cnt,
        attack_length, release_length;
    int frame_type, above_threshold, prev_nb_samples;
    Ebur rin, rout;
    uint64_t hin[1000], sin_[1000], hout[1000], sout[1000];
} Ln;

static int ln_frame_size(int sample_rate, int frame_len_msec) {
    const int fsz = (int)round((double)sample_rate * (frame_len_msec / 1000.0));
    return fsz + (fsz % 2);
}

static double ln_energy_to_loudness(double e) { return 10 * log10(e) - 0.691; }

static double ln_shortterm(const Ebur *e) { return ln_energy_to_loudness(ebur_block_energy(e, e->h100 * 30)); }

static double ln_global(const Ebur *e) {
    double s[3];
    orc_loudness_stats(e->hist, e->st_hist, s);
    return s[0];
}

static double ln_relative_threshold(const Ebur *e) {
    double s[3];
    orc_loudness_stats(e->hist, e->st_hist, s);
    return s[2];
}

static void ln_init(Ln *s, int fs, int ch, const orc_loudnorm_opts *o) {
    memset(s, 0, sizeof *s);
    s->ch = ch;
    s->fs = fs;
    s->target_i = o->target_i;
    s->target_lra = o->target_lra;
    s->target_tp = o->target_tp;
    s->measured_i = o->measured_i;
    s->measured_lra = o->measured_lra;
    s->measured_tp = o->measured_tp;
    s->measured_thresh = o->measured_thresh;
    s->offset = o->offset;
    s->buf_size = ln_frame_size(fs, 3000) * ch;
    s->buf = (double *)calloc((size_t)s->buf_size, sizeof(double));
    s->limiter_buf_size = ln_frame_size(fs, 210) * ch;
    s->limiter_buf = (double *)calloc((size_t)s->buf_size, sizeof(double));
    /* init_gaussian_filter */
    {
        double total = 0.0;
        const double sigma = 3.5;
        const int off = 21 / 2;
        const double c1 = 1.0 / (sigma * sqrt(2.0 * M_PI));
        const double c2 = 2.0 * pow(sigma, 2.0);
        for (int i = 0; i < 21; i++) {
            const int x = i - off;
            s->weights[i] = c1 * exp(-(pow(x, 2.0) / c2));
            total += s->weights[i];
        }
        const double adjust = 1.0 / total;
        for (int i = 0; i < 21; i++) s->weights[i] *= adjust;
    }
    s->frame_type = LN_FIRST;
    s->index = 1;
    s->limiter_state = LIM_OUT;
    s->offset = pow(10., s->offset / 20.);
    s->target_tp = pow(10., s->target_tp / 20.);
    s->attack_length = ln_frame_size(fs, 10);
    s->release_length = ln_frame_size(fs, 100);
    ebur_init(&s->rin, fs, ch, s->hin, s->sin_);
    ebur_init(&s->rout, fs, ch, s->hout, s->sout);
}

static void ln_free(Ln *s) {
    free(s->buf);
    free(s->limiter_buf);
    free(s->rin.ring);
    free(s->rout.ring);
}

static double ln_gaussian(const Ln *s, int index) {
    double result = 0.;
    index = index - 10 > 0 ? index - 10 : index + 20;
    for (int i = 0; i < 21; i++)
        result += s->delta[((index + i) < 30) ? (index + i) : (index + i - 30)] * s->weights[i];
    return result;
}

#define LN_W(i) ((i) < s->limiter_buf_size ? (i) : (i) - s->limiter_buf_size)

static void ln_detect_peak(Ln *s, int offset, int nb_samples, int channels, int *peak_delta,
                           double *peak_value) {
    const double *buf = s->limiter_buf;
    const double ceiling = s->target_tp;
    *peak_delta = -1;
    int index = s->limiter_buf_index + (offset * channels) + (1920 * channels);
    if (index >= s->limiter_buf_size) index -= s->limiter_buf_size;
    if (s->frame_type == LN_FIRST)
        for (int c = 0; c < channels; c++) s->prev_smp[c] = fabs(buf[index + c - channels]);
    for (int n = 0; n < nb_samples; n++) {
        for (int c = 0; c < channels; c++) {
            double th = fabs(buf[LN_W(index + c)]);
            double next = fabs(buf[LN_W(index + c + channels)]);
            if ((s->prev_smp[c] <= th) && (next <= th) && (th > ceiling) && (n > 0)) {
                int detected = 1;
                for (int i = 2; i < 12; i++) {
                    next = fabs(buf[LN_W(index + c + (i * channels))]);
                    if (next > th) {
                        detected = 0;
                        break;
                    }
                }
                if (!detected) continue;
                double max_peak = 0.0;
                for (c = 0; c < channels; c++) {
                    if (c == 0 || fabs(buf[index + c]) > max_peak) max_peak = fabs(buf[index + c]);
                    s->prev_smp[c] = fabs(buf[LN_W(index + c)]);
                }
                *peak_delta = n;
                s->peak_index = index;
                *peak_value = max_peak;
                return;
            }
            s->prev_smp[c] = th;
        }
        index += channels;
        if (index >= s->limiter_buf_size) index -= s->limiter_buf_size;
    }
}

static void ln_true_peak_limiter(Ln *s, double *out, int nb_samples, int channels) {
    double *buf = s->limiter_buf;
    const double ceiling = s->target_tp;
    int index = s->limiter_buf_index, smp_cnt = 0, peak_delta = -1;
    double peak_value = 0.0;
    if (s->frame_type == LN_FIRST) {
        double max = 0.;
        for (int n = 0; n < 1920; n++) {
            for (int c = 0; c < channels; c++) max = fabs(buf[c]) > max ? fabs(buf[c]) : max;
            buf += channels;
        }
        if (max > ceiling) {
            s->gain_reduction[1] = ceiling / max;
            s->limiter_state = LIM_SUSTAIN;
            buf = s->limiter_buf;
            for (int n = 0; n < 1920; n++) {
                for (int c = 0; c < channels; c++) buf[c] *= s->gain_reduction[1];
                buf += channels;
            }
        }
        buf = s->limiter_buf;
    }
    do {
        switch (s->limiter_state) {
        case LIM_OUT:
            ln_detect_peak(s, smp_cnt, nb_samples - smp_cnt, channels, &peak_delta, &peak_value);
            if (peak_delta != -1) {
                s->env_cnt = 0;
                smp_cnt += (peak_delta - s->attack_length);
                s->gain_reduction[0] = 1.;
                s->gain_reduction[1] = ceiling / peak_value;
                s->limiter_state = LIM_ATTACK;
                s->env_index = s->peak_index - (s->attack_length * channels);
                if (s->env_index < 0) s->env_index += s->limiter_buf_size;
                s->env_index += (s->env_cnt * channels);
                if (s->env_index > s->limiter_buf_size) s->env_index -= s->limiter_buf_size;
            } else {
                smp_cnt = nb_samples;
            }
            break;
        case LIM_ATTACK:
            for (; s->env_cnt < s->attack_length; s->env_cnt++) {
                for (int c = 0; c < channels; c++) {
                    double env = s->gain_reduction[0] - ((double)s->env_cnt / (s->attack_length - 1) *
                                                         (s->gain_reduction[0] - s->gain_reduction[1]));
                    buf[s->env_index + c] *= env;
                }
                s->env_index += channels;
                if (s->env_index >= s->limiter_buf_size) s->env_index -= s->limiter_buf_size;
                smp_cnt++;
                if (smp_cnt >= nb_samples) {
                    s->env_cnt++;
                    break;
                }
            }
            if (smp_cnt < nb_samples) {
                s->env_cnt = 0;
                s->attack_length = 1920;
                s->limiter_state = LIM_SUSTAIN;
            }
            break;
        case LIM_SUSTAIN:
            ln_detect_peak(s, smp_cnt, nb_samples, channels, &peak_delta, &peak_value);
            if (peak_delta == -1) {
                s->limiter_state = LIM_RELEASE;
                s->gain_reduction[0] = s->gain_reduction[1];
                s->gain_reduction[1] = 1.;
                s->env_cnt = 0;
                break;
            } else {
                double gain_reduction = ceiling / peak_value;
                if (gain_reduction < s->gain_reduction[1]) {
                    s->limiter_state = LIM_ATTACK;
                    s->attack_length = peak_delta;
                    if (s->attack_length <= 1) s->attack_length = 2;
                    s->gain_reduction[0] = s->gain_reduction[1];
                    s->gain_reduction[1] = gain_reduction;
                    s->env_cnt = 0;
                    break;
                }
                for (s->env_cnt = 0; s->env_cnt < peak_delta; s->env_cnt++) {
                    for (int c = 0; c < channels; c++) buf[s->env_index + c] *= s->gain_reduction[1];
                    s->env_index += channels;
                    if (s->env_index >= s->limiter_buf_size) s->env_index -= s->limiter_buf_size;
                    smp_cnt++;
                    if (smp_cnt >= nb_samples) {
                        s->env_cnt++;
                        break;
                    }
                }
            }
            break;
        case LIM_RELEASE:
            for (; s->env_cnt < s->release_length; s->env_cnt++) {
                for (int c = 0; c < channels; c++) {
                    double env = s->gain_reduction[0] + (((double)s->env_cnt / (s->release_length - 1)) *
                                                         (s->gain_reduction[1] - s->gain_reduction[0]));
                    buf[s->env_index + c] *= env;
                }
                s->env_index += channels;
                if (s->env_index >= s->limiter_buf_size) s->env_index -= s->limiter_buf_size;
                smp_cnt++;
                if (smp_cnt >= nb_samples) {
                    s->env_cnt++;
                    break;
                }
            }
            if (smp_cnt < nb_samples) {
                s->env_cnt = 0;
                s->limiter_state = LIM_OUT;
            }
            break;
        }
    } while (smp_cnt < nb_samples);
    for (int n = 0; n < nb_samples; n++) {
        for (int c = 0; c < channels; c++) {
            out[c] = buf[index + c];
            if (fabs(out[c]) > ceiling) out[c] = ceiling * (out[c] < 0 ? -1 : 1);
        }
        out += channels;
        index += channels;
        if (index >= s->limiter_buf_size) index -= s->limiter_buf_size;
    }
}

/* filter_frame on one input frame of nb frames (src interleaved); writes the output
 * frame to dst and returns its frame count */
static int ln_filter_frame(Ln *s, const double *src, int nb, double *dst, int feed_in) {
    const int ch = s->ch;
    double *buf = s->buf, *limiter_buf = s->limiter_buf;
    int out_nb = nb;
    if (feed_in) ebur_add(&s->rin, src, (size_t)nb);
    if (s->frame_type == LN_FIRST && nb < ln_frame_size(s->fs, 3000)) {
        double global = ln_global(&s->rin), true_peak = 0.0;
        for (int c = 0; c < ch; c++)
            if (c == 0 || s->rin.peak[c] > true_peak) true_peak = s->rin.peak[c];
        const double offset = pow(10., (s->target_i - global) / 20.);
        const double offset_tp = true_peak * offset;
        s->offset = offset_tp < s->target_tp ? offset : s->target_tp / true_peak;
        s->frame_type = LN_LINEAR;
    }
    switch (s->frame_type) {
    case LN_FIRST: {
        for (int n = 0; n < nb; n++) {
            for (int c = 0; c < ch; c++) buf[s->buf_index + c] = src[c];
            src += ch;
            s->buf_index += ch;
        }
        const double shortterm = ln_shortterm(&s->rin);
        double env_shortterm;
        if (shortterm < s->measured_thresh) {
            s->above_threshold = 0;
            env_shortterm = shortterm <= -70. ? 0. : s->target_i - s->measured_i;
        } else {
            s->above_threshold = 1;
            env_shortterm = shortterm <= -70. ? 0. : s->target_i - shortterm;
        }
        for (int n = 0; n < 30; n++) s->delta[n] = pow(10., env_shortterm / 20.);
        s->prev_delta = s->delta[s->index];
        s->buf_index = s->limiter_buf_index = 0;
        for (int n = 0; n < (s->limiter_buf_size / ch); n++) {
            for (int c = 0; c < ch; c++)
                s->limiter_buf[s->limiter_buf_index + c] = buf[s->buf_index + c] * s->delta[s->index] * s->offset;
            s->limiter_buf_index += ch;
            if (s->limiter_buf_index >= s->limiter_buf_size) s->limiter_buf_index -= s->limiter_buf_size;
            s->buf_index += ch;
        }
        const int sub = ln_frame_size(s->fs, 100);
        ln_true_peak_limiter(s, dst, sub, ch);
        ebur_add(&s->rout, dst, (size_t)sub);
        out_nb = sub;
        s->frame_type = LN_INNER;
        break;
    }
    case LN_INNER: {
        const double gain = ln_gaussian(s, s->index + 10 < 30 ? s->index + 10 : s->index + 10 - 30);
        const double gain_next = ln_gaussian(s, s->index + 11 < 30 ? s->index + 11 : s->index + 11 - 30);
        for (int n = 0; n < nb; n++) {
            for (int c = 0; c < ch; c++) {
                buf[s->prev_buf_index + c] = src[c];
                limiter_buf[s->limiter_buf_index + c] =
                    buf[s->buf_index + c] * (gain + (((double)n / nb) * (gain_next - gain))) * s->offset;
            }
            src += ch;
            s->limiter_buf_index += ch;
            if (s->limiter_buf_index >= s->limiter_buf_size) s->limiter_buf_index -= s->limiter_buf_size;
            s->prev_buf_index += ch;
            if (s->prev_buf_index >= s->buf_size) s->prev_buf_index -= s->buf_size;
            s->buf_index += ch;
            if (s->buf_index >= s->buf_size) s->buf_index -= s->buf_size;
        }
        const int sub = (ln_frame_size(s->fs, 100) - nb) * ch;
        s->limiter_buf_index = s->limiter_buf_index + sub < s->limiter_buf_size
                                   ? s->limiter_buf_index + sub
                                   : s->limiter_buf_index + sub - s->limiter_buf_size;
        ln_true_peak_limiter(s, dst, nb, ch);
        ebur_add(&s->rout, dst, (size_t)nb);
        const double global = ln_global(&s->rin);
        const double shortterm = ln_shortterm(&s->rin);
        const double relative_threshold = ln_relative_threshold(&s->rin);
        if (s->above_threshold == 0) {
            if (shortterm > s->measured_thresh) s->prev_delta *= 1.0058;
            const double shortterm_out = ln_shortterm(&s->rout);
            if (shortterm_out >= s->target_i) s->above_threshold = 1;
        }
        if (shortterm < relative_threshold || shortterm <= -70. || s->above_threshold == 0) {
            s->delta[s->index] = s->prev_delta;
        } else {
            const double env_global = fabs(shortterm - global) < (s->target_lra / 2.)
                                          ? shortterm - global
                                          : (s->target_lra / 2.) * ((shortterm - global) < 0 ? -1 : 1);
            const double env_shortterm = s->target_i - shortterm;
            s->delta[s->index] = pow(10., (env_global + env_shortterm) / 20.);
        }
        s->prev_delta = s->delta[s->index];
        s->index++;
        if (s->index >= 30) s->index -= 30;
        s->prev_nb_samples = nb;
        break;
    }
    case LN_FINAL: {
        const double gain = ln_gaussian(s, s->index + 10 < 30 ? s->index + 10 : s->index + 10 - 30);
        int src_index = 0;
        s->limiter_buf_index = 0;
        for (int n = 0; n < s->limiter_buf_size / ch; n++) {
            for (int c = 0; c < ch; c++) s->limiter_buf[s->limiter_buf_index + c] = src[src_index + c] * gain * s->offset;
            src_index += ch;
            s->limiter_buf_index += ch;
            if (s->limiter_buf_index >= s->limiter_buf_size) s->limiter_buf_index -= s->limiter_buf_size;
        }
        const int sub = ln_frame_size(s->fs, 100);
        double *d = dst;
        for (int i = 0; i < nb / sub; i++) {
            ln_true_peak_limiter(s, d, sub, ch);
            for (int n = 0; n < sub; n++) {
                for (int c = 0; c < ch; c++) {
                    if (src_index < (nb * ch))
                        limiter_buf[s->limiter_buf_index + c] = src[src_index + c] * gain * s->offset;
                    else
                        limiter_buf[s->limiter_buf_index + c] = 0.;
                }
                if (src_index < (nb * ch)) src_index += ch;
                s->limiter_buf_index += ch;
                if (s->limiter_buf_index >= s->limiter_buf_size) s->limiter_buf_index -= s->limiter_buf_size;
            }
            d += (sub * ch);
        }
        ebur_add(&s->rout, dst, (size_t)nb);
        break;
    }
    case LN_LINEAR:
        for (int n = 0; n < nb; n++) {
            for (int c = 0; c < ch; c++) dst[c] = src[c] * s->offset;
            src += ch;
            dst += ch;
        }
        ebur_add(&s->rout, dst - (size_t)nb * ch, (size_t)nb);
        break;
    }
    return out_nb;
}

/* flush_frame: the last 3 s minus one frame, re-read from the ring, as FINAL_FRAME */
static int ln_flush(Ln *s, double *tmp, double *dst) {
    if (s->frame_type != LN_INNER) return 0;
    const int ch = s->ch;
    int nb = (s->buf_size / ch) - s->prev_nb_samples;
    nb -= (ln_frame_size(s->fs, 100) - s->prev_nb_samples);
    int offset = ((s->limiter_buf_size / ch) - s->prev_nb_samples) * ch;
    offset -= (ln_frame_size(s->fs, 100) - s->prev_nb_samples) * ch;
    s->buf_index = s->buf_index - offset < 0 ? s->buf_index - offset + s->buf_size : s->buf_index - offset;
    double *src = tmp;
    for (int n = 0; n < nb; n++) {
        for (int c = 0; c < ch; c++) src[c] = s->buf[s->buf_index + c];
        src += ch;
        s->buf_index += ch;
        if (s->buf_index >= s->buf_size) s->buf_index -= s->buf_size;
    }
    s->frame_type = LN_FINAL;
    /* filter_frame's r128_in feed is skipped for the flush frame (see the open point) */
    return ln_filter_frame(s, tmp, nb, dst, 0);
}

/* The filter over the whole 192 kHz stream of an s16 track: returns the output
 * frames (192 kHz; the input's count when it is >= 3 s), writes them as s16 the way
 * the WAV muxer's conversion does (dbl -> s16: av_clip_int16(llrint(x * 32768))) when
 * out16 is given, and the summary: stats = [input_i, input_tp (dB), input_lra,
 * input_thresh, output_i, output_tp (dB), output_lra, output_thresh, mode (1 linear,
 * 0 dynamic), target_offset].  -1: no 192 kHz resampler for fs. */
EXPORT int64_t orc_loudnorm(const int16_t *x, int64_t n, int fs, int channels,
                            const orc_loudnorm_opts *o, int16_t *out16, double *stats) {
    const int out_rate = 192000;
    Swr r;
    if (swr_open(&r, fs, out_rate)) return -1;
    const int64_t n_out = n > 0 ? orc_swr_out_frames(n, fs, out_rate) : 0;
    Ln s;
    ln_init(&s, out_rate, channels, o);
    const int first = ln_frame_size(out_rate, 3000), step = ln_frame_size(out_rate, 100);
    double *in = (double *)malloc(sizeof(double) * (size_t)first * channels);
    double *out = (double *)malloc(sizeof(double) * (size_t)first * channels);
    int64_t w = 0;                                   /* output frames written */
    for (int64_t j = 0; j < n_out;) {
        const int64_t want = s.frame_type == LN_FIRST ? first : step;
        const int take = (int)(want < n_out - j ? want : n_out - j);
        swr_block(x, n, channels, &r, j, j + take, in);
        const int m = ln_filter_frame(&s, in, take, out, 1);
        if (out16)
            for (int64_t i = 0; i < (int64_t)m * channels; i++) {
                double v = llrint(out[i] * 32768.0);
                out16[w * channels + i] = (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
            }
        w += m;
        j += take;
    }
    {
        const int m = ln_flush(&s, in, out);
        if (out16)
            for (int64_t i = 0; i < (int64_t)m * channels; i++) {
                double v = llrint(out[i] * 32768.0);
                out16[w * channels + i] = (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
            }
        w += m;
    }
    if (stats) {
        double a[3], b[3], tin = 0.0, tout = 0.0;
        orc_loudness_stats(s.hin, s.sin_, a);
        orc_loudness_stats(s.hout, s.sout, b);
        for (int c = 0; c < channels; c++) {
            if (c == 0 || s.rin.peak[c] > tin) tin = s.rin.peak[c];
            if (c == 0 || s.rout.peak[c] > tout) tout = s.rout.peak[c];
        }
        stats[0] = a[0]; stats[1] = 20. * log10(tin); stats[2] = a[1]; stats[3] = a[2];
        stats[4] = b[0]; stats[5] = 20. * log10(tout); stats[6] = b[1]; stats[7] = b[2];
        stats[8] = s.frame_type == LN_LINEAR ? 1.0 : 0.0;
        stats[9] = s.target_i - b[0];
    }
    free(in);
    free(out);
    free(r.bank);
    ln_free(&s);
    return w;
}
