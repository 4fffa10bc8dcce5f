"""ctypes front-end of the CPU parity oracle (amx_oracle.c).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker.  Never by the product package.

Coefficients are designed here with the very calls the reference makes
(scipy.signal.butter at audio_mastering_engine.py:285, :296, :301-302) and the
analog-character float32 tanh table with numpy's own float32 ``np.tanh``
(:263), so the C restatement sees exactly the reference's numbers.
"""
import ctypes
import os
import subprocess

import numpy as np
from scipy.signal import butter

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libamx_oracle.so")

_i16p = ctypes.POINTER(ctypes.c_int16)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i64 = ctypes.c_int64


class OrcEq(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int * 4), ("gain_db", ctypes.c_double * 4),
                ("g", ctypes.c_double * 4), ("coef", (ctypes.c_double * 24) * 4)]


class OrcChunk(ctypes.Structure):
    _fields_ = [("fs", ctypes.c_int), ("analog_on", ctypes.c_int),
                ("an_b_lo", ctypes.c_double * 3), ("an_a_lo", ctypes.c_double * 3),
                ("an_g_lo", ctypes.c_double), ("an_b_hi", ctypes.c_double * 3),
                ("an_a_hi", ctypes.c_double * 3), ("an_g_hi", ctypes.c_double),
                ("tanh_lut", _f32p), ("eq", OrcEq), ("width_on", ctypes.c_int),
                ("width", ctypes.c_float), ("mb_on", ctypes.c_int),
                ("xlo", ctypes.c_double * 12), ("xhi", ctypes.c_double * 12),
                ("thr_db", ctypes.c_double * 3), ("ratio", ctypes.c_double * 3)]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_overlay_len.restype = _i64
        L.orc_overlay3.restype = _i64
        L.orc_chunk.restype = _i64
        L.orc_chunk_mc.restype = _i64
        L.orc_overlay3_mc.restype = _i64
        L.orc_swr_out_frames.restype = _i64
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


# ------------------------------------------------------------------ design
def tanh_lut(character_percent):
    """np.tanh(float32(s/32768) * drive) for all 65536 s16 values (:258-263)."""
    cf = character_percent / 100.0
    drive = 1.0 + (cf * 0.5)
    s = np.arange(-32768, 32768, dtype=np.int16)
    x = s.astype(np.float32) / (2 ** 15)
    return np.ascontiguousarray(np.tanh(x * drive), dtype=np.float32)


def shelf_ba(fs, cutoff_hz, btype):
    b, a = butter(2, cutoff_hz / (0.5 * fs), btype=btype)   # :285
    return np.asarray(b, np.float64), np.asarray(a, np.float64)


def peak_sos(fs, center_hz, q=1.41):
    nyquist = 0.5 * fs                                        # :292-296
    center_norm = center_hz / nyquist
    bandwidth = center_norm / q
    low, high = center_norm - (bandwidth / 2), center_norm + (bandwidth / 2)
    if low <= 0:
        low = 1e-9
    if high >= 1.0:
        high = 0.999999
    return np.ascontiguousarray(butter(4, [low, high], btype='bandpass', output='sos'), np.float64)


def eq_struct(fs, settings):
    eq = OrcEq()
    stages = [("shelf", 250, settings.get("bass_boost", 0.0), 'low'),   # :278-281
              ("peak", 1000, -settings.get("mid_cut", 0.0), None),
              ("peak", 4000, settings.get("presence_boost", 0.0), None),
              ("shelf", 8000, settings.get("treble_boost", 0.0), 'high')]
    for i, (kind, fc, gdb, bt) in enumerate(stages):
        if gdb == 0:
            eq.kind[i] = 0
            continue
        eq.gain_db[i] = float(gdb)
        if kind == "shelf":
            eq.kind[i] = 1
            eq.g[i] = 10.0 ** (gdb / 20.0)                          # :287
            b, a = shelf_ba(fs, fc, bt)
            for k in range(3):
                eq.coef[i][k] = b[k]
                eq.coef[i][3 + k] = a[k]
        else:
            eq.kind[i] = 2
            eq.g[i] = 10 ** (gdb / 20.0)                             # :297
            sos = peak_sos(fs, fc)
            for k, v in enumerate(sos.reshape(-1)):
                eq.coef[i][k] = v
    return eq


def crossover_sos(fs, low_crossover=250, high_crossover=4000):
    lo = butter(4, low_crossover, btype='lowpass', fs=fs, output='sos')      # :301
    hi = butter(4, high_crossover, btype='highpass', fs=fs, output='sos')    # :302
    return (np.ascontiguousarray(lo, np.float64), np.ascontiguousarray(hi, np.float64))


# ------------------------------------------------------------------ stages
def analog(x16, fs, character_percent):
    x16 = np.ascontiguousarray(x16, np.int16)
    n = x16.shape[0]
    cf = character_percent / 100.0
    lut = tanh_lut(character_percent)
    blo, alo = shelf_ba(fs, 120, 'low')
    bhi, ahi = shelf_ba(fs, 12000, 'high')
    glo = 10.0 ** ((cf * 1.0) / 20.0)
    ghi = 10.0 ** ((cf * 1.5) / 20.0)
    out = np.empty_like(x16)
    lib().orc_analog(_p(x16, _i16p), _i64(n), _p(lut, _f32p), _p(blo, _f64p), _p(alo, _f64p),
                     ctypes.c_double(glo), _p(bhi, _f64p), _p(ahi, _f64p),
                     ctypes.c_double(ghi), _p(out, _i16p))
    return out


def eq(samples_f32, fs, settings):
    x = np.ascontiguousarray(samples_f32, np.float32).copy()
    st = eq_struct(fs, settings)
    n = x.shape[0]
    for c in range(x.shape[1]):
        lib().orc_eq_channel(_p(x[:, c:], _f32p), _i64(n), ctypes.c_int(x.shape[1]),
                             ctypes.byref(st), _p(x[:, c:], _f32p))
    return x


def width(samples_f32, w):
    x = np.ascontiguousarray(samples_f32, np.float32).copy()
    lib().orc_width(_p(x, _f32p), _i64(x.shape[0]), ctypes.c_float(w))
    return x


def f32_to_s16(x):
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty(x.shape, np.int16)
    lib().orc_f32_to_s16(_p(x, _f32p), _i64(x.size), _p(out, _i16p))
    return out


def crossover(p16, fs):
    p16 = np.ascontiguousarray(p16, np.int16)
    lo_sos, hi_sos = crossover_sos(fs)
    bands = [np.empty_like(p16) for _ in range(3)]
    lib().orc_crossover(_p(p16, _i16p), _i64(p16.shape[0]), _p(lo_sos, _f64p), _p(hi_sos, _f64p),
                        *[_p(b, _i16p) for b in bands])
    return bands


def compress(band16, fs, threshold, ratio, trace=False):
    band16 = np.ascontiguousarray(band16, np.int16)
    out = np.empty_like(band16)
    n = band16.shape[0]
    att = np.empty(n, np.float64) if trace else None
    lib().orc_compress(_p(band16, _i16p), _i64(n), ctypes.c_int(fs), ctypes.c_double(threshold),
                       ctypes.c_double(ratio), _p(out, _i16p),
                       _p(att, _f64p) if trace else None)
    return (out, att) if trace else out


def compress_mc(band16, fs, threshold, ratio):
    """orc_compress_mc: pydub's compressor on frames of C samples (band16 [n, C])"""
    band16 = np.ascontiguousarray(band16, np.int16)
    out = np.empty_like(band16)
    lib().orc_compress_mc(_p(band16, _i16p), _i64(band16.shape[0]), ctypes.c_int(band16.shape[1]),
                          ctypes.c_int(fs), ctypes.c_double(threshold), ctypes.c_double(ratio),
                          _p(out, _i16p), None)
    return out


def overlay_len(n, fs):
    return int(lib().orc_overlay_len(_i64(n), ctypes.c_int(fs)))


def overlay3(lo, mid, hi, fs):
    n = lo.shape[0]
    out = np.zeros((max(n, overlay_len(n, fs)) + 8, 2), np.int16)
    m = lib().orc_overlay3(_p(np.ascontiguousarray(lo), _i16p), _p(np.ascontiguousarray(mid), _i16p),
                           _p(np.ascontiguousarray(hi), _i16p), _i64(n), ctypes.c_int(fs),
                           _p(out, _i16p))
    return out[:m]


def chunk_struct(fs, settings):
    p = OrcChunk()
    p.fs = fs
    ac = settings.get("analog_character", 0)
    keep = []
    if ac > 0:
        p.analog_on = 1
        cf = ac / 100.0
        blo, alo = shelf_ba(fs, 120, 'low')
        bhi, ahi = shelf_ba(fs, 12000, 'high')
        for k in range(3):
            p.an_b_lo[k], p.an_a_lo[k] = blo[k], alo[k]
            p.an_b_hi[k], p.an_a_hi[k] = bhi[k], ahi[k]
        p.an_g_lo = 10.0 ** ((cf * 1.0) / 20.0)
        p.an_g_hi = 10.0 ** ((cf * 1.5) / 20.0)
        lut = tanh_lut(ac)
        keep.append(lut)
        p.tanh_lut = _p(lut, _f32p)
    p.eq = eq_struct(fs, settings)
    w = settings.get("width", 1.0)
    if w != 1.0:
        p.width_on = 1
        p.width = float(np.float32(w))
    if settings.get("multiband"):
        p.mb_on = 1
        lo, hi = crossover_sos(fs)
        for k, v in enumerate(lo.reshape(-1)):
            p.xlo[k] = v
        for k, v in enumerate(hi.reshape(-1)):
            p.xhi[k] = v
        for i, b in enumerate(("low", "mid", "high")):
            p.thr_db[i] = float(settings.get(b + "_thresh"))
            p.ratio[i] = float(settings.get(b + "_ratio"))
    return p, keep


def chunk(in16, fs, settings):
    """Whole chunk body (:189-197) on an s16 chunk [n,2] (mono already duplicated)."""
    in16 = np.ascontiguousarray(in16, np.int16)
    if in16.ndim == 1 or in16.shape[1] == 1:
        in16 = np.repeat(in16.reshape(-1, 1), 2, axis=1)
    n = in16.shape[0]
    p, keep = chunk_struct(fs, settings)
    out = np.zeros((max(n, overlay_len(n, fs) if n else 0) + 8, 2), np.int16)
    m = lib().orc_chunk(ctypes.byref(p), _p(in16, _i16p), _i64(n), _p(out, _i16p))
    del keep
    return out[:m]


def chunk_mc(in16, fs, settings):
    """The chunk body (:189-197) on an s16 chunk [n, C] with C > 2 channels: one
    interleaved 1-D stream through analog / EQ / crossover, no width (:252, :268),
    the compressor and overlay on C-sample frames.  Returns int16 [n', C]."""
    in16 = np.ascontiguousarray(in16, np.int16)
    n, C = in16.shape
    p, keep = chunk_struct(fs, settings)
    out = np.zeros(((max(n, overlay_len(n, fs) if n else 0) + 8), C), np.int16)
    m = lib().orc_chunk_mc(ctypes.byref(p), _p(in16, _i16p), _i64(n), ctypes.c_int(C), _p(out, _i16p))
    del keep
    return out[:m]


def quantize(x_f32):
    """A.1 ffmpeg f32 -> s16 (mono duplicated to stereo, :190)."""
    x = np.ascontiguousarray(x_f32, np.float32)
    if x.ndim == 1:
        x = x.reshape(-1, 1)
    if x.shape[1] > 2:                    # the file's own C channels, no duplication
        out = np.empty(x.shape, np.int16)
        lib().orc_quantize_flat(_p(x, _f32p), _i64(x.size), _p(out, _i16p))
        return out
    out = np.empty((x.shape[0], 2), np.int16)
    lib().orc_quantize(_p(x, _f32p), _i64(x.shape[0]), ctypes.c_int(x.shape[1]), _p(out, _i16p))
    return out


# ------------------------------------------------------ ffmpeg restatements
def ebur128(x16, fs):
    x16 = np.ascontiguousarray(x16, np.int16)
    ch = x16.shape[1]
    hist = np.zeros(1000, np.uint64)
    st_hist = np.zeros(1000, np.uint64)
    peak = np.zeros(ch, np.float64)
    nb = _i64(0)
    lib().orc_ebur128(_p(x16, _i16p), _i64(x16.shape[0]), ctypes.c_int(fs), ctypes.c_int(ch),
                      _p(hist, _u64p), _p(st_hist, _u64p), _p(peak, _f64p), ctypes.byref(nb))
    return hist, st_hist, peak, int(nb.value)


def ebur128_192k(x16, fs):
    """libebur128 over the track resampled to 192 kHz as ffmpeg's loudnorm pass 1
    does (amx_oracle.c orc_ebur128_192k)."""
    x16 = np.ascontiguousarray(x16, np.int16)
    ch = x16.shape[1]
    hist = np.zeros(1000, np.uint64)
    st_hist = np.zeros(1000, np.uint64)
    peak = np.zeros(ch, np.float64)
    nb = _i64(0)
    rc = lib().orc_ebur128_192k(_p(x16, _i16p), _i64(x16.shape[0]), ctypes.c_int(fs), ctypes.c_int(ch),
                                _p(hist, _u64p), _p(st_hist, _u64p), _p(peak, _f64p), ctypes.byref(nb))
    if rc != 0:
        raise ValueError("no 192 kHz resampler for %d Hz input" % fs)
    return hist, st_hist, peak, int(nb.value)


def swr_geometry(fs, out_rate=192000):
    L, M = ctypes.c_int(), ctypes.c_int()
    if lib().orc_swr_geometry(ctypes.c_int(fs), ctypes.c_int(out_rate), ctypes.byref(L), ctypes.byref(M)):
        raise ValueError("unsupported rate %d" % fs)
    return L.value, M.value


def swr_phases(fs, out_rate=192000):
    """the bank's phase count: L (exact rational) or 1024 (libswresample's default)"""
    pc = lib().orc_swr_phases(ctypes.c_int(fs), ctypes.c_int(out_rate))
    if pc < 0:
        raise ValueError("unsupported rate %d" % fs)
    return pc


def swr_incr(fs, out_rate=192000):
    a, b = ctypes.c_int64(), ctypes.c_int64()
    if lib().orc_swr_incr(ctypes.c_int(fs), ctypes.c_int(out_rate), ctypes.byref(a), ctypes.byref(b)):
        raise ValueError("unsupported rate %d" % fs)
    return a.value, b.value


def swr_filter(fs, out_rate=192000):
    """resample_init's filter: (filter_length taps, filter_alloc row stride, factor)"""
    t, al, f = ctypes.c_int(), ctypes.c_int(), ctypes.c_double()
    if lib().orc_swr_filter(ctypes.c_int(fs), ctypes.c_int(out_rate), ctypes.byref(t), ctypes.byref(al),
                            ctypes.byref(f)):
        raise ValueError("unsupported rate %d" % fs)
    return t.value, al.value, f.value


def swr_bank(fs, out_rate=192000):
    """[phases][filter_alloc] float32 bank (zeros past filter_length)"""
    bank = np.zeros((swr_phases(fs, out_rate), swr_filter(fs, out_rate)[1]), np.float32)
    lib().orc_swr_bank(ctypes.c_int(fs), ctypes.c_int(out_rate), _p(bank, _f32p))
    return bank


def swr_table(fs, out_rate=192000):
    """one period (L outputs over M input frames) of the per-output base frame, phase
    row and interpolation weight; lin = the linear (interpolating) kernel runs"""
    L, _ = swr_geometry(fs, out_rate)
    ob = np.zeros(L, np.int32)
    ph = np.zeros(L, np.int32)
    wt = np.zeros(L, np.float32)
    lin = lib().orc_swr_table(ctypes.c_int(fs), ctypes.c_int(out_rate), _p(ob, ctypes.POINTER(ctypes.c_int32)),
                              _p(ph, ctypes.POINTER(ctypes.c_int32)), _p(wt, _f32p))
    return ob, ph, wt, bool(lin)


def upsample(x16, fs, out_rate=192000):
    """the 192 kHz float stream (as doubles) the pass-1 measurement sees"""
    x16 = np.ascontiguousarray(x16, np.int16)
    ch = x16.shape[1]
    n_out = int(lib().orc_swr_out_frames(_i64(x16.shape[0]), ctypes.c_int(fs), ctypes.c_int(out_rate)))
    out = np.zeros((max(n_out, 0), ch), np.float64)
    lib().orc_upsample(_p(x16, _i16p), _i64(x16.shape[0]), ctypes.c_int(ch), ctypes.c_int(fs),
                       ctypes.c_int(out_rate), _p(out, _f64p))
    return out


def ebur128_tables():
    e = np.zeros(1000, np.float64)
    b = np.zeros(1001, np.float64)
    lib().orc_ebur128_tables(_p(e, _f64p), _p(b, _f64p))
    return e, b


def kweight_coefs(fs):
    b = np.zeros(5)
    a = np.zeros(5)
    lib().orc_kweight_coefs(ctypes.c_int(fs), _p(b, _f64p), _p(a, _f64p))
    return b, a


def alimiter(x16, fs, level_in=1.0, level_out=1.0, limit=0.98, attack=5.0, release=50.0,
             auto_level=True):
    x16 = np.ascontiguousarray(x16, np.int16)
    out = np.empty_like(x16)
    lib().orc_alimiter(_p(x16, _i16p), _i64(x16.shape[0]), ctypes.c_int(fs),
                       ctypes.c_int(x16.shape[1]), ctypes.c_double(level_in),
                       ctypes.c_double(level_out), ctypes.c_double(limit),
                       ctypes.c_double(attack), ctypes.c_double(release),
                       ctypes.c_int(1 if auto_level else 0), _p(out, _i16p))
    return out


def linear_gain(x16, gain):
    x16 = np.ascontiguousarray(x16, np.int16)
    out = np.empty_like(x16)
    lib().orc_linear_gain(_p(x16, _i16p), _i64(x16.size), ctypes.c_double(gain), _p(out, _i16p))
    return out


def loudness_stats(hist, st_hist):
    out = np.zeros(3, np.float64)
    h = np.ascontiguousarray(hist, np.uint64)
    s = np.ascontiguousarray(st_hist, np.uint64)
    lib().orc_loudness_stats(_p(h, _u64p), _p(s, _u64p), _p(out, _f64p))
    return float(out[0]), float(out[1]), float(out[2])


def loudnorm_measure(x16, fs, native=False):
    """pass-1 JSON 'input_*' strings: ffmpeg measures the track resampled to 192 kHz
    (amx_oracle.c orc_ebur128_192k); native=True measures at the track's own rate."""
    hist, st, peak, _ = ebur128(x16, fs) if native else ebur128_192k(x16, fs)
    I, lra, thr = loudness_stats(hist, st)
    tp = float(peak.max()) if peak.size else 0.0
    tp_db = 20.0 * np.log10(tp) if tp > 0 else -np.inf
    f = lambda v: "%.2f" % v
    return {"input_i": f(I), "input_tp": f(tp_db), "input_lra": f(lra), "input_thresh": f(thr)}


def loudnorm_linear_gain(stats, target_i, target_tp=-1.5, target_lra=11.0):
    if stats["input_i"] == "-inf":
        return "skip", None
    mi, mtp = float(stats["input_i"]), float(stats["input_tp"])
    mlra, mth = float(stats["input_lra"]), float(stats["input_thresh"])
    off = target_i - mi
    if mtp != 99 and mth != -70 and mlra != 0 and mi != 0:
        if mtp + off <= target_tp and mlra <= target_lra:
            return "linear", 10.0 ** (off / 20.0)
    return "dynamic", None


class _LoudnormOpts(ctypes.Structure):
    _fields_ = [(k, ctypes.c_double) for k in ("target_i", "target_lra", "target_tp", "measured_i",
                                                 "measured_lra", "measured_tp", "measured_thresh",
                                                 "offset")]


def loudnorm(x16, fs, target_i, target_tp=-1.5, target_lra=11.0, measured=None, offset=0.0):
    """af_loudnorm at 192 kHz over an s16 track (amx_oracle.c orc_loudnorm): the
    dynamic mode (or the < 3 s linear fallback).  measured: dict of the pass-1 strings
    (input_i, input_lra, input_tp, input_thresh) or None (pass 1's defaults).  Returns
    (s16 output at 192 kHz, summary dict of ffmpeg's print_format=json strings)."""
    x16 = np.ascontiguousarray(x16, np.int16)
    ch = x16.shape[1]
    o = _LoudnormOpts(target_i, target_lra, target_tp, 0.0, 0.0, 99.0, -70.0, offset)
    if measured is not None:
        o.measured_i = float(measured["input_i"])
        o.measured_lra = float(measured["input_lra"])
        o.measured_tp = float(measured["input_tp"])
        o.measured_thresh = float(measured["input_thresh"])
    n_out = int(lib().orc_swr_out_frames(_i64(x16.shape[0]), ctypes.c_int(fs), ctypes.c_int(192000)))
    if n_out < 0:
        raise ValueError("no 192 kHz resampler for %d Hz input" % fs)
    out = np.zeros((max(n_out, 1), ch), np.int16)
    st = np.zeros(10, np.float64)
    f = lib().orc_loudnorm
    f.restype = ctypes.c_int64
    m = f(_p(x16, _i16p), _i64(x16.shape[0]), ctypes.c_int(fs), ctypes.c_int(ch), ctypes.byref(o),
          _p(out, _i16p), _p(st, _f64p))
    fmt = lambda v: "%.2f" % v
    summary = {"input_i": fmt(st[0]), "input_tp": fmt(st[1]), "input_lra": fmt(st[2]),
               "input_thresh": fmt(st[3]), "output_i": fmt(st[4]), "output_tp": "%+.2f" % st[5],
               "output_lra": fmt(st[6]), "output_thresh": "%+.2f" % st[7],
               "normalization_type": "linear" if st[8] else "dynamic", "target_offset": fmt(st[9])}
    return out[:m], summary


def loudnorm_pass1(x16, fs, target_i, target_tp=-1.5, target_lra=11.0):
    """pass 1 (:229) as ffmpeg prints it: the whole filter runs (dynamic mode) and
    target_offset is target_i minus its output's integrated loudness"""
    return loudnorm(x16, fs, target_i, target_tp, target_lra)[1]


def pipeline(x, fs, settings, chunks):
    """Whole process_audio_with_ffmpeg_pipeline (:171-226) on CPU.

    x: int16 [n, C] (already the ffmpeg s16 conversion) ; chunks: [(start, n)].
    Returns (int16 output [n', max(C, 2)], info dict).  C > 2: chunk_mc per chunk,
    libebur128's channel weights in the measurement, the C-channel alimiter."""
    x = np.asarray(x)
    if x.ndim == 1:
        x = x.reshape(-1, 1)
    if x.shape[1] == 1:
        x = np.repeat(x, 2, axis=1)
    C = x.shape[1]
    body = chunk if C == 2 else chunk_mc           # C > 2: the 1-D stream chain (:252)
    outs = [body(x[s:s + n], fs, settings) for s, n in chunks]
    cat = np.concatenate(outs, axis=0) if outs else np.zeros((0, C), np.int16)
    info = {"concat": cat}
    y = cat
    lufs = settings.get("lufs")
    out_fs = fs
    if lufs is not None:
        st = loudnorm_measure(cat, fs)
        mode, g = loudnorm_linear_gain(st, float(lufs))
        info.update(stats=st, mode=mode, gain=g)
        if mode == "linear":
            y = linear_gain(cat, g)
        elif mode == "dynamic":
            # pass 1's target_offset needs the whole filter run; pass 2 at 192 kHz
            p1 = loudnorm_pass1(cat, fs, float(lufs))
            y, _ = loudnorm(cat, fs, float(lufs), measured=st, offset=float(p1["target_offset"]))
            info.update(pass1=p1)
            out_fs = 192000
    info["normalized"] = y
    info["sample_rate"] = out_fs
    return alimiter(y, out_fs), info
