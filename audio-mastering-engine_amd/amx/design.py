"""Plan-time filter design: settings -> amx ChainDesc.

The coefficients are designed with exactly the calls the reference makes
(scipy.signal.butter, audio_mastering_engine.py:285, :296, :301-302), and the
analog-character waveshaper table with numpy's own float32 ``np.tanh`` (:263),
so the HIP kernels consume the reference's numbers bit for bit.  This is
O(1) host work per plan (a few dozen coefficients and one 65536-entry
transfer curve); every per-sample operation runs on the GPU.
"""
import numpy as np
from scipy.signal import butter

from . import capi
from .settings import LOW_CROSSOVER, HIGH_CROSSOVER


def shelf_ba(fs, cutoff_hz, btype):
    b, a = butter(2, cutoff_hz / (0.5 * fs), btype=btype)      # :285
    return np.asarray(b, np.float64), np.asarray(a, np.float64)


def peak_sos(fs, center_hz, q=1.41):
    nyquist = 0.5 * fs                                           # :292-296
    center_norm = center_hz / nyquist
    bandwidth = center_norm / q
    low, high = center_norm - (bandwidth / 2), center_norm + (bandwidth / 2)
    if low <= 0:
        low = 1e-9
    if high >= 1.0:
        high = 0.999999
    return np.asarray(butter(4, [low, high], btype='bandpass', output='sos'), np.float64)


def tanh_table(character_percent):
    """float32 tanh(float32(s/32768) * drive) for s = -32768..32767 (:258-263)."""
    cf = character_percent / 100.0
    drive = 1.0 + (cf * 0.5)
    s = np.arange(-32768, 32768, dtype=np.int16)
    x = s.astype(np.float32) / (2 ** 15)
    return np.ascontiguousarray(np.tanh(x * drive), dtype=np.float32), np.float32(drive)


def chain_desc(fs, channels_in, settings):
    """Returns (ChainDesc, keepalive) for one sample rate and settings dict."""
    d = capi.ChainDesc()
    keep = []
    d.sample_rate = int(fs)
    d.channels_in = int(channels_in)
    # compressor envelope work split (amx_dyn.hip); exact for any value -- the
    # underscore keys exist so the tests can force the fix-up paths
    d.env_warm_frames = int(settings.get("_env_warm", -1))
    d.env_rounds = int(settings.get("_env_rounds", -1))
    ac = settings.get("analog_character", 0)
    if ac > 0:                                                    # :192
        cf = ac / 100.0
        d.analog_on = 1
        lut, drive = tanh_table(ac)
        keep.append(lut)
        d.tanh_lut = lut.ctypes.data_as(capi.c_float_p)
        d.analog_drive = float(drive)
        blo, alo = shelf_ba(fs, 120, 'low')                        # :264
        bhi, ahi = shelf_ba(fs, 12000, 'high')                     # :265
        for k in range(3):
            d.analog_lo_ba[k], d.analog_lo_ba[3 + k] = blo[k], alo[k]
            d.analog_hi_ba[k], d.analog_hi_ba[3 + k] = bhi[k], ahi[k]
        d.analog_lo_gain = 10.0 ** ((cf * 1.0) / 20.0)             # :287
        d.analog_hi_gain = 10.0 ** ((cf * 1.5) / 20.0)
    stages = [("shelf", 250, settings.get("bass_boost", 0.0), 'low'),     # :278-281
              ("peak", 1000, -settings.get("mid_cut", 0.0), None),
              ("peak", 4000, settings.get("presence_boost", 0.0), None),
              ("shelf", 8000, settings.get("treble_boost", 0.0), 'high')]
    for i, (kind, fc, gdb, bt) in enumerate(stages):
        if gdb == 0:                                               # :284, :291
            continue
        d.eq_gain_db[i] = float(gdb)
        if kind == "shelf":
            d.eq_kind[i] = 1
            d.eq_gain[i] = 10.0 ** (gdb / 20.0)                    # :287
            b, a = shelf_ba(fs, fc, bt)
            for k in range(3):
                d.eq_coef[i][k], d.eq_coef[i][3 + k] = b[k], a[k]
        else:
            d.eq_kind[i] = 2
            d.eq_gain[i] = 10 ** (gdb / 20.0)                      # :297
            for k, v in enumerate(peak_sos(fs, fc).reshape(-1)):
                d.eq_coef[i][k] = v
    w = settings.get("width", 1.0)
    if w != 1.0:                                                   # :195
        d.width_on = 1
        d.width = float(np.float32(w))
    if settings.get("multiband"):                                  # :197
        d.multiband_on = 1
        lo = butter(4, LOW_CROSSOVER, btype='lowpass', fs=fs, output='sos')     # :301
        hi = butter(4, HIGH_CROSSOVER, btype='highpass', fs=fs, output='sos')   # :302
        for k, v in enumerate(np.asarray(lo, np.float64).reshape(-1)):
            d.xover_lo_sos[k] = v
        for k, v in enumerate(np.asarray(hi, np.float64).reshape(-1)):
            d.xover_hi_sos[k] = v
        for i, band in enumerate(("low", "mid", "high")):
            t, r = settings.get(band + "_thresh"), settings.get(band + "_ratio")
            if t is None or r is None:
                # the reference passes None into pydub, which fails on it (:306-308)
                raise TypeError("multiband requires %s_thresh and %s_ratio" % (band, band))
            d.comp_threshold_db[i] = float(t)
            d.comp_ratio[i] = float(r)
    return d, keep
