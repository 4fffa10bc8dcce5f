"""Host arithmetic of ffmpeg's loudnorm measurement on GPU-made histograms.

The per-sample work (K-weighting, 400 ms gating blocks, 3 s short-term blocks,
sample peak) runs in libamx; what is left is O(1000) double arithmetic on the
histograms, restated here from FFmpeg's libavfilter/ebur128.c (a port of
libebur128) and af_loudnorm.c (normalize_loudness_on_disk_with_ffmpeg,
audio_mastering_engine.py:227-246).  Loop orders follow the C code so the
results are bit-identical for identical histograms.

PARITY: ffmpeg is not available in this image -- the loudnorm restatement is
"parity unpinned" beyond the EBU Tech 3341/3342 known answers (tests).  ffmpeg's
pass 1 measures at 192 kHz (dynamic mode resamples); this build measures at the
native rate, so ``measured_I`` may differ from ffmpeg's by a few 0.01 LU.
"""
import math

import numpy as np

RELATIVE_GATE_FACTOR = math.pow(10.0, -10.0 / 10.0)
MINUS_20DB = math.pow(10.0, -20.0 / 10.0)


def _tables():
    energies = [math.pow(10.0, (i / 10.0 - 69.95 + 0.691) / 10.0) for i in range(1000)]
    bounds = [math.pow(10.0, (-70.0 + 0.691) / 10.0)] + \
             [math.pow(10.0, (i / 10.0 - 70.0 + 0.691) / 10.0) for i in range(1, 1001)]
    return energies, bounds


HIST_ENERGIES, HIST_BOUNDS = _tables()


def find_histogram_index(energy):
    lo, hi = 0, 1000
    while True:
        mid = (lo + hi) // 2
        if energy >= HIST_BOUNDS[mid]:
            lo = mid
        else:
            hi = mid
        if hi - lo == 1:
            return lo


def energy_to_loudness(e):
    return 10 * math.log10(e) - 0.691 if e > 0 else -math.inf


def _nz(hist):
    """Indices of non-empty bins, ascending (adding an empty bin's 0.0 is exact,
    so summing only these keeps libebur128's sequential double sums bit-identical)."""
    return [int(j) for j in np.flatnonzero(np.asarray(hist))]


def relative_threshold_energy(hist):
    rel, count = 0.0, 0
    for j in _nz(hist):
        h = int(hist[j])
        rel += h * HIST_ENERGIES[j]
        count += h
    if count:
        rel /= float(count)
        rel *= RELATIVE_GATE_FACTOR
    return rel, count


def integrated_loudness(hist):
    """ebur128_gated_loudness (one state)."""
    rel, count = relative_threshold_energy(hist)
    if not count:
        return -math.inf
    if rel < HIST_BOUNDS[0]:
        start = 0
    else:
        start = find_histogram_index(rel)
        if rel > HIST_ENERGIES[start]:
            start += 1
    gated, above = 0.0, 0
    for j in _nz(hist):
        if j < start:
            continue
        h = int(hist[j])
        gated += h * HIST_ENERGIES[j]
        above += h
    if not above:
        return -math.inf
    gated /= float(above)
    return energy_to_loudness(gated)


def relative_threshold(hist):
    """ff_ebur128_relative_threshold -> LUFS (-70 when no block)."""
    rel, count = relative_threshold_energy(hist)
    if not count:
        return -70.0
    return energy_to_loudness(rel)


def loudness_range(st_hist):
    """ff_ebur128_loudness_range_multiple (one state)."""
    hist = [int(v) for v in st_hist]
    stl_size, stl_power = 0.0, 0.0
    for j in _nz(hist):
        stl_size += hist[j]
        stl_power += hist[j] * HIST_ENERGIES[j]
    if not stl_size:
        return 0.0
    stl_power /= stl_size
    stl_integrated = MINUS_20DB * stl_power
    if stl_integrated < HIST_BOUNDS[0]:
        index = 0
    else:
        index = find_histogram_index(stl_integrated)
        if stl_integrated > HIST_ENERGIES[index]:
            index += 1
    stl_size = 0
    for j in range(index, 1000):
        stl_size += hist[j]
    if not stl_size:
        return 0.0
    percentile_low = int((stl_size - 1) * 0.1 + 0.5)
    percentile_high = int((stl_size - 1) * 0.95 + 0.5)
    stl_size = 0
    j = index
    while stl_size <= percentile_low:
        stl_size += hist[j]
        j += 1
    l_en = HIST_ENERGIES[j - 1]
    while stl_size <= percentile_high:
        stl_size += hist[j]
        j += 1
    h_en = HIST_ENERGIES[j - 1]
    return energy_to_loudness(h_en) - energy_to_loudness(l_en)


def _fmt(v):
    return "%.2f" % v


def measure(hist, st_hist, peaks):
    """loudnorm pass-1 'input_*' statistics, as the JSON strings ffmpeg prints."""
    i_in = integrated_loudness(hist)
    lra_in = loudness_range(st_hist)
    thresh_in = relative_threshold(hist)
    tp_in = max(float(p) for p in peaks) if len(peaks) else 0.0
    tp_db = 20.0 * math.log10(tp_in) if tp_in > 0 else -math.inf
    return {"input_i": _fmt(i_in), "input_tp": _fmt(tp_db), "input_lra": _fmt(lra_in),
            "input_thresh": _fmt(thresh_in)}


def linear_gain(stats, target_i, target_tp=-1.5, target_lra=11.0):
    """af_loudnorm init(): pass-2 LINEAR mode decision on the measured strings.

    Returns (mode, gain): mode 'skip' (input_i == '-inf', :238), 'linear' with the
    gain 10**((I_t - I_meas)/20), or 'dynamic' (not yet supported)."""
    if stats["input_i"] == "-inf":
        return "skip", 1.0
    measured_i = float(stats["input_i"])
    measured_tp = float(stats["input_tp"])
    measured_lra = float(stats["input_lra"])
    measured_thresh = float(stats["input_thresh"])
    offset = target_i - measured_i
    offset_tp = measured_tp + offset
    if (measured_tp != 99 and measured_thresh != -70 and measured_lra != 0 and measured_i != 0):
        if offset_tp <= target_tp and measured_lra <= target_lra:
            return "linear", math.pow(10.0, offset / 20.0)
    return "dynamic", None


def max_after_gain(peak_abs_max, gain):
    """Conservative |sample| bound after the linear gain stage (llrint(x*g), clip)."""
    x16 = float(np.rint(peak_abs_max * 32768.0))
    if gain is None or gain <= 0:
        return x16 / 32768.0
    v = (x16 * (1.0 / 32768.0)) * gain
    return min(float(np.rint(v * 32768.0)), 32768.0) / 32768.0
