"""Seeded synthetic "music-like" test signals.

Used by the benchmark, the tests and the golden-vector generator; no network, no
datasets.  Stereo float32 frames ``[n, C]`` built from 8 sines (log-uniform
40 Hz - 12 kHz, random phases), 1/f noise and a 0.5-4 Hz amplitude envelope so
that the compressor's RMS detector crosses its thresholds in both directions.
"""
import numpy as np

SEED_BASE = 20250912


def music_like(n_frames, sample_rate, channels=2, seed=0, peak_dbfs=-6.0,
               env_depth=0.85):
    rng = np.random.default_rng(SEED_BASE + int(seed))
    n = int(n_frames)
    out = np.zeros((n, channels), dtype=np.float64)
    if n == 0:
        return out.astype(np.float32)
    t = np.arange(n, dtype=np.float64) / float(sample_rate)
    nyq = 0.45 * sample_rate
    freqs = np.exp(rng.uniform(np.log(40.0), np.log(min(12000.0, nyq)), size=8))
    amps = rng.uniform(0.2, 1.0, size=8) / np.sqrt(np.arange(1, 9))
    env_f = rng.uniform(0.5, 4.0, size=2)
    env_p = rng.uniform(0, 2 * np.pi, size=2)
    env = 1.0 - env_depth * 0.5 * (1.0 + np.sin(2 * np.pi * env_f[0] * t + env_p[0]))
    env *= 0.75 + 0.25 * np.sin(2 * np.pi * env_f[1] * t + env_p[1])
    for c in range(channels):
        sig = np.zeros(n)
        for k in range(8):
            ph = rng.uniform(0, 2 * np.pi)
            sig += amps[k] * np.sin(2 * np.pi * freqs[k] * t + ph)
        # 1/f noise by spectral shaping of white noise
        w = rng.standard_normal(n)
        spec = np.fft.rfft(w)
        f = np.fft.rfftfreq(n, 1.0 / sample_rate)
        f[0] = f[1] if len(f) > 1 else 1.0
        spec /= np.sqrt(f)
        pink = np.fft.irfft(spec, n)
        pink /= (np.abs(pink).max() + 1e-12)
        out[:, c] = sig + 0.6 * pink
    out *= env[:, None]
    peak = np.abs(out).max()
    if peak > 0:
        out *= (10.0 ** (peak_dbfs / 20.0)) / peak
    return out.astype(np.float32)


def square(n_frames, sample_rate, channels=2, freq=220.0, amp=1.0):
    t = np.arange(int(n_frames)) / float(sample_rate)
    s = np.where(np.sin(2 * np.pi * freq * t) >= 0, amp, -amp)
    return np.repeat(s[:, None], channels, axis=1).astype(np.float32)


def sine(n_frames, sample_rate, channels=2, freq=997.0, dbfs=-20.0):
    t = np.arange(int(n_frames)) / float(sample_rate)
    s = (10.0 ** (dbfs / 20.0)) * np.sin(2 * np.pi * freq * t)
    return np.repeat(s[:, None], channels, axis=1).astype(np.float32)


def to_s16(x):
    """ffmpeg's f32 -> s16 conversion (libswresample): clip(lrintf(x*32768)).

    SURVEY.md Appendix A.1. ``np.rint`` rounds half to even like lrintf.
    """
    y = np.rint(np.asarray(x, dtype=np.float32) * np.float32(32768.0))
    return np.clip(y, -32768, 32767).astype(np.int16)


def mix_tiled(n_frames, sample_rate, channels=2, seed=0, block_seconds=60.0):
    """mix_like of one block_seconds block, repeated (each repeat circularly shifted by a
    seeded amount) to n_frames: the same kind of program at a fraction of the host time
    (mix_like costs ~1 s per 20 s of 48 kHz stereo), for long benchmark inputs."""
    n = int(n_frames)
    nb = min(n, int(block_seconds * sample_rate))
    if n == 0 or nb == n:
        return mix_like(n, sample_rate, channels, seed)
    blk = mix_like(nb, sample_rate, channels, seed)
    rng = np.random.default_rng(SEED_BASE + 2000 + int(seed))
    out = np.empty((n, channels), np.float32)
    for o in range(0, n, nb):
        k = min(nb, n - o)
        out[o:o + k] = np.roll(blk, int(rng.integers(0, nb)), axis=0)[:k]
    return out


def mix_like(n_frames, sample_rate, channels=2, seed=0, peak_dbfs=-3.0):
    """A "mixed" program signal with a modest peak-to-loudness ratio (~9-11 dB):
    a bass line of partials in 110-240 Hz, mid/high partials and 1/f noise, slow
    section-scale (9-14 s period, ~4 dB) and 0.2-0.6 Hz level changes.  After the reference's EQ presets it stays in
    loudnorm's linear mode at -14 LUFS (TP + offset <= -1.5 dBTP, LRA in (0, 11]),
    which is the mode the build implements."""
    rng = np.random.default_rng(SEED_BASE + 1000 + int(seed))
    n = int(n_frames)
    if n == 0:
        return np.zeros((0, channels), np.float32)
    t = np.arange(n, dtype=np.float64) / float(sample_rate)
    # section-scale level changes (LRA > 0) plus a faster 0.2-0.6 Hz swell
    env = 1.0 - 0.35 * 0.5 * (1.0 + np.sin(2 * np.pi * t / rng.uniform(9.0, 14.0) + rng.uniform(0, 6.3)))
    env *= 1.0 - 0.1 * 0.5 * (1.0 + np.sin(2 * np.pi * rng.uniform(0.2, 0.6) * t + rng.uniform(0, 6.3)))
    out = np.zeros((n, channels))
    bass = rng.uniform(110.0, 240.0, size=4)
    mids = np.exp(rng.uniform(np.log(400.0), np.log(min(9000.0, 0.45 * sample_rate)), size=5))
    for c in range(channels):
        sig = np.zeros(n)
        for f in bass:
            sig += rng.uniform(0.6, 1.0) * np.sin(2 * np.pi * f * t + rng.uniform(0, 6.3))
        for f in mids:
            sig += rng.uniform(0.1, 0.3) * np.sin(2 * np.pi * f * t + rng.uniform(0, 6.3))
        w = rng.standard_normal(n)
        spec = np.fft.rfft(w)
        fr = np.fft.rfftfreq(n, 1.0 / sample_rate)
        fr[0] = fr[1] if len(fr) > 1 else 1.0
        pink = np.fft.irfft(spec / np.sqrt(fr), n)
        pink /= (np.abs(pink).max() + 1e-12)
        out[:, c] = sig + 0.3 * pink
    out *= env[:, None]
    peak = np.abs(out).max()
    if peak > 0:
        out *= (10.0 ** (peak_dbfs / 20.0)) / peak
    return out.astype(np.float32)
