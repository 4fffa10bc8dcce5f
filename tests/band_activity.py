"""Compressor band activity on the bench programme (C3 settings, 40 s): the fraction of
frames whose RMS is above each band's threshold, and of 16-frame tiles with any such
frame -- the oracle's chain up to the crossover, numpy for the RMS."""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd")); sys.path.insert(0, ROOT)
import bench
from oracle import oracle as O
fs = 48000; n = fs * 40
x = bench.synth_input(n, fs, 0, "mix")
s = bench.C3
q = O.quantize(x)
a = O.analog(q, fs, s["analog_character"])
e = O.eq(a.astype(np.float32) / 32768.0, fs, s)
w = O.width(e, np.float32(s["width"]))
p16 = O.f32_to_s16(w)
bands = O.crossover(p16, fs)
look = 240
for b, name in enumerate(("low", "mid", "high")):
    v = bands[b].astype(np.int64)
    sq = (v[:, 0] ** 2 + v[:, 1] ** 2)
    P = np.concatenate([[0], np.cumsum(sq)])
    i = np.arange(n)
    lo = np.maximum(i - look, 0)
    S = P[i] - P[lo]
    cnt = 2 * (i - lo)
    r = np.floor(np.sqrt(np.where(cnt > 0, S / np.maximum(cnt, 1), 0)))
    thr = 32768 * 10 ** (s[name + "_thresh"] / 20)
    act = r > thr
    t16 = act[: n // 16 * 16].reshape(-1, 16).any(1)
    print(name, "thr %.0f" % thr, "frames active %.3f" % act.mean(), "16-tiles active %.3f" % t16.mean())
