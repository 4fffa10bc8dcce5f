"""Envelope warm-up study (CPU, test infrastructure): how often a segment's speculative
start state -- the pydub attenuation recurrence run over W frames before the segment from
a guessed state -- equals the true state, for several guesses and W.  Bands of the
bench's synthetic programme (C3 settings), crossover + rms per frame as the compressor
sees them.

    python scripts/env_warm_sim.py --seconds 60 --fs 48000
"""
import argparse
import ctypes
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))

C_SRC = r"""
#include <math.h>
#include <stdint.h>
static inline double step(double att, double m, double A, double R) {
    double inc = m / A, dec = m / R;
    double up = fmin(att + inc, m), dn = fmax(att - dec, 0.0);
    return att <= m ? up : dn;
}
void truth(const double *m, int64_t n, double A, double R, double *att) {
    double a = 0.0;
    for (int64_t i = 0; i < n; i++) { att[i] = a; a = step(a, m[i], A, R); }
}
/* for each start s (state before frame s): run from guess g over [s - W, s) and
   report equality with truth; guess kind 0: 0, 1: m[s - W], 2: hull [0, M] merged */
void spec(const double *m, const double *att, int64_t n, double A, double R,
          const int64_t *starts, int ns, int W, int kind, double M, int *ok) {
    for (int k = 0; k < ns; k++) {
        int64_t s = starts[k], b = s - W < 0 ? 0 : s - W;
        double a = kind == 1 ? m[b] : 0.0, h = M;
        for (int64_t i = b; i < s; i++) {
            a = step(a, m[i], A, R);
            if (kind == 2) h = step(h, m[i], A, R);
        }
        if (s - W < 0) a = att[s];      /* chunk start: exact */
        ok[k] = kind == 2 ? (a == h && a == att[s]) : (a == att[s]);
    }
}
"""


def clib():
    d = tempfile.mkdtemp()
    src, so = os.path.join(d, "s.c"), os.path.join(d, "s.so")
    open(src, "w").write(C_SRC)
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", src, "-o", so, "-lm"])
    L = ctypes.CDLL(so)
    dp, ip = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)
    L.truth.argtypes = [dp, ctypes.c_int64, ctypes.c_double, ctypes.c_double, dp]
    L.spec.argtypes = [dp, dp, ctypes.c_int64, ctypes.c_double, ctypes.c_double, ip, ctypes.c_int,
                       ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_int)]
    return L


def band_m(b16, fs, thr_db, ratio):
    look = int(fs * 5 / 1000)
    x = b16.astype(np.int64)
    sq = (x * x).sum(axis=1)
    P = np.concatenate([[0], np.cumsum(sq)])
    i = np.arange(b16.shape[0])
    lo = np.maximum(i - look, 0)
    cnt = 2 * (i - lo)
    S = P[i] - P[lo]
    r = np.where(cnt > 0, np.floor(np.sqrt(S / np.maximum(cnt, 1))), 0.0)
    thr = 32768.0 * 10 ** (thr_db / 20.0)
    with np.errstate(divide="ignore"):
        db = np.where(r > 0, 20 * np.log10(np.maximum(r, 1e-300) / thr), 0.0)
    return (1 - 1 / ratio) * np.maximum(db, 0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--fs", type=int, default=48000)
    ap.add_argument("--le", type=int, default=1408)
    ap.add_argument("--seed", type=int, default=7)
    a = ap.parse_args()
    from oracle import oracle as orc
    from amx import synth
    fs = a.fs
    C3 = dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0, width=1.3,
              analog_character=40.0)
    x16 = orc.quantize(synth.mix_like(int(fs * a.seconds), fs, 2, seed=a.seed))
    an = orc.analog(x16, fs, C3["analog_character"])
    f = orc.eq(an.astype(np.float32) / np.float32(32768.0), fs, C3)
    p16 = orc.f32_to_s16(orc.width(f, np.float32(C3["width"])))
    bands = orc.crossover(p16, fs)
    L = clib()
    A, R = fs * 5 / 1000.0, fs * 50 / 1000.0
    dp = ctypes.POINTER(ctypes.c_double)
    for j, (t, rt) in enumerate([(-25.0, 6.0), (-20.0, 3.0), (-15.0, 4.0)]):
        m = np.ascontiguousarray(band_m(bands[j], fs, t, rt))
        n = m.size
        att = np.empty(n)
        L.truth(m.ctypes.data_as(dp), n, A, R, att.ctypes.data_as(dp))
        starts = np.arange(a.le, n, a.le, dtype=np.int64)
        M = float(m.max())
        line = "band %d (over threshold %.0f %%):" % (j, 100.0 * (m > 0).mean())
        for W in (256, 512, 768, 1024, 1536, 2048, 2304):
            res = []
            for kind in (0, 1, 2):
                ok = np.zeros(starts.size, np.int32)
                L.spec(m.ctypes.data_as(dp), att.ctypes.data_as(dp), n, A, R,
                       starts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), starts.size, W, kind, M,
                       ok.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
                res.append(100.0 * (1 - ok.mean()))
            line += "\n  W=%4d  wrong: from 0 %5.1f %%  from m %5.1f %%  hull not merged %5.1f %%" % (W, *res)
        print(line, flush=True)


if __name__ == "__main__":
    main()
