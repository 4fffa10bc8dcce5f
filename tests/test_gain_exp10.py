"""The compressor's gain (pydub db_to_float(-att) = 10 ** (-att / 20), CPython's pow from
the platform libm, audio_mastering_engine.py:306-308 via compress_dynamic_range) is
formed on the GPU by ROCm's ocml exp10 sequence (amx_dyn.hip exp10_gain).  The two are
not the same function: the exp10 sequence is 1 ulp off glibc's pow on ~8 % of
attenuations.  What reaches the output is audioop.mul's floor(clip(v * f)) for an int16
sample v, and a 1-ulp change of f moves v * f by at most 2^-37 relative -- it changes the
floor only if v * f lies that close to an integer.  This test measures both: the share of
gains that differ, and that no int16 sample's output changes for any of them (every v in
-32768 .. 32767, for every differing gain of the sample).  DESIGN.md §4 cites it."""
import ctypes
import os
import subprocess
import tempfile

import numpy as np

C_SRC = r"""
#include <math.h>
#include <stdint.h>
/* exp10_gain of amx_dyn.hip with the plan's constants (ChainDev::exc), and the quotient
   -att / 20 as the device forms it (reciprocal multiply + one FMA residual step) */
static const double E[16] = {
    0x1.a934f0979a371p+1, -0x1.34413509f79ffp-2, 0x1.9dc1da994fd21p-59,
    -0x1.f48ad494ea3e9p-53, 0x1.26bb1bbb55516p+1, 0x1.ade156a5dcb37p-26,
    0x1.28af3fca7ab0cp-22, 0x1.71dee623fde64p-19, 0x1.a01997c89e6b0p-16,
    0x1.a01a014761f6ep-13, 0x1.6c16c1852b7b0p-10, 0x1.1111111122322p-7,
    0x1.55555555502a1p-5, 0x1.5555555555511p-3, 0x1.000000000000bp-1, 0.05};
static double exp10g(double x) {
    const double k = rint(x * E[0]);
    double r = fma(E[1], k, x);
    r = fma(E[2], k, r);
    double u = r * E[3];
    u = fma(E[4], r, u);
    double p = fma(E[5], u, E[6]);
    for (int i = 7; i < 15; i++) p = fma(u, p, E[i]);
    p = fma(u, p, 1.0);
    p = fma(u, p, 1.0);
    return ldexp(p, (int)k);
}
void gains(const double *att, int64_t n, double *dev, double *ref) {
    for (int64_t i = 0; i < n; i++) {
        const double q = -att[i] * E[15];
        const double x = fma(fma(-q, 20.0, -att[i]), E[15], q);
        dev[i] = exp10g(x);
        ref[i] = pow(10.0, (-att[i]) / 20.0);
    }
}
"""


def _lib():
    d = tempfile.mkdtemp()
    src, so = os.path.join(d, "g.c"), os.path.join(d, "g.so")
    with open(src, "w") as f:
        f.write(C_SRC)
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", src, "-o", so, "-lm"])
    L = ctypes.CDLL(so)
    dp = ctypes.POINTER(ctypes.c_double)
    L.gains.argtypes = [dp, ctypes.c_int64, dp, dp]
    return L


def test_exp10_gain_vs_libm_pow_never_changes_audioop_mul():
    L = _lib()
    rng = np.random.default_rng(7)
    att = np.concatenate([rng.uniform(0.0, 60.0, 150000), rng.uniform(0.0, 1.0, 50000),
                          np.array([0.0, -0.0, 5e-324, 1e-300, 1e-17, 2.0 ** -30]),
                          np.exp(rng.uniform(np.log(1e-12), np.log(3.0), 20000))])
    dev = np.empty_like(att)
    ref = np.empty_like(att)
    dp = ctypes.POINTER(ctypes.c_double)
    L.gains(att.ctypes.data_as(dp), att.size, dev.ctypes.data_as(dp), ref.ctypes.data_as(dp))
    # 0 <= f <= 1 for every attenuation >= 0: the clamp of audioop.mul never acts on an
    # int16 sample times f (amx_dyn.hip mul16 leaves it out)
    assert dev.min() >= 0.0 and dev.max() <= 1.0 and dev[att == 0.0].min() == 1.0
    diff = dev != ref
    ulps = np.abs(dev.view(np.int64) - ref.view(np.int64))
    assert ulps.max() <= 1
    share = diff.mean()
    assert 0.0 < share < 0.15, share
    v = np.arange(-32768, 32768, dtype=np.float64)

    def mul16(f):   # audioop.mul: clip then floor (CPython Modules/audioop.c fbound)
        return np.floor(np.clip(v * f, -32768.0, 32767.0))

    for a, b in zip(dev[diff], ref[diff]):
        assert np.array_equal(mul16(a), mul16(b)), (a, b)
