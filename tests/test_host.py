"""CPU: host logic of the product (design, chunk plan, WAV I/O, C-ABI exports,
drop-in call surface)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT


def test_libamx_builds_and_exports_every_header_symbol():
    import re
    from amx import build, capi
    build.build()
    lib = ctypes.CDLL(capi.LIB_PATH)
    with open(os.path.join(ROOT, "include", "amx.h")) as f:
        declared = set(re.findall(r"AMX_API\s+[\w\s\*]*?\b(amx_\w+)\s*\(", f.read()))
    assert declared == set(capi.EXPORTS), declared ^ set(capi.EXPORTS)
    for sym in declared:
        assert hasattr(lib, sym), sym
    L = capi.load()
    assert L.amx_abi_version() == capi.ABI_VERSION


def test_build_provenance_stamp(tmp_path):
    """the library carries the hash of the sources it was built from, and the binding
    refuses a library whose stamp is not this tree's"""
    import shutil
    from amx import build, capi
    build.build()
    assert capi.build_id() == build.source_hash() == build.built_hash()
    # a copy of the library loaded as the in-tree path after a source change would be
    # refused: simulate by comparing against a perturbed hash
    assert build.built_hash() != build.source_hash()[::-1]
    other = tmp_path / "libamx_other.so"
    shutil.copy(capi.LIB_PATH, other)
    assert build.built_hash(str(other)) == build.source_hash()


def test_struct_sizes_match_header():
    """ctypes mirrors of the ABI structs have the C sizes (compiled probe)."""
    import subprocess
    import tempfile
    from amx import capi
    src = r'''
#include <stdio.h>
#include "amx.h"
int main(){printf("%zu %zu %zu %zu %zu %zu %zu\n", sizeof(amx_chain_desc), sizeof(amx_chunk),
  sizeof(amx_final_desc), sizeof(amx_plan_info), sizeof(amx_track_span),
  sizeof(amx_decide_desc), sizeof(amx_loudnorm_desc));return 0;}'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        sizes = [int(v) for v in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    assert sizes == [ctypes.sizeof(capi.ChainDesc), ctypes.sizeof(capi.Chunk),
                     ctypes.sizeof(capi.FinalDesc), ctypes.sizeof(capi.PlanInfo),
                     ctypes.sizeof(capi.TrackSpan), ctypes.sizeof(capi.DecideDesc),
                     ctypes.sizeof(capi.LoudnormDesc)]


def test_design_uses_reference_coefficients():
    from scipy.signal import butter
    from amx import design
    s = dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0,
             analog_character=40.0, width=1.3, multiband=True, low_thresh=-25.0, low_ratio=6.0,
             mid_thresh=-20.0, mid_ratio=3.0, high_thresh=-15.0, high_ratio=4.0)
    d, keep = design.chain_desc(48000, 2, s)
    b, a = butter(2, 250 / 24000.0, btype='low')
    assert list(d.eq_coef[0])[:6] == list(b) + list(a)
    assert list(d.eq_kind) == [1, 2, 2, 1]
    assert d.eq_gain[1] == 10 ** (-2.0 / 20.0)
    lo = butter(4, 250, btype='lowpass', fs=48000, output='sos')
    assert list(d.xover_lo_sos) == list(lo.reshape(-1))
    assert d.width == np.float32(1.3) and d.analog_on == 1
    lut = np.ctypeslib.as_array(d.tanh_lut, shape=(65536,))
    x = np.arange(-32768, 32768, dtype=np.int16).astype(np.float32) / 32768
    np.testing.assert_array_equal(lut, np.tanh(x * (1.0 + 0.4 * 0.5)))
    d0, _ = design.chain_desc(48000, 2, dict())
    assert list(d0.eq_kind) == [0, 0, 0, 0] and d0.width_on == 0 and d0.multiband_on == 0
    with pytest.raises(TypeError):
        design.chain_desc(48000, 2, dict(multiband=True))


def test_chunk_bounds_follow_segment_rule():
    from amx.chunking import chunk_bounds, packet_frames
    fs = 48000
    q = packet_frames(8)
    assert q == 512
    n = fs * 301 + 77
    b = chunk_bounds(n, fs, q)
    assert sum(m for _, m in b) == n and b[0][0] == 0
    for k, (s, m) in enumerate(b[1:], start=1):
        assert s % q == 0 and s >= k * 30 * fs and s - q < k * 30 * fs
    assert len(b) == 11
    assert chunk_bounds(0, fs, q) == []
    assert chunk_bounds(100, fs, q) == [(0, 100)]


def test_wav_roundtrip_and_ffmpeg_s16_rules(tmp_path):
    from amx import wavio
    rng = np.random.default_rng(0)
    x16 = rng.integers(-32768, 32767, size=(1000, 2)).astype(np.int16)
    p = str(tmp_path / "a.wav")
    wavio.write_wav_s16(p, x16, 44100)
    nat, info = wavio.read_wav_native(p)
    assert info.sample_rate == 44100 and info.channels == 2 and info.bits == 16
    np.testing.assert_array_equal(wavio.to_s16(nat, info), x16)
    xf = rng.uniform(-1.2, 1.2, size=(500, 1)).astype(np.float32)
    p2 = str(tmp_path / "b.wav")
    wavio.write_wav_f32(p2, xf, 48000)
    nat2, info2 = wavio.read_wav_native(p2)
    exp = np.clip(np.rint(xf * np.float32(32768)), -32768, 32767).astype(np.int16)
    np.testing.assert_array_equal(wavio.to_s16(nat2, info2), exp)


def test_settings_presets():
    from amx.settings import EQ_PRESETS, apply_preset
    assert EQ_PRESETS["Vocal Clarity"] == {"bass_boost": -1.0, "mid_cut": 2.0,
                                           "presence_boost": 2.5, "treble_boost": 1.0}
    s = apply_preset({}, "Lo-Fi Haze")
    assert s["treble_boost"] == -4.0
    assert apply_preset(s, "None")["bass_boost"] == 0


def test_dropin_errors_like_reference(tmp_path):
    import audio_mastering_engine as ame
    with pytest.raises(ValueError, match="Input or output file not specified."):
        ame.master_audio({"input_file": None, "output_file": "x.wav"})
    msgs, prog, art, tag = [], [], [], []
    ame.process_audio({"input_file": "", "output_file": ""}, msgs.append,
                      lambda a, b: prog.append((a, b)), art.append, tag.append)
    assert msgs[-1] == "Error: Input or output file not specified."
    assert prog == [(0, 1)] and art == [None] and tag == ["Processing failed."]


def test_reciprocal_division_is_ieee_quotient(tmp_path):
    """The compressor kernels form m / A, m / R and -att / 20 as q = x (1/b) plus one
    FMA residual step (amx_dyn.hip env_div, gain_frame).  Markstein's theorem makes
    that the IEEE quotient for a correctly rounded 1/b; checked here on random and
    edge operands with the C library's fma (the plan additionally checks every
    compressor table value, amx_plan.cpp env_rcp)."""
    import ctypes
    import subprocess
    import numpy as np
    src = tmp_path / "mk.c"
    src.write_text(r'''
#include <math.h>
#include <stdint.h>
int64_t check(const double *x, int64_t n, double b) {
    const double y = 1.0 / b;
    int64_t bad = 0;
    for (int64_t i = 0; i < n; i++) {
        const double q = x[i] * y;
        const double c = fma(fma(-q, b, x[i]), y, q);
        if (c != x[i] / b) bad++;
    }
    return bad;
}
''')
    so = tmp_path / "mk.so"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-shared", "-fPIC", str(src), "-o", str(so), "-lm"],
                   check=True)
    lib = ctypes.CDLL(str(so))
    lib.check.restype = ctypes.c_int64
    lib.check.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_double]
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(0, 200, 1_000_000), rng.uniform(0, 1e-6, 100_000),
                        np.abs(rng.standard_normal(100_000)) * 30, -rng.uniform(0, 200, 100_000),
                        np.arange(0, 5000, 0.125)])
    x = np.ascontiguousarray(x, np.float64)
    for fs in (44100, 48000, 96000, 22050, 192000):
        for b in (5.0 * (fs / 1000.0), 50.0 * (fs / 1000.0)):
            assert lib.check(x.ctypes.data, x.size, b) == 0, (fs, b)
    assert lib.check(x.ctypes.data, x.size, 20.0) == 0


def test_rms_integer_form_matches_audioop():
    """k_rms forms audioop.rms's (unsigned) sqrt((double) S / cnt) as max{k : k^2 cnt <= S}
    from a float estimate plus one exact test (amx_dyn.hip rms_floor).  Check the identity
    and the estimate's +-1 correction on the worst cases: S at and one below k^2 cnt, for
    every window size the compressor uses (cnt = 2 * frames, 5 ms at 8 .. 192 kHz) and
    the head of a chunk (cnt = 2 .. 2 look)."""
    import math
    rng = np.random.default_rng(0)
    cnts = sorted({2 * i for i in range(1, 1025, 7)} | {80, 441 * 2, 480, 960, 2048})
    for cnt in cnts:
        ks = np.unique(np.concatenate([np.arange(0, 64), rng.integers(0, 32769, 200), [32767, 32768]]))
        for k in ks.tolist():
            for S in {k * k * cnt - 1, k * k * cnt, k * k * cnt + 1, (k + 1) * (k + 1) * cnt - 1}:
                if S < 0 or S > cnt * 2 ** 30:
                    continue
                ref = int(math.sqrt(S / cnt))
                assert max(0, math.isqrt(S // cnt)) == ref, (S, cnt)
                est = int(np.sqrt(np.float32(float(S) * (1.0 / cnt))))
                r = est + (1 if (est + 1) ** 2 * cnt <= S else 0)
                if not (est + 1) ** 2 * cnt <= S and est * est * cnt > S:
                    r = est - 1
                assert min(r, 32768) == ref, (S, cnt, est)


@pytest.mark.parametrize("code", ["s8", "s16be", "s24be", "s32be", "f32be", "f64be", "s16"])
@pytest.mark.parametrize("channels", [1, 2])
def test_aiff_reader(tmp_path, code, channels):
    """AIFF / AIFF-C (the GUI's *.aiff, mastering_gui.py:170): the parser's raw bytes,
    PCM code and sample rate, and its native decode, round-trip through the test writer;
    plain AIFF PCM is also read by the stdlib's independent aifc parser."""
    import warnings
    from amx import aiffio, capi, wavio
    rng = np.random.default_rng(3)
    n = 1001
    if code.startswith("f"):
        v = rng.uniform(-1.2, 1.2, (n, channels))
    else:
        bits = {"s8": 8, "s16be": 16, "s16": 16, "s24be": 24, "s32be": 32}[code]
        v = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), (n, channels))
    x = v if channels == 2 else v.reshape(-1)
    p = str(tmp_path / "x.aiff")
    aiffio.write_aiff(p, x, 44100, code)
    raw, info, c = wavio.read_audio_raw(p)
    assert c == code and c in capi.PCM_FORMATS and info.sample_rate == 44100 and info.channels == channels
    assert raw.size == n * info.block_align
    nat, info2 = wavio.read_audio_native(p)
    want = v.astype(np.float32 if code == "f32be" else np.float64) if code.startswith("f") else v
    if code == "s8":
        want = v + 128                                   # pcm_s8 decodes to u8 (v + 0x80)
    np.testing.assert_array_equal(nat, want.reshape(n, channels))
    # ffmpeg's s16 values: 8-bit v << 8, 24/32-bit >> 8 / >> 16, floats lrint(v 32768)
    s16 = wavio.to_s16(nat, info2)
    if code == "s8":
        np.testing.assert_array_equal(s16, (v << 8).reshape(n, channels))
    if code in ("s8", "s16be", "s24be", "s32be"):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", DeprecationWarning)
            import aifc
        with aifc.open(p, "rb") as f:
            assert (f.getnchannels(), f.getframerate(), f.getnframes()) == (channels, 44100, n)
            assert f.readframes(n) == raw.tobytes()


def test_aiff_ext80_rates():
    from amx import aiffio
    for fs in (8000, 22050, 44100, 48000, 88200, 96000, 192000):
        assert aiffio._ext80(aiffio._to_ext80(fs)) == fs


def test_pipelined_slots_keep_every_exchange_tensor():
    """r05f's hipErrorLaunchFailure: a slot's captured graph read gather indices that the
    other slot's _setup_exchange had replaced (and the allocator had reused).  Every
    attribute _setup_exchange assigns must be kept per slot (ShardedTrack._SLOT_KEYS)."""
    import ast
    import inspect
    import textwrap
    from amx.dist import ShardedTrack
    src = textwrap.dedent(inspect.getsource(ShardedTrack._setup_exchange))
    names = set()
    for node in ast.walk(ast.parse(src)):
        if isinstance(node, ast.Assign):
            for t in node.targets:
                if isinstance(t, ast.Attribute) and isinstance(t.value, ast.Name) and t.value.id == "self":
                    names.add(t.attr)
    names -= {"ne", "nl"}                 # plain ints, the same for both slots
    assert names, "no attributes found"
    missing = names - set(ShardedTrack._SLOT_KEYS)
    assert not missing, "exchange tensors not kept per slot: %s" % sorted(missing)
