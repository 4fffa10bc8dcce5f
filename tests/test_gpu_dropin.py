"""The file-level drop-in on the GPU: master_audio / process_audio
(audio_mastering_engine.py:94-137, :171-226) from WAV files of every supported PCM
format, mono and stereo, with recording callbacks.  The status strings and the
progress sequence must be the reference's exactly, and the output WAV must equal
the oracle's pipeline on the s16 chunks ffmpeg's split would write, bit for bit."""
import os
import shutil
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MB = dict(multiband=True, low_thresh=-25.0, low_ratio=6.0, mid_thresh=-20.0, mid_ratio=3.0,
          high_thresh=-15.0, high_ratio=4.0)
C3 = dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0, lufs=-14.0,
          width=1.3, analog_character=40.0, **MB)


def _native(x, code):
    """float [-1, 1) signal -> the file's native samples for `code`."""
    if code in ("f32", "f64"):
        return x.astype(np.float32 if code == "f32" else np.float64)
    if code == "u8":
        return np.clip(np.round(x * 127.0) + 128, 0, 255).astype(np.uint8)
    if code == "s16":
        return np.clip(np.round(x * 32767.0), -32768, 32767).astype(np.int16)
    if code == "s24":
        return np.clip(np.round(x * 8388607.0), -8388608, 8388607).astype(np.int32)
    return np.clip(np.round(x.astype(np.float64) * 2147483647.0), -2147483648, 2147483647).astype(np.int32)


def _expected_calls(n_chunks, lufs):
    n = n_chunks
    st = ["Splitting audio into manageable chunks...", "Splitting complete."]
    st += ["Processing chunk %d of %d..." % (i + 1, n) for i in range(n)]
    st += ["Re-assembling processed chunks with concat filter...", "Concatenation complete."]
    if lufs:
        st += ["Normalizing final loudness..."]
    st += ["Applying final limiting and exporting..."]
    pr = [(0, 100)] + [(i + 1, n + 4) for i in range(n)] + [(n + 1, n + 4)]
    if lufs:
        pr += [(n + 2, n + 4)]
    pr += [(n + 3, n + 4), (n + 4, n + 4)]
    return st, pr


@pytest.mark.parametrize("code,channels,seconds,settings", [
    ("s16", 2, 64.0, C3), ("s16", 1, 31.0, dict(bass_boost=3.0, treble_boost=3.0)),
    ("s24", 2, 33.0, C3), ("s24", 1, 12.0, dict(C3, lufs=None)),
    ("f32", 2, 45.0, C3), ("f32", 1, 30.5, dict(bass_boost=-2.0, lufs=-16.0)),
    ("u8", 2, 6.0, dict(mid_cut=2.0)), ("s32", 2, 8.0, C3), ("f64", 1, 7.0, dict(C3, width=1.0)),
])
def test_master_audio_files(gpu, oracle_mod, code, channels, seconds, settings):
    import audio_mastering_engine as ame
    from amx import synth, wavio
    from amx.chunking import chunk_bounds, packet_frames
    fs = 44100 if code in ("s16",) and channels == 1 else 48000
    n = int(fs * seconds)
    x = synth.mix_like(n, fs, channels, seed=int(seconds * 7) + channels)
    if channels == 1:
        x = x.reshape(-1)
    nat = _native(x, code)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.wav"), os.path.join(d, "out.wav")
        wavio.write_wav_pcm(src, nat, fs, code)
        st, pr = [], []
        out = ame.master_audio(dict(settings, input_file=src, output_file=dst), st.append,
                               lambda a, b: pr.append((a, b)))
        assert out == dst
        y, info = wavio.read_wav_native(dst)
        # what ffmpeg's split writes (host restatement, test side only) + the oracle
        raw, winfo, _ = wavio.read_wav_raw(src)
        x16 = wavio.to_s16(wavio.read_wav_native(src)[0], winfo)
        bounds = chunk_bounds(n, fs, packet_frames(winfo.block_align))
    assert info.sample_rate == fs and info.bits == 16 and info.channels == 2
    want_st, want_pr = _expected_calls(len(bounds), settings.get("lufs") is not None)
    assert st == want_st
    assert pr == want_pr
    ref, _ = oracle_mod.pipeline(x16, fs, settings, bounds)
    assert y.shape == ref.shape
    d = np.abs(y.astype(np.int32) - ref.astype(np.int32))
    assert d.max() == 0, "max |diff| %d LSB" % d.max()


@pytest.mark.parametrize("fs", [22050, 11025])
@pytest.mark.parametrize("lufs", [None, -14.0])
def test_master_audio_rates_inexact_192k_resampler(gpu, oracle_mod, fs, lufs):
    """22.05 / 11.025 kHz: 192000 / gcd > 1024, so libswresample keeps 1024 phases and
    interpolates between them (resample_linear; restated in the oracle, parity unpinned
    against ffmpeg itself).  With lufs=-14 -- the GUI's default (mastering_gui.py:48) --
    the 192 kHz pass-1 measurement runs that resampler: the statistics strings equal the
    oracle's and the output is within 3 LSB of it (bit-exact so far); with lufs=None no
    loudnorm runs and the output is the oracle's bit for bit."""
    import audio_mastering_engine as ame
    from amx import synth, wavio
    from amx.chunking import chunk_bounds, packet_frames
    n = int(fs * 40.0)
    x = synth.mix_like(n, fs, 2, seed=fs)
    # (the analog stage's 12 kHz and the treble's 8 kHz shelves are past these rates'
    # Nyquist: scipy's butter raises in the reference as in amx.design)
    settings = dict(bass_boost=2.0, mid_cut=1.5, presence_boost=1.0, width=1.2, lufs=lufs, **MB)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.wav"), os.path.join(d, "out.wav")
        wavio.write_wav_pcm(src, _native(x, "s16"), fs, "s16")
        statuses = []
        out = ame.master_audio(dict(settings, input_file=src, output_file=dst), status_callback=statuses.append)
        assert out == dst
        y, info = wavio.read_wav_native(dst)
        raw, winfo, _ = wavio.read_wav_raw(src)
        x16 = wavio.to_s16(wavio.read_wav_native(src)[0], winfo)
        bounds = chunk_bounds(n, fs, packet_frames(winfo.block_align))
    ref, rinfo = oracle_mod.pipeline(x16, fs, settings, bounds)
    assert info.sample_rate == rinfo["sample_rate"]
    assert y.shape == ref.shape
    d = int(np.abs(y.astype(np.int32) - ref.astype(np.int32)).max())
    if lufs is None:
        assert d == 0
    else:
        from amx.engine import master_array
        assert rinfo["mode"] == "linear", rinfo["stats"]
        assert d <= 3, "max |diff| %d LSB" % d
        _, rep = master_array(np.ascontiguousarray(x16), fs, settings, quantum=packet_frames(winfo.block_align))
        assert rep["stats"][0] == rinfo["stats"], (rep["stats"][0], rinfo["stats"])


@pytest.mark.parametrize("stage", ["loudness_pass2", "histograms", "dynamic_track"])
def test_master_audio_normalization_failure_fallback(gpu, oracle_mod, monkeypatch, caplog, stage):
    """:243-246: any error inside the loudness normalisation is logged and the
    unnormalised track goes on to the alimiter -- the output equals the oracle's
    pipeline with lufs=None, and the status / progress sequence is the reference's
    (with the "Normalizing final loudness..." step, which ran and failed)."""
    import logging
    import audio_mastering_engine as ame
    from amx import capi, engine, synth, wavio
    from amx.chunking import chunk_bounds, packet_frames
    fs = 48000
    n = int(fs * 34.0)
    x = synth.mix_like(n, fs, 2, seed=34)
    if stage == "dynamic_track":
        # a quiet programme with full-scale bursts: loudnorm takes dynamic mode
        x = x * np.float32(0.12)
        rng = np.random.default_rng(3)
        for k in rng.integers(0, n - 200, 60):
            x[k:k + 50] += rng.uniform(-0.9, 0.9, (50, 2)).astype(np.float32)
        x = np.clip(x, -1.0, 1.0).astype(np.float32)

    def boom(*a, **k):
        raise capi.AmxError("injected failure in %s" % stage)
    monkeypatch.setattr(engine.MasteringJob, stage, boom)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.wav"), os.path.join(d, "out.wav")
        wavio.write_wav_f32(src, x, fs)
        st, pr = [], []
        with caplog.at_level(logging.ERROR):
            out = ame.master_audio(dict(C3, input_file=src, output_file=dst), st.append,
                                   lambda a, b: pr.append((a, b)))
        assert out == dst
        y, info = wavio.read_wav_native(dst)
        bounds = chunk_bounds(n, fs, packet_frames(8))
    assert "Error during disk-based normalization." in caplog.text
    want_st, want_pr = _expected_calls(len(bounds), True)
    assert st == want_st and pr == want_pr
    x16 = oracle_mod.quantize(x)
    if stage == "dynamic_track":
        _, rinfo = oracle_mod.pipeline(x16, fs, C3, bounds)
        assert rinfo["mode"] == "dynamic", rinfo.get("stats")
    ref, _ = oracle_mod.pipeline(x16, fs, dict(C3, lufs=None), bounds)
    assert info.sample_rate == fs
    assert y.shape == ref.shape
    dd = np.abs(y.astype(np.int32) - ref.astype(np.int32))
    assert dd.max() == 0, "max |diff| %d LSB" % dd.max()


def test_master_audio_192k_dynamic(gpu, oracle_mod):
    """a 192 kHz input that loudnorm sends to dynamic mode: ffmpeg inserts no resampler
    (only s16 -> dbl), the filter and the alimiter run at the input rate"""
    import audio_mastering_engine as ame
    from amx import synth, wavio
    from amx.chunking import chunk_bounds, packet_frames
    fs = 192000
    n = int(fs * 8.0)
    x = synth.mix_like(n, fs, 2, seed=19) * 0.12
    rng = np.random.default_rng(19)
    for k in rng.integers(0, n - 800, 16):
        x[k:k + 200] += rng.uniform(-0.9, 0.9, (200, 2))
    x = np.clip(x, -1.0, 1.0).astype(np.float32)
    settings = dict(bass_boost=1.0, lufs=-14.0)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.wav"), os.path.join(d, "out.wav")
        wavio.write_wav_f32(src, x, fs)
        ame.master_audio(dict(settings, input_file=src, output_file=dst))
        y, info = wavio.read_wav_native(dst)
        raw, winfo, _ = wavio.read_wav_raw(src)
        x16 = wavio.to_s16(wavio.read_wav_native(src)[0], winfo)
        bounds = chunk_bounds(n, fs, packet_frames(winfo.block_align))
    ref, rinfo = oracle_mod.pipeline(x16, fs, settings, bounds)
    assert rinfo["mode"] == "dynamic", rinfo.get("stats")
    assert info.sample_rate == 192000 == rinfo["sample_rate"]
    assert y.shape == ref.shape
    d = np.abs(y.astype(np.int32) - ref.astype(np.int32))
    print("192 kHz dynamic: max |diff| %d LSB, exact %.7f" % (d.max(), (d == 0).mean()))
    assert d.max() <= 3 and (d == 0).mean() >= 0.999


@pytest.mark.parametrize("code", ["u8", "s16", "s24", "s32", "f32", "f64"])
@pytest.mark.parametrize("channels", [1, 2])
def test_pcm_to_s16_decode(gpu, code, channels):
    """amx_pcm_to_s16 equals the host restatement of ffmpeg's conversions on every
    edge value (full scale, clipping floats, rounding ties, negative shifts)."""
    import torch
    from amx import capi, wavio
    rng = np.random.default_rng(5)
    n = 70001
    if code in ("f32", "f64"):
        edge = np.array([0.0, -0.0, 1.0, -1.0, 1.5, -1.5, 0.5 / 32768, 1.5 / 32768, -0.5 / 32768,
                         32767.5 / 32768, -32768.5 / 32768, 2.5 / 32768])
        v = np.concatenate([edge, rng.uniform(-1.2, 1.2, n * channels - edge.size)])
        v = v.astype(np.float32 if code == "f32" else np.float64)
    elif code == "u8":
        v = rng.integers(0, 256, n * channels).astype(np.uint8)
    elif code == "s16":
        v = rng.integers(-32768, 32768, n * channels).astype(np.int16)
    elif code == "s24":
        v = np.concatenate([[-8388608, 8388607, -1, 0, 255, -256],
                            rng.integers(-8388608, 8388608, n * channels - 6)]).astype(np.int32)
    else:
        v = np.concatenate([[-2147483648, 2147483647, -1, 0, 65535, -65536],
                            rng.integers(-2147483648, 2147483648, n * channels - 6)]).astype(np.int32)
    v = v.reshape(n, channels)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "x.wav")
        wavio.write_wav_pcm(p, v if channels == 2 else v.reshape(-1), 48000, code)
        raw, info, c = wavio.read_wav_raw(p)
        want = wavio.to_s16(wavio.read_wav_native(p)[0], info)
    if channels == 1:
        want = np.repeat(want.reshape(-1, 1), 2, axis=1)
    d_raw = torch.from_numpy(np.ascontiguousarray(raw)).cuda()
    out = torch.empty((n, 2), dtype=torch.int16, device="cuda")
    capi.check(capi.load().amx_pcm_to_s16(capi.ptr(d_raw), n, channels, capi.PCM_FORMATS[c],
                                          capi.ptr(out), capi.ptr_stream()), "amx_pcm_to_s16")
    np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_process_audio_callbacks_and_mp3(gpu):
    """process_audio (:94-137): success path with create_mp3 -- the external ffmpeg
    when the box has one, else the reference's own failure message -- and the
    error path's four callbacks."""
    import audio_mastering_engine as ame
    from amx import synth, wavio
    fs = 48000
    x = synth.mix_like(fs * 12, fs, 2, seed=9)     # long enough for a loudness range (linear mode)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.wav"), os.path.join(d, "out.wav")
        wavio.write_wav_f32(src, x, fs)
        st, pr, art, tag = [], [], [], []
        ame.process_audio(dict(C3, input_file=src, output_file=dst, create_mp3=True), st.append,
                          lambda a, b: pr.append((a, b)), art.append, tag.append)
        assert os.path.exists(dst)
        mp3 = ["Creating high-quality MP3..."]
        if shutil.which("ffmpeg"):
            mp3.append("High-quality MP3 created successfully.")
            assert os.path.exists(os.path.join(d, "out.mp3"))
        else:
            mp3.append("Error: Failed to create MP3 file.")
        k = st.index("Applying final limiting and exporting...")
        assert st[k + 1:] == mp3 + ["Mastering complete. Preparing for AI analysis...",
                                    "Success: Processing complete! (No art generated)"]
        assert art == [None] and tag == []
        # error path: a missing input file
        st, pr, art, tag = [], [], [], []
        ame.process_audio(dict(input_file=os.path.join(d, "nope.wav"), output_file=dst), st.append,
                          lambda a, b: pr.append((a, b)), art.append, tag.append)
        assert st[-1].startswith("Error: ") and pr[-1] == (0, 1)
        assert art == [None] and tag == ["Processing failed."]


def _native_aiff(x, code):
    if code.startswith("f"):
        return x.astype(np.float32 if code == "f32be" else np.float64)
    bits = {"s8": 8, "s16be": 16, "s16": 16, "s24be": 24, "s32be": 32}[code]
    m = float((1 << (bits - 1)) - 1)
    return np.clip(np.round(x.astype(np.float64) * m), -m - 1, m).astype(np.int64)


@pytest.mark.parametrize("code", ["s8", "s16be", "s24be", "s32be", "f32be", "f64be"])
@pytest.mark.parametrize("channels", [1, 2])
def test_pcm_to_s16_decode_aiff(gpu, code, channels):
    """the big-endian / signed-8-bit codes of amx_pcm_to_s16 on AIFF payloads equal the
    host restatement of ffmpeg's conversions, edge values included"""
    import torch
    from amx import aiffio, capi, wavio
    rng = np.random.default_rng(6)
    n = 50003
    if code.startswith("f"):
        edge = np.array([0.0, -0.0, 1.0, -1.0, 1.5, -1.5, 0.5 / 32768, 1.5 / 32768, -0.5 / 32768,
                         32767.5 / 32768, -32768.5 / 32768, 2.5 / 32768])
        v = np.concatenate([edge, rng.uniform(-1.2, 1.2, n * channels - edge.size)])
    else:
        bits = {"s8": 8, "s16be": 16, "s24be": 24, "s32be": 32}[code]
        lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
        v = np.concatenate([[lo, hi, -1, 0, 1], rng.integers(lo, hi + 1, n * channels - 5)])
    v = v.reshape(n, channels)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "x.aiff")
        aiffio.write_aiff(p, v if channels == 2 else v.reshape(-1), 48000, code)
        raw, info, c = wavio.read_audio_raw(p)
        want = wavio.to_s16(wavio.read_audio_native(p)[0], info)
    assert c == code
    if channels == 1:
        want = np.repeat(want.reshape(-1, 1), 2, axis=1)
    d_raw = torch.from_numpy(np.ascontiguousarray(raw)).cuda()
    out = torch.empty((n, 2), dtype=torch.int16, device="cuda")
    capi.check(capi.load().amx_pcm_to_s16(capi.ptr(d_raw), n, channels, capi.PCM_FORMATS[c],
                                          capi.ptr(out), capi.ptr_stream()), "amx_pcm_to_s16")
    np.testing.assert_array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("code,channels,seconds,settings", [
    ("s16be", 2, 33.0, C3), ("s24be", 1, 12.0, dict(bass_boost=2.0, lufs=-16.0)),
    ("f32be", 2, 20.0, C3), ("s8", 2, 6.0, dict(mid_cut=2.0)), ("s16", 2, 9.0, dict(C3, lufs=None)),
])
def test_master_audio_aiff(gpu, oracle_mod, code, channels, seconds, settings):
    """master_audio from AIFF / AIFF-C files (the GUI's *.aiff): the reference's callbacks
    and the oracle's output on the s16 chunks ffmpeg's split would write, bit for bit"""
    import audio_mastering_engine as ame
    from amx import aiffio, synth, wavio
    from amx.chunking import chunk_bounds, packet_frames
    fs = 44100
    n = int(fs * seconds)
    x = synth.mix_like(n, fs, channels, seed=int(seconds * 3) + channels)
    nat = _native_aiff(x if channels == 2 else x.reshape(-1), code)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.aiff"), os.path.join(d, "out.wav")
        aiffio.write_aiff(src, nat, fs, code)
        st, pr = [], []
        out = ame.master_audio(dict(settings, input_file=src, output_file=dst), st.append,
                               lambda a, b: pr.append((a, b)))
        assert out == dst
        y, info = wavio.read_wav_native(dst)
        raw, ainfo, _ = wavio.read_audio_raw(src)
        x16 = wavio.to_s16(wavio.read_audio_native(src)[0], ainfo)
        if channels == 1:
            x16 = x16.reshape(-1)
        bounds = chunk_bounds(n, fs, packet_frames(ainfo.block_align))
    assert info.sample_rate == fs and info.bits == 16 and info.channels == 2
    want_st, want_pr = _expected_calls(len(bounds), settings.get("lufs") is not None)
    assert st == want_st and pr == want_pr
    ref, _ = oracle_mod.pipeline(x16, fs, settings, bounds)
    assert y.shape == ref.shape
    d = np.abs(y.astype(np.int32) - ref.astype(np.int32))
    assert d.max() == 0, "max |diff| %d LSB" % d.max()


@pytest.mark.parametrize("bps,channels,seconds,variable,settings", [
    (16, 2, 31.0, False, C3), (24, 2, 12.0, True, dict(C3, lufs=None)), (16, 1, 8.0, True, dict(bass_boost=2.0)),
])
def test_master_audio_flac(gpu, oracle_mod, bps, channels, seconds, variable, settings):
    """master_audio from FLAC files (the GUI's *.flac): libamx's decoder, the device decode
    of its s32 samples, chunk cuts at the FLAC frames (the demuxer's packets); the
    reference's callbacks and the oracle's output on the s16 chunks ffmpeg would write,
    bit for bit"""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    import flac_enc
    import audio_mastering_engine as ame
    from amx import synth, wavio
    from amx.chunking import bounds_for
    fs = 44100
    n = int(fs * seconds)
    x = synth.mix_like(n, fs, channels, seed=int(seconds) + bps)
    hi = (1 << (bps - 1)) - 1
    nat = np.clip(np.round(np.asarray(x, np.float64).reshape(n, channels) * hi), -hi - 1, hi).astype(np.int64)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.flac"), os.path.join(d, "out.wav")
        with open(src, "wb") as f:
            f.write(flac_enc.encode(nat, fs, bps, seed=bps, variable=variable, kinds=["fixed2", "lpc", "verbatim"]))
        st, pr = [], []
        out = ame.master_audio(dict(settings, input_file=src, output_file=dst), st.append,
                               lambda a, b: pr.append((a, b)))
        assert out == dst
        y, info = wavio.read_wav_native(dst)
        xn, finfo = wavio.read_audio_native(src)
        x16 = wavio.to_s16(xn, finfo)
        if channels == 1:
            x16 = x16.reshape(-1)
        bounds = bounds_for(n, fs, finfo)
    assert np.array_equal(wavio.to_s16(xn, finfo).astype(np.int64).reshape(n, channels),
                          (nat << (16 - bps)) if bps <= 16 else (nat >> (bps - 16)))
    assert info.sample_rate == fs and info.bits == 16 and info.channels == 2
    want_st, want_pr = _expected_calls(len(bounds), settings.get("lufs") is not None)
    assert st == want_st and pr == want_pr
    ref, _ = oracle_mod.pipeline(x16, fs, settings, bounds)
    assert y.shape == ref.shape
    dd = np.abs(y.astype(np.int32) - ref.astype(np.int32))
    assert dd.max() == 0, "max |diff| %d LSB" % dd.max()


@pytest.mark.parametrize("fs", [384000, 352800])
@pytest.mark.parametrize("kind", ["mix", "dynamic"])
def test_master_audio_above_192k(gpu, oracle_mod, fs, kind):
    """inputs above 192 kHz with lufs=-14 (the GUI's default, mastering_gui.py:48): ffmpeg's
    loudnorm (:229, :240) resamples them DOWN to 192 kHz with libswresample's longer,
    narrower filter (66 taps at 384 kHz, 62 at 352.8 kHz; restated in the oracle, parity
    unpinned against ffmpeg itself).  Linear mode keeps the input rate; dynamic mode
    writes 192 kHz.  The statistics strings equal the oracle's and the output is within
    3 LSB of it (round 4 refused these rates with ERANGE)."""
    import audio_mastering_engine as ame
    from amx import synth, wavio
    from amx.chunking import chunk_bounds, packet_frames
    n = int(fs * 9.0)
    x = synth.mix_like(n, fs, 2, seed=fs % 1000)
    if kind == "dynamic":
        x = x * np.float32(0.12)
        rng = np.random.default_rng(fs % 997)
        for k in rng.integers(0, n - 2000, 18):
            x[k:k + 400] += rng.uniform(-0.9, 0.9, (400, 2)).astype(np.float32)
        x = np.clip(x, -1.0, 1.0).astype(np.float32)
    settings = dict(bass_boost=1.5, presence_boost=1.0, lufs=-14.0)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.wav"), os.path.join(d, "out.wav")
        wavio.write_wav_f32(src, x, fs)
        st = []
        ame.master_audio(dict(settings, input_file=src, output_file=dst), st.append)
        y, info = wavio.read_wav_native(dst)
        bounds = chunk_bounds(n, fs, packet_frames(8))
    assert "Error" not in " ".join(st)
    ref, rinfo = oracle_mod.pipeline(oracle_mod.quantize(x), fs, settings, bounds)
    assert rinfo["mode"] == ("dynamic" if kind == "dynamic" else "linear"), rinfo.get("stats")
    assert info.sample_rate == rinfo["sample_rate"] == (192000 if kind == "dynamic" else fs)
    assert y.shape == ref.shape
    dd = np.abs(y.astype(np.int32) - ref.astype(np.int32))
    print("%d Hz %s: max |diff| %d LSB, exact %.7f" % (fs, kind, dd.max(), (dd == 0).mean()))
    assert dd.max() <= 3 and (dd == 0).mean() >= 0.999
    from amx.engine import master_array
    _, rep = master_array(np.ascontiguousarray(oracle_mod.quantize(x)), fs, settings, quantum=packet_frames(8))
    assert rep["stats"][0] == rinfo["stats"], (rep["stats"][0], rinfo["stats"])
