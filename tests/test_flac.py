"""FLAC input (the GUI's *.flac, mastering_gui.py:170): libamx's host decoder
(amx_flac_decode) against the round trip through the test-side encoder (flac_enc.py),
which writes every subframe type, residual coding, channel assignment and header form
of RFC 9639.  No FLAC files ship with the reference and no FLAC tool is installed, so
the round trip is the pin: decode(encode(x)) == x, bit for bit.  Then the samples the
device path sees: ffmpeg's s16 chunk values (s32 >> 16 of the left-justified samples)."""
import os
import tempfile

import numpy as np
import pytest

import flac_enc


def _signal(n, ch, bps, seed, kind="music"):
    rng = np.random.default_rng(seed)
    hi = (1 << (bps - 1)) - 1
    if kind == "noise":
        return rng.integers(-hi - 1, hi + 1, size=(n, ch), dtype=np.int64)
    t = np.arange(n) / 48000.0
    x = np.zeros((n, ch))
    for c in range(ch):
        f = 220.0 * (1 + c) * rng.uniform(0.9, 1.1)
        x[:, c] = 0.6 * np.sin(2 * np.pi * f * t) + 0.2 * np.sin(2 * np.pi * 3.1 * f * t)
        x[:, c] += 0.05 * rng.standard_normal(n)
    x[n // 3: n // 3 + 600] = 0.0                         # a silent stretch (constant subframes)
    v = np.clip(np.round(x * hi), -hi - 1, hi).astype(np.int64)
    return v


def _decode(data, threads=0):
    from amx import flacio
    return flacio.decode_flac(data, threads=threads)


@pytest.mark.parametrize("bps", [8, 12, 16, 20, 24])
@pytest.mark.parametrize("ch", [1, 2])
def test_round_trip_depths(bps, ch):
    x = _signal(20000 + 37 * bps, ch, bps, seed=bps * 10 + ch)
    data = flac_enc.encode(x, 48000, bps, seed=bps + ch)
    y, info = _decode(data)
    assert (info.sample_rate, info.channels, info.bits_per_sample) == (48000, ch, bps)
    assert info.total_frames == len(x)
    assert y.shape == x.shape
    assert np.array_equal(y.astype(np.int64) >> (32 - bps), x)
    assert np.all((y.astype(np.int64) & ((1 << (32 - bps)) - 1)) == 0)    # left-justified


@pytest.mark.parametrize("fs", [44100, 96000, 22050, 7350, 192000, 100000])
@pytest.mark.parametrize("variable", [False, True])
def test_round_trip_rates_and_blocking(fs, variable):
    x = _signal(30000, 2, 16, seed=fs % 97)
    for block in (192, 576, 1152, 4096):
        data = flac_enc.encode(x, fs, 16, seed=block + fs, block=block, variable=variable)
        y, info = _decode(data)
        assert info.sample_rate == fs
        assert np.array_equal(y.astype(np.int64) >> 16, x), (fs, variable, block)


@pytest.mark.parametrize("assign", [0, 8, 9, 10])
@pytest.mark.parametrize("kind", ["verbatim", "fixed0", "fixed1", "fixed2", "fixed3", "fixed4", "lpc"])
def test_each_subframe_kind_and_assignment(assign, kind):
    x = _signal(9000, 2, 16, seed=assign * 7 + len(kind))
    data = flac_enc.encode(x, 48000, 16, seed=assign, kinds=[kind], assigns=[assign], block=1152)
    y, _ = _decode(data)
    assert np.array_equal(y.astype(np.int64) >> 16, x)


def test_false_syncs_in_noise_and_threads():
    """full-scale noise in verbatim subframes puts many 0xFFF8 byte pairs (false frame
    syncs) inside frame data: the chain from the first frame must skip them, with any
    number of decoding threads"""
    x = _signal(120000, 2, 16, seed=5, kind="noise")
    data = flac_enc.encode(x, 48000, 16, seed=3, kinds=["verbatim", "fixed1"], block=4096)
    body = np.frombuffer(data, np.uint8)
    syncs = int(np.sum((body[:-1] == 0xFF) & ((body[1:] & 0xFE) == 0xF8)))
    assert syncs > len(x) // 4096 + 5
    for th in (1, 2, 8):
        y, _ = _decode(data, threads=th)
        assert np.array_equal(y.astype(np.int64) >> 16, x)


def test_corrupt_frame_and_not_flac():
    from amx import capi
    x = _signal(20000, 2, 16, seed=9)
    data = bytearray(flac_enc.encode(x, 48000, 16, seed=1, block=4096))
    data[len(data) // 2] ^= 0x10                            # a flipped bit: that frame's CRC-16 fails
    with pytest.raises(capi.AmxError):
        _decode(bytes(data))
    with pytest.raises(capi.AmxError):
        _decode(b"RIFF" + bytes(100))


def test_read_flac_files_and_s16(tmp_path):
    """the file readers: ID3v2-prefixed FLAC, read_audio_native / read_audio_raw, and the
    s16 values the chain gets: ffmpeg's s16 for depths <= 16 (sample << (16 - bps)),
    s32 >> 16 above (wavio.to_s16 of the left-justified samples)"""
    from amx import wavio
    for bps, code_ok in ((16, True), (24, True), (12, True)):
        x = _signal(15000, 2, bps, seed=bps)
        data = flac_enc.encode(x, 44100, bps, seed=bps)
        id3 = b"ID3\x04\x00\x00" + bytes([0, 0, 0, 20]) + bytes(20)
        p = os.path.join(str(tmp_path), "t%d.flac" % bps)
        with open(p, "wb") as f:
            f.write(id3 + data)
        y, fmt = wavio.read_audio_native(p)
        assert fmt.sample_rate == 44100 and fmt.bits == 32 and fmt.channels == 2
        s16 = wavio.to_s16(y, fmt)
        want = (x << (16 - bps)) if bps <= 16 else (x >> (bps - 16))
        assert np.array_equal(s16.astype(np.int64), want)
        raw, fmt2, code = wavio.read_audio_raw(p)
        assert code == "s32" and raw.size == x.size * 4
        assert np.array_equal(raw.view(np.int32).reshape(x.shape), y)


def test_chunk_bounds_follow_flac_packets():
    """the segment split cuts at the first packet starting at or after k x 30 s: FLAC
    frames are the packets (fixed blocking = the PCM rule with the block as quantum;
    variable blocking cuts at the variable frame starts)"""
    from amx.chunking import chunk_bounds, chunk_bounds_packets
    fs, n = 48000, 48000 * 95 + 123
    ps = np.arange(0, n, 4096)
    assert chunk_bounds_packets(n, fs, ps) == chunk_bounds(n, fs, 4096)
    rng = np.random.default_rng(1)
    sizes = rng.integers(16, 8192, size=4000)
    ps = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    ps = ps[ps < n]
    b = chunk_bounds_packets(n, fs, ps)
    assert b[0][0] == 0 and sum(ln for _, ln in b) == n
    for k, (s, _) in enumerate(b[1:], start=1):
        i = np.searchsorted(ps, k * 30 * fs)
        assert s == ps[i]


def test_read_flac_packet_starts(tmp_path):
    from amx import wavio
    x = _signal(48000 * 2, 2, 16, seed=3)
    data = flac_enc.encode(x, 48000, 16, seed=2, variable=True, block=1024)
    p = os.path.join(str(tmp_path), "v.flac")
    with open(p, "wb") as f:
        f.write(data)
    y, info = wavio.read_audio_native(p)
    assert info.packet_starts[0] == 0 and np.all(np.diff(info.packet_starts) >= 16)
    assert info.packet_starts[-1] < len(x)
