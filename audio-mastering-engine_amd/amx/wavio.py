"""Minimal RIFF/WAVE reader/writer (PCM 8/16/24/32 and IEEE float 32/64).

Host I/O for master_audio(): the reference reads any format ffmpeg decodes and
writes 16-bit PCM (:178, :223); this build reads WAV, AIFF / AIFF-C (aiffio.py) and
FLAC (flacio.py) -- read_audio_raw -- and writes s16 WAV.
"""
import struct

import numpy as np


class WavInfo:
    def __init__(self, fs, channels, fmt_tag, bits):
        self.sample_rate, self.channels, self.fmt_tag, self.bits = fs, channels, fmt_tag, bits

    @property
    def block_align(self):
        return self.channels * self.bits // 8


PCM_CODE = {(1, 8): "u8", (1, 16): "s16", (1, 24): "s24", (1, 32): "s32", (3, 32): "f32", (3, 64): "f64"}


def _parse(path):
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE file: %s" % path)
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            tag, ch, fs, _, _, bits = struct.unpack("<HHIIHH", body[:16])
            if tag == 0xFFFE and len(body) >= 26:
                tag = struct.unpack("<H", body[24:26])[0]
            fmt = WavInfo(fs, ch, tag, bits)
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError("WAV without fmt/data chunk: %s" % path)
    if fmt.block_align <= 0:
        raise ValueError("WAV with a zero block size: %s" % path)
    return fmt, payload


def read_wav_raw(path):
    """(payload bytes as a uint8 array of whole frames, WavInfo, PCM code) -- the
    file's samples untouched, for the device decode (amx_pcm_to_s16)."""
    fmt, payload = _parse(path)
    code = PCM_CODE.get((fmt.fmt_tag, fmt.bits))
    if code is None:
        raise ValueError("unsupported WAV format tag %d / %d bits" % (fmt.fmt_tag, fmt.bits))
    n = len(payload) // fmt.block_align
    raw = np.frombuffer(payload, np.uint8, count=n * fmt.block_align)
    return raw, fmt, code


def read_audio_raw(path):
    """read_wav_raw for a WAV file, aiffio.read_aiff_raw for AIFF / AIFF-C,
    flacio.read_flac_raw for FLAC (the GUI's *.wav / *.aiff / *.flac inputs,
    mastering_gui.py:170)"""
    from . import aiffio, flacio
    if aiffio.is_aiff(path):
        return aiffio.read_aiff_raw(path)
    if flacio.is_flac(path):
        return flacio.read_flac_raw(path)
    return read_wav_raw(path)


def read_audio_native(path):
    """read_wav_native / aiffio.read_aiff_native / flacio.read_flac_native by the file's
    own header"""
    from . import aiffio, flacio
    if aiffio.is_aiff(path):
        return aiffio.read_aiff_native(path)
    if flacio.is_flac(path):
        return flacio.read_flac_native(path)
    return read_wav_native(path)


def read_wav_native(path):
    """Returns (array [frames, channels] in the file's own sample type, WavInfo).

    PCM 8 -> uint8, 16 -> int16, 24 -> int32 (sign-extended 24-bit value),
    32 -> int32; IEEE float -> float32/float64."""
    fmt, payload = _parse(path)
    n = len(payload) // fmt.block_align
    raw = payload[:n * fmt.block_align]
    if fmt.fmt_tag == 3:
        x = np.frombuffer(raw, dtype={32: "<f4", 64: "<f8"}[fmt.bits])
    elif fmt.fmt_tag == 1:
        if fmt.bits == 16:
            x = np.frombuffer(raw, "<i2")
        elif fmt.bits == 8:
            x = np.frombuffer(raw, "u1")
        elif fmt.bits == 24:
            b = np.frombuffer(raw, "u1").reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            x = np.where(v >= 1 << 23, v - (1 << 24), v).astype(np.int32)
        elif fmt.bits == 32:
            x = np.frombuffer(raw, "<i4")
        else:
            raise ValueError("unsupported PCM bit depth %d" % fmt.bits)
    else:
        raise ValueError("unsupported WAV format tag %d" % fmt.fmt_tag)
    return x.reshape(n, fmt.channels), fmt


def to_s16(x, fmt):
    """ffmpeg's conversion of the decoded samples to s16 for the segment WAVs (:178),
    libswresample audioconvert.c: u8 (v-0x80)<<8; s32 >>16 (24-bit PCM decodes to
    s32 = v<<8); float/double av_clip_int16(lrint(x*32768))."""
    if fmt.fmt_tag == 3:
        if x.dtype == np.float64:
            return np.clip(np.rint(x * 32768.0), -32768, 32767).astype(np.int16)
        y = np.rint(x.astype(np.float32) * np.float32(32768.0))
        return np.clip(y, -32768, 32767).astype(np.int16)
    if fmt.bits == 16:
        return x.astype(np.int16)
    if fmt.bits == 8:
        return ((x.astype(np.int32) - 0x80) << 8).astype(np.int16)
    if fmt.bits == 24:
        return ((x.astype(np.int64) << 8) >> 16).astype(np.int16)
    return (x.astype(np.int64) >> 16).astype(np.int16)


def read_wav(path):
    """Returns (float32 array [frames, channels], WavInfo)."""
    x, fmt = read_wav_native(path)
    if fmt.fmt_tag == 3:
        return x.astype(np.float32), fmt
    scale = {8: 128.0, 16: 32768.0, 24: float(1 << 23), 32: float(1 << 31)}[fmt.bits]
    off = 128.0 if fmt.bits == 8 else 0.0
    return ((x.astype(np.float64) - off) / scale).astype(np.float32), fmt


def write_wav_s16(path, x16, fs):
    x16 = np.ascontiguousarray(x16, dtype="<i2")
    ch = 1 if x16.ndim == 1 else x16.shape[1]
    raw = x16.tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(raw)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, ch, fs, fs * ch * 2, ch * 2, 16)
    hdr += b"data" + struct.pack("<I", len(raw))
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(raw)


def write_wav_f32(path, x, fs):
    x = np.ascontiguousarray(x, dtype="<f4")
    ch = 1 if x.ndim == 1 else x.shape[1]
    raw = x.tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(raw)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 3, ch, fs, fs * ch * 4, ch * 4, 32)
    hdr += b"data" + struct.pack("<I", len(raw))
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(raw)


def write_wav_pcm(path, x, fs, code):
    """Test helper: write x (float in [-1, 1] or the native integer samples) as a WAV
    of the given PCM code (u8 / s16 / s24 / s32 / f32 / f64)."""
    x = np.asarray(x)
    ch = 1 if x.ndim == 1 else x.shape[1]
    tag, bits = {"u8": (1, 8), "s16": (1, 16), "s24": (1, 24), "s32": (1, 32),
                 "f32": (3, 32), "f64": (3, 64)}[code]
    if code == "f32":
        raw = np.ascontiguousarray(x, "<f4").tobytes()
    elif code == "f64":
        raw = np.ascontiguousarray(x, "<f8").tobytes()
    elif code == "u8":
        raw = np.ascontiguousarray(x, "u1").tobytes()
    elif code == "s16":
        raw = np.ascontiguousarray(x, "<i2").tobytes()
    elif code == "s32":
        raw = np.ascontiguousarray(x, "<i4").tobytes()
    else:
        v = np.ascontiguousarray(x, np.int32).reshape(-1)
        b = np.empty((v.size, 3), np.uint8)
        b[:, 0] = v & 0xFF
        b[:, 1] = (v >> 8) & 0xFF
        b[:, 2] = (v >> 16) & 0xFF
        raw = b.tobytes()
    ba = ch * bits // 8
    hdr = b"RIFF" + struct.pack("<I", 36 + len(raw)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, tag, ch, fs, fs * ba, ba, bits)
    hdr += b"data" + struct.pack("<I", len(raw))
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(raw)
