"""AIFF / AIFF-C reader (and a writer for tests): the GUI's file dialog offers *.aiff
beside *.wav (mastering_gui.py:170), and ffmpeg's split (audio_mastering_engine.py:178)
decodes it like any PCM input.  The host only parses the container; the file's own bytes
go to the device, where amx_pcm_to_s16 converts them (big-endian codes s16be ... f64be,
AIFF's signed 8-bit s8), as it does for WAV.

Container (Apple "Audio Interchange File Format" 1.3 / AIFF-C draft): "FORM" <size BE>
"AIFF" | "AIFC", then chunks <id> <size BE> <data, padded to even>:
  COMM: channels i16, sample frames u32, sample size i16, sample rate 80-bit IEEE
        extended; AIFF-C adds the compression type (4 bytes) and a Pascal-string name;
  SSND: offset u32, block size u32, then the samples from `offset`.
Sample formats (ffmpeg's aiffdec codec choice): AIFF and AIFF-C NONE / twos ->
big-endian signed PCM in ceil(bits / 8) bytes (left-justified); sowt -> little-endian
signed PCM; fl32 / fl64 -> big-endian IEEE float; raw -> unsigned 8-bit.
"""
import struct

import numpy as np

from .wavio import WavInfo


def _ext80(b):
    """80-bit IEEE 754 extended (big-endian) -> float"""
    exp = struct.unpack(">H", b[0:2])[0]
    mant = struct.unpack(">Q", b[2:10])[0]
    sign = -1.0 if exp & 0x8000 else 1.0
    exp &= 0x7FFF
    if exp == 0 and mant == 0:
        return 0.0
    return sign * mant * 2.0 ** (exp - 16383 - 63)


def _to_ext80(v):
    """positive integer sample rate -> 80-bit extended"""
    v = int(v)
    if v <= 0:
        return b"\x00" * 10
    shift = 63 - (v.bit_length() - 1)
    return struct.pack(">HQ", 16383 + 63 - shift, v << shift)


def is_aiff(path):
    with open(path, "rb") as f:
        h = f.read(12)
    return h[:4] == b"FORM" and h[8:12] in (b"AIFF", b"AIFC")


def _parse(path):
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"FORM" or data[8:12] not in (b"AIFF", b"AIFC"):
        raise ValueError("not an AIFF / AIFF-C file: %s" % path)
    aifc = data[8:12] == b"AIFC"
    pos, comm, ssnd = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack(">I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"COMM":
            ch, frames, bits = struct.unpack(">hIh", body[:8])
            fs = _ext80(body[8:18])
            comp = body[18:22] if aifc and len(body) >= 22 else b"NONE"
            comm = (ch, frames, bits, fs, comp)
        elif cid == b"SSND":
            off = struct.unpack(">I", body[:4])[0]
            ssnd = body[8 + off:]
        pos += 8 + size + (size & 1)
    if comm is None or ssnd is None:
        raise ValueError("AIFF without COMM/SSND chunk: %s" % path)
    ch, frames, bits, fs, comp = comm
    if ch <= 0 or bits <= 0:
        raise ValueError("AIFF with %d channels / %d-bit samples: %s" % (ch, bits, path))
    nbytes = (bits + 7) // 8
    if comp in (b"NONE", b"twos"):
        code = {1: "s8", 2: "s16be", 3: "s24be", 4: "s32be"}.get(nbytes)
    elif comp == b"sowt":
        code = {1: "s8", 2: "s16", 3: "s24", 4: "s32"}.get(nbytes)
    elif comp in (b"fl32", b"FL32"):
        code, nbytes = "f32be", 4
    elif comp in (b"fl64", b"FL64"):
        code, nbytes = "f64be", 8
    elif comp == b"raw ":
        code, nbytes = ("u8", 1) if nbytes == 1 else (None, nbytes)
    else:
        code = None
    if code is None:
        raise ValueError("unsupported AIFF-C compression %r / %d-bit samples" % (comp, bits))
    tag = 3 if code.startswith("f") else 1
    info = WavInfo(int(round(fs)), ch, tag, 8 * nbytes)
    n = min(frames, len(ssnd) // info.block_align)
    return info, code, ssnd[:n * info.block_align]


def read_aiff_raw(path):
    """(payload bytes as a uint8 array of whole frames, info, PCM code) -- the file's
    samples untouched, for the device decode (amx_pcm_to_s16)."""
    info, code, payload = _parse(path)
    return np.frombuffer(payload, np.uint8), info, code


def read_aiff_native(path):
    """(array [frames, channels], info) in the canonical sample types of wavio's reader:
    int16; int32 for 24 / 32 bits; float32 / float64; 8-bit as uint8 = v + 0x80 (what
    ffmpeg's pcm_s8 decoder produces), so wavio.to_s16 gives ffmpeg's s16 values."""
    info, code, raw = _parse(path)
    n = len(raw) // info.block_align
    if code in ("s16be", "s16"):
        x = np.frombuffer(raw, ">i2" if code == "s16be" else "<i2").astype(np.int16)
    elif code in ("s24be", "s24"):
        b = np.frombuffer(raw, "u1").reshape(-1, 3).astype(np.int32)
        v = (b[:, 0] << 16 | b[:, 1] << 8 | b[:, 2]) if code == "s24be" else (b[:, 2] << 16 | b[:, 1] << 8 | b[:, 0])
        x = np.where(v >= 1 << 23, v - (1 << 24), v).astype(np.int32)
    elif code in ("s32be", "s32"):
        x = np.frombuffer(raw, ">i4" if code == "s32be" else "<i4").astype(np.int32)
    elif code == "f32be":
        x = np.frombuffer(raw, ">f4").astype(np.float32)
    elif code == "f64be":
        x = np.frombuffer(raw, ">f8").astype(np.float64)
    elif code == "s8":
        x = (np.frombuffer(raw, "i1").astype(np.int16) + 128).astype(np.uint8)
    else:  # u8
        x = np.frombuffer(raw, "u1")
    return x.reshape(n, info.channels), info


def write_aiff(path, x, fs, code):
    """Test helper: x [frames, channels] (or [frames]) of native samples -> an AIFF
    (s8, s16be, s24be, s32be) or AIFF-C (f32be, f64be, sowt s16) file."""
    x = np.asarray(x)
    ch = 1 if x.ndim == 1 else x.shape[1]
    n = x.shape[0]
    comp = {"f32be": b"fl32", "f64be": b"fl64", "s16": b"sowt"}.get(code)
    bits = {"s8": 8, "s16be": 16, "s24be": 24, "s32be": 32, "f32be": 32, "f64be": 64, "s16": 16}[code]
    v = x.reshape(-1)
    if code == "s8":
        raw = v.astype(np.int8).tobytes()
    elif code == "s16be":
        raw = v.astype(">i2").tobytes()
    elif code == "s16":
        raw = v.astype("<i2").tobytes()
    elif code == "s24be":
        u = v.astype(np.int64) & 0xFFFFFF
        raw = np.stack([(u >> 16) & 255, (u >> 8) & 255, u & 255], axis=1).astype(np.uint8).tobytes()
    elif code == "s32be":
        raw = v.astype(">i4").tobytes()
    elif code == "f32be":
        raw = v.astype(">f4").tobytes()
    else:
        raw = v.astype(">f8").tobytes()
    comm = struct.pack(">hIh", ch, n, bits) + _to_ext80(fs)
    if comp is not None:
        name = b"\x00\x00"
        comm += comp + name
    ssnd = struct.pack(">II", 0, 0) + raw
    chunks = b""
    for cid, body in ((b"COMM", comm), (b"SSND", ssnd)):
        chunks += cid + struct.pack(">I", len(body)) + body + (b"\x00" if len(body) & 1 else b"")
    if comp is not None:
        chunks = b"FVER" + struct.pack(">II", 4, 0xA2805140) + chunks
    form = (b"AIFC" if comp is not None else b"AIFF") + chunks
    with open(path, "wb") as f:
        f.write(b"FORM" + struct.pack(">I", len(form)) + form)
