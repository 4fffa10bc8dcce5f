"""FLAC input (the GUI's *.flac, mastering_gui.py:170; ffmpeg decodes it at :178).

The bitstream is decoded by libamx's host decoder (amx_flac_decode, csrc/amx_flac.cpp:
frames decoded on a thread pool) into int32 samples left-justified to 32 bits -- the
value ffmpeg's FLAC decoder hands on -- so the file reaches the device decode as s32
PCM (amx_pcm_to_s16: >> 16, what the segment muxer's s16 WAV chunks hold).
"""
import ctypes

import numpy as np

from . import capi
from .wavio import WavInfo


def _skip_id3(data):
    """offset past a leading ID3v2 tag (taggers prepend one; ffmpeg skips it)"""
    if len(data) >= 10 and data[:3] == b"ID3":
        size = ((data[6] & 0x7F) << 21) | ((data[7] & 0x7F) << 14) | ((data[8] & 0x7F) << 7) | (data[9] & 0x7F)
        off = 10 + size + (10 if data[5] & 0x10 else 0)
        return off
    return 0


def is_flac(path):
    with open(path, "rb") as f:
        head = f.read(4096)
    o = _skip_id3(head)
    if o + 4 > len(head):
        with open(path, "rb") as f:
            f.seek(o)
            return f.read(4) == b"fLaC"
    return head[o:o + 4] == b"fLaC"


# samples per byte a FLAC stream can reach at most: a frame of the largest block
# (65535 samples) is at least ~11 bytes (a 6-byte header + the 16-bit block size, one
# constant subframe of 2 bytes, the CRC-16), i.e. <= ~5958 samples per byte; a
# STREAMINFO length beyond 6144 per byte is not trusted for the allocation (a size
# query decides it first), so valid streams -- long silence included -- decode once
_MAX_SAMPLES_PER_BYTE = 6144


def decode_flac(data, threads=0, with_blocks=False):
    """(int32 array [frames, channels] left-justified to 32 bits, FlacInfo) of FLAC bytes;
    with_blocks: also the FLAC frames' block sizes in stream order (the demuxer's packets)"""
    # the decoder reads the caller's bytes in place (no copy): a numpy view of them
    raw = np.frombuffer(data, np.uint8)
    o = _skip_id3(raw[:10].tobytes())
    size = raw.size - o
    if size <= 0:
        raise capi.AmxError("not a FLAC stream (empty)")
    buf = ctypes.c_void_p(raw.ctypes.data + o)
    L = capi.load()
    info = capi.FlacInfo()
    rc = L.amx_flac_info(buf, size, ctypes.byref(info))
    if rc != capi.AMX_OK:
        raise capi.AmxError("not a FLAC stream (amx_flac_info %d)" % rc)
    n = ctypes.c_int64(info.total_frames)
    if n.value <= 0 or n.value > size * _MAX_SAMPLES_PER_BYTE:
        # STREAMINFO without the length, or one the file cannot hold: a size query first
        rc = L.amx_flac_decode(buf, size, None, 0, ctypes.byref(n), int(threads), None, 0, None)
        if rc != capi.AMX_OK:
            raise capi.AmxError("corrupt FLAC stream (amx_flac_decode %d)" % rc)
    out = np.empty((n.value, info.channels), np.int32)
    got = ctypes.c_int64(0)
    # frames of at least 16 samples (the format's minimum block size but the last)
    max_blocks = n.value // 16 + 2
    blocks = np.zeros(max_blocks, np.int32)
    nb = ctypes.c_int64(0)
    rc = L.amx_flac_decode(buf, size, out.ctypes.data_as(ctypes.c_void_p), n.value, ctypes.byref(got),
                           int(threads), blocks.ctypes.data_as(ctypes.c_void_p), max_blocks, ctypes.byref(nb))
    if rc != capi.AMX_OK or got.value != n.value:
        raise capi.AmxError("corrupt FLAC stream (amx_flac_decode %d)" % rc)
    if with_blocks:
        return out, info, blocks[:nb.value].copy()
    return out, info


def read_flac_native(path):
    """(int32 [frames, channels] left-justified samples, WavInfo of s32 PCM).  The WavInfo
    also carries packet_starts: the first sample of every FLAC frame, the packets the
    segment split cuts at (chunking.chunk_bounds_packets)"""
    with open(path, "rb") as f:
        x, info, blocks = decode_flac(f.read(), with_blocks=True)
    w = WavInfo(info.sample_rate, info.channels, 1, 32)
    w.packet_starts = np.concatenate([[0], np.cumsum(blocks.astype(np.int64))[:-1]])
    return x, w


def read_flac_raw(path):
    """read_wav_raw's triple for a FLAC file: the decoded samples as s32 PCM bytes (the
    WavInfo with packet_starts)"""
    x, fmt = read_flac_native(path)
    return np.ascontiguousarray(x).view(np.uint8).reshape(-1), fmt, "s32"
