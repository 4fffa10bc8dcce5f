"""Chunk planner: the ffmpeg segment split of audio_mastering_engine.py:178.

``ffmpeg -i in -f segment -segment_time 30 chunk_%04d.wav`` cuts at the first
packet whose start time is >= k*30 s.  For a WAV input the demuxer delivers
packets of 4096 bytes (block-aligned), i.e. ``4096 // block_align`` frames, so
boundaries are ``ceil(k*30*fs / q) * q`` frames.  (ffmpeg is absent here: the
packet rule is restated from FFmpeg's wavdec.c/segment.c and is "unpinned";
callers can pass explicit boundaries.)  Chunks also define where the DSP state
restarts (:185-204), so the planner is part of the parity contract.
"""
import numpy as np

from .settings import SEGMENT_TIME_S


def packet_frames(block_align):
    q = max(1, 4096 // max(1, int(block_align)))
    return q


def chunk_bounds(n_frames, fs, quantum=512, segment_time=SEGMENT_TIME_S):
    """[(start, length), ...] for one track."""
    n = int(n_frames)
    if n <= 0:
        return []
    q = int(quantum)
    starts = [0]
    k = 1
    while True:
        cut = -(-(k * segment_time * int(fs)) // q) * q
        if cut >= n:
            break
        if cut > starts[-1]:
            starts.append(cut)
        k += 1
    ends = starts[1:] + [n]
    return [(s, e - s) for s, e in zip(starts, ends)]


def chunk_bounds_packets(n_frames, fs, packet_starts, segment_time=SEGMENT_TIME_S):
    """chunk_bounds for packets of varying length (a FLAC stream's frames): a chunk starts
    at the first packet whose start is at or after k * segment_time"""
    n = int(n_frames)
    if n <= 0:
        return []
    ps = np.asarray(packet_starts, np.int64)
    starts = [0]
    k = 1
    while True:
        t = k * segment_time * int(fs)
        i = int(np.searchsorted(ps, t, side="left"))
        if i >= len(ps) or ps[i] >= n:
            break
        if ps[i] > starts[-1]:
            starts.append(int(ps[i]))
        k += 1
    ends = starts[1:] + [n]
    return [(s, e - s) for s, e in zip(starts, ends)]


def bounds_for(n_frames, fs, info):
    """the split of :178 for an input file's WavInfo: packets of varying length when the
    reader found them (FLAC), else the PCM demuxer's 4096-byte packets"""
    ps = getattr(info, "packet_starts", None)
    if ps is not None:
        return chunk_bounds_packets(n_frames, fs, ps)
    return chunk_bounds(n_frames, fs, packet_frames(info.block_align))


def plan_tracks(track_frames, fs, quantum=512, segment_time=SEGMENT_TIME_S, explicit=None):
    """Chunks for tracks laid out back to back in one input buffer.

    Returns [(track, in_offset, frames)] ordered by track then time."""
    out, off = [], 0
    for t, n in enumerate(track_frames):
        bounds = explicit[t] if explicit is not None else chunk_bounds(n, fs, quantum, segment_time)
        for s, ln in bounds:
            out.append((t, off + s, ln))
        off += int(n)
    return out


def to_s16_ffmpeg(x, wav_info=None):
    """What ffmpeg's f32/f64/PCM -> s16 conversion gives (libswresample).

    float32/float64: av_clip_int16(lrint(x * 32768)); int PCM: shifts (exact)."""
    x = np.asarray(x)
    if x.dtype == np.int16:
        return x
    if x.dtype == np.float64:
        return np.clip(np.rint(x * 32768.0), -32768, 32767).astype(np.int16)
    y = np.rint(x.astype(np.float32) * np.float32(32768.0))
    return np.clip(y, -32768, 32767).astype(np.int16)
