"""Drop-in replacement module for the reference's mastering entry points.

Mirrors audio_mastering_engine.py's call surface for the hot path:

* ``master_audio(settings, status_callback=None, progress_callback=None) -> str``
  -- the semantics of ``process_audio_with_ffmpeg_pipeline`` (:171-226): same
  ``settings`` keys and defaults, same status strings and progress sequence
  (``(0,100)``, ``(i+1, n+4)`` per chunk, ``n+1``, ``n+2`` only with ``lufs``,
  ``n+3``, ``n+4``), same ``ValueError`` for missing files, writes a 16-bit WAV.
* ``process_audio_with_ffmpeg_pipeline`` -- alias of ``master_audio``.
* ``process_audio(settings, status_cb, progress_cb, art_cb, tag_cb)`` -- the GUI
  wrapper (:94-137): mastering, the optional MP3 export (:97-98, ``export_to_mp3``
  :140-150, through an ``ffmpeg`` on PATH exactly as the reference calls it), and
  the AI/art branches out of scope: it reports
  ``"Success: Processing complete! (No art generated)"``, ``art_callback(None)``;
  on any error ``"Error: ..."``, ``progress(0, 1)``, ``art(None)``,
  ``tag("Processing failed.")`` exactly like :131-137.
* ``EQ_PRESETS`` (:32-38).

All per-sample work runs on the GPU (libamx.so via amx.engine): the host parses the
WAV container and moves the file's own bytes to the device; the s16 conversion of
ffmpeg's split (any PCM format, mono duplicated) is a kernel (amx_pcm_to_s16), and a
float32 file goes straight into the chain, whose first kernel quantises it.
"""
import logging
import os
import subprocess
import sys
import traceback

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import numpy as np  # noqa: E402

from amx import wavio  # noqa: E402
from amx.chunking import bounds_for  # noqa: E402
from amx.settings import EQ_PRESETS  # noqa: E402,F401

__all__ = ["master_audio", "process_audio", "process_audio_with_ffmpeg_pipeline", "EQ_PRESETS",
           "master_array", "export_to_mp3"]


def _noop(*a, **k):
    return None


def _device_input(path):
    """The input file on the device, as the chunk chain reads it: (d_in, fs, frames,
    channels_in, input_s16, WavInfo).  float32 stays float32 (the chain's first
    kernel quantises it, A.1); every other format is decoded to stereo s16 by
    amx_pcm_to_s16 (what ffmpeg's split writes + pydub's set_channels(2))."""
    import torch
    from amx import capi
    raw, info, code = wavio.read_audio_raw(path)          # WAV, AIFF / AIFF-C or FLAC
    if not 1 <= info.channels <= 8:
        raise ValueError("1 to 8 channels are supported (%d channels)" % info.channels)
    frames = raw.size // info.block_align
    d_raw = torch.from_numpy(raw.copy()).to("cuda")
    if code == "f32":
        return d_raw.view(torch.float32), info.sample_rate, frames, info.channels, False, info
    if info.channels > 2:
        # 3..8 channels: s16 [frames][C] as the split writes them (no duplication, :190)
        if code == "s16":
            return d_raw.view(torch.int16), info.sample_rate, frames, info.channels, True, info
        d_in = torch.empty((max(1, frames), info.channels), dtype=torch.int16, device="cuda")
        capi.check(capi.load().amx_pcm_to_s16(capi.ptr(d_raw), frames, info.channels,
                                              capi.PCM_FORMATS[code], capi.ptr(d_in),
                                              capi.ptr_stream()), "amx_pcm_to_s16")
        return d_in, info.sample_rate, frames, info.channels, True, info
    if code == "s16" and info.channels == 2:
        return d_raw.view(torch.int16), info.sample_rate, frames, 2, True, info
    d_in = torch.empty((max(1, frames), 2), dtype=torch.int16, device="cuda")
    capi.check(capi.load().amx_pcm_to_s16(capi.ptr(d_raw), frames, info.channels,
                                          capi.PCM_FORMATS[code], capi.ptr(d_in),
                                          capi.ptr_stream()), "amx_pcm_to_s16")
    return d_in, info.sample_rate, frames, 2, True, info


def _normalize(job):
    """normalize_loudness_on_disk_with_ffmpeg (:227-242) on the device: the rest of pass
    1's measurement, the statistics and decision; dynamic mode (:240 when the linear
    conditions fail) runs the 192 kHz path and returns its (output, info), linear
    mode (and the -inf skip, :238) returns None -- the gain rides in amx_finalize."""
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    report = job.fetch_report(raise_dynamic=False)
    mode = report["modes"][0] if report["modes"] else "off"
    if mode == "skip":
        logging.warning("Measured loudness is -inf (silent audio). Skipping normalization.")
    if mode == "dynamic":
        # loudnorm pass 2 in dynamic mode (:240): 192 kHz AGC + true-peak limiter
        return job.dynamic_track(0, report["stats"][0])
    return None


def master_audio(settings, status_callback=None, progress_callback=None):
    import torch
    from amx.engine import MasteringJob

    status = status_callback or _noop
    progress = progress_callback or _noop
    input_file, output_file = settings.get("input_file"), settings.get("output_file")
    if not input_file or not output_file:
        raise ValueError("Input or output file not specified.")              # :173
    status("Splitting audio into manageable chunks...")                       # :176
    progress(0, 100)                                                          # :177
    d_in, fs, frames, ch_in, s16, info = _device_input(input_file)
    bounds = bounds_for(frames, fs, info)                                     # :178
    status("Splitting complete.")                                             # :180
    num_chunks = len(bounds)
    total_steps = num_chunks + 4                                              # :184
    if ch_in > 2:
        return _master_multichannel(settings, status, progress, d_in, fs, frames, ch_in, s16, bounds,
                                    output_file)
    job = MasteringJob(fs, ch_in, settings, [frames], input_s16=s16,
                       chunks=[(0, s, n) for s, n in bounds])
    # every chunk's chain runs in the same launches (chunks are independent,
    # :185-204); the per-chunk callbacks fire while the device works on them and
    # "Re-assembling" fires once the chain is done
    if num_chunks:
        job.run_chunks(d_in)
    for i in range(num_chunks):
        status(f"Processing chunk {i+1} of {num_chunks}...")                  # :186
        progress(i + 1, total_steps)                                          # :187
    torch.cuda.current_stream().synchronize()
    status("Re-assembling processed chunks with concat filter...")           # :205
    progress(num_chunks + 1, total_steps)                                     # :206
    status("Concatenation complete.")                                         # :213
    # the sample peaks the limiter's path decision needs (and, with lufs, the first
    # half of loudnorm's 192 kHz measurement)
    job.loudness_pass1()
    dyn = None
    if settings.get("lufs") is not None:                                      # :216
        status("Normalizing final loudness...")                               # :217
        progress(num_chunks + 2, total_steps)                                 # :218
        try:
            dyn = _normalize(job)
        except Exception as e:                                                # :243-246
            # the reference logs any normalisation error and carries on with a copy of
            # the unnormalised track: here the track is finalised without the gain
            logging.exception("Error during disk-based normalization.")
            if isinstance(e, subprocess.CalledProcessError):
                logging.error(f"FFMPEG STDERR:\n{e.stderr}")
            dyn = None
            job.dd.lufs_on = 0
            job.decide()
    else:
        job.decide()
    status("Applying final limiting and exporting...")                        # :221
    progress(num_chunks + 3, total_steps)                                     # :222
    if dyn is None:
        job.finalize(None)
        y, out_fs = job.y[:job.info.out_frames].cpu().numpy(), fs
    else:
        # the alimiter ran on the 192 kHz file inside dynamic_track (:223 keeps its rate)
        y, out_fs = dyn[0].cpu().numpy(), dyn[1]["sample_rate"]
    wavio.write_wav_s16(output_file, y, out_fs)
    progress(total_steps, total_steps)                                        # :224
    logging.info(f"Finished GPU pipeline, exported to {output_file}")
    return output_file


def _master_multichannel(settings, status, progress, d_in, fs, frames, channels, s16, bounds, output_file):
    """master_audio for a file with 3..8 channels: the chain over the interleaved stream
    (:252), the measurement over the C channels and the C-channel alimiter
    (amx.engine.MultiChannelJob), with the same status strings and progress sequence.
    Loudnorm's dynamic mode is not run for such a file (DynamicModeUnsupported)."""
    import torch
    from amx.engine import MultiChannelJob
    num_chunks = len(bounds)
    total_steps = num_chunks + 4
    job = MultiChannelJob(fs, channels, settings, frames, input_s16=s16, chunks=[(0, s, n) for s, n in bounds])
    if num_chunks:
        job.run_chunks(d_in)
    for i in range(num_chunks):
        status(f"Processing chunk {i+1} of {num_chunks}...")                  # :186
        progress(i + 1, total_steps)                                          # :187
    torch.cuda.current_stream().synchronize()
    status("Re-assembling processed chunks with concat filter...")           # :205
    progress(num_chunks + 1, total_steps)                                     # :206
    status("Concatenation complete.")                                         # :213
    if settings.get("lufs") is not None:                                      # :216
        status("Normalizing final loudness...")                               # :217
        progress(num_chunks + 2, total_steps)                                 # :218
        job.measure(lufs_on=True)
        rep = job.fetch_report(raise_dynamic=True)
        if rep["modes"] and rep["modes"][0] == "skip":
            logging.warning("Measured loudness is -inf (silent audio). Skipping normalization.")
    else:
        job.measure(lufs_on=False)
    status("Applying final limiting and exporting...")                        # :221
    progress(num_chunks + 3, total_steps)                                     # :222
    y = job.finalize().cpu().numpy()
    wavio.write_wav_s16(output_file, y, fs)
    progress(total_steps, total_steps)                                        # :224
    logging.info(f"Finished GPU pipeline, exported to {output_file}")
    job.close()
    return output_file


process_audio_with_ffmpeg_pipeline = master_audio


def export_to_mp3(input_wav_path, status_callback):
    """:140-150 as the reference does it: the external ffmpeg encodes the mastered
    WAV to VBR MP3 (-q:a 0); a missing ffmpeg fails the same way (status
    "Error: Failed to create MP3 file.")."""
    if not input_wav_path or not os.path.exists(input_wav_path):
        logging.warning("Input WAV file not found for MP3 conversion.")
        status_callback("Warning: Could not find master WAV to create MP3.")
        return
    output_mp3_path = os.path.splitext(input_wav_path)[0] + ".mp3"
    status_callback("Creating high-quality MP3...")
    logging.info(f"Exporting WAV to MP3: {input_wav_path} -> {output_mp3_path}")
    try:
        mp3_command = ['ffmpeg', '-i', input_wav_path, '-q:a', '0', '-y', output_mp3_path]
        subprocess.run(mp3_command, check=True, capture_output=True, text=True)
        logging.info("MP3 export successful.")
        status_callback("High-quality MP3 created successfully.")
    except Exception:
        logging.exception("Error during MP3 export.")
        status_callback("Error: Failed to create MP3 file.")


def process_audio(settings, status_callback, progress_callback, art_callback, tag_callback):
    """:94-137 with the AI / art branches out of scope."""
    try:
        output_wav_path = master_audio(settings, status_callback, progress_callback)
        if settings.get("create_mp3", False):                                 # :97-98
            export_to_mp3(output_wav_path, status_callback)
        status_callback("Mastering complete. Preparing for AI analysis...")
        status_callback("Success: Processing complete! (No art generated)")
        art_callback(None)
    except Exception as e:
        logging.error(f"FATAL ERROR in process_audio: {traceback.format_exc()}")
        status_callback(f"Error: {e}")
        progress_callback(0, 1)
        art_callback(None)
        tag_callback("Processing failed.")


def master_array(x, sample_rate, settings, **kw):
    from amx.engine import master_array as _m
    return _m(x, sample_rate, settings, **kw)
