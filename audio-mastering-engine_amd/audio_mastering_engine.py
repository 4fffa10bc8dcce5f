"""Drop-in replacement module for the reference's mastering entry points.

Mirrors audio_mastering_engine.py's call surface for the hot path:

* ``master_audio(settings, status_callback=None, progress_callback=None) -> str``
  -- the semantics of ``process_audio_with_ffmpeg_pipeline`` (:171-226): same
  ``settings`` keys and defaults, same status strings and progress sequence
  (``(0,100)``, ``(i+1, n+4)`` per chunk, ``n+1``, ``n+2`` only with ``lufs``,
  ``n+3``, ``n+4``), same ``ValueError`` for missing files, writes a 16-bit WAV.
* ``process_audio_with_ffmpeg_pipeline`` -- alias of ``master_audio``.
* ``process_audio(settings, status_cb, progress_cb, art_cb, tag_cb)`` -- the GUI
  wrapper (:94-137) with the AI/art/MP3 branches out of scope: it reports
  ``"Success: Processing complete! (No art generated)"``, ``art_callback(None)``;
  on any error ``"Error: ..."``, ``progress(0, 1)``, ``art(None)``,
  ``tag("Processing failed.")`` exactly like :131-137.
* ``EQ_PRESETS`` (:32-38).

All DSP runs on the GPU (libamx.so via amx.engine); nothing here computes samples.
"""
import logging
import os
import sys
import traceback

_HERE = os.path.dirname(os.path.abspath(__file__))
if _HERE not in sys.path:
    sys.path.insert(0, _HERE)

import numpy as np  # noqa: E402

from amx import wavio  # noqa: E402
from amx.chunking import chunk_bounds, packet_frames  # noqa: E402
from amx.settings import EQ_PRESETS  # noqa: E402,F401

__all__ = ["master_audio", "process_audio", "process_audio_with_ffmpeg_pipeline", "EQ_PRESETS",
           "master_array"]


def _noop(*a, **k):
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
    native, info = wavio.read_wav_native(input_file)
    x16 = wavio.to_s16(native, info)                                          # ffmpeg -> s16 chunks
    fs = info.sample_rate
    bounds = chunk_bounds(x16.shape[0], fs, packet_frames(info.block_align))
    status("Splitting complete.")                                             # :180
    num_chunks = len(bounds)
    total_steps = num_chunks + 4                                              # :184
    d_in = torch.from_numpy(np.ascontiguousarray(x16)).to("cuda")
    job = MasteringJob(fs, x16.shape[1], settings, [x16.shape[0]], input_s16=True,
                       chunks=[(0, s, n) for s, n in bounds])
    for i in range(num_chunks):
        status(f"Processing chunk {i+1} of {num_chunks}...")                  # :186
        progress(i + 1, total_steps)                                          # :187
    job.run_chunks(d_in)
    status("Re-assembling processed chunks with concat filter...")           # :205
    progress(num_chunks + 1, total_steps)                                     # :206
    status("Concatenation complete.")                                         # :213
    job.loudness_pass1()
    if settings.get("lufs") is not None:                                      # :216
        status("Normalizing final loudness...")                               # :217
        progress(num_chunks + 2, total_steps)                                 # :218
        job.loudness_pass2(carry=False)
        job.histograms()
    job.decide()
    report = job.fetch_report()          # raises DynamicModeUnsupported before any output
    if report["modes"][0] == "skip":
        logging.warning("Measured loudness is -inf (silent audio). Skipping normalization.")
    status("Applying final limiting and exporting...")                        # :221
    progress(num_chunks + 3, total_steps)                                     # :222
    job.finalize(None)
    y = job.y[:job.info.out_frames].cpu().numpy()
    wavio.write_wav_s16(output_file, y, fs)
    progress(total_steps, total_steps)                                        # :224
    logging.info(f"Finished GPU pipeline, exported to {output_file}")
    return output_file


process_audio_with_ffmpeg_pipeline = master_audio


def process_audio(settings, status_callback, progress_callback, art_callback, tag_callback):
    """:94-137 with the MP3/AI/art branches out of scope."""
    try:
        master_audio(settings, status_callback, progress_callback)
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
