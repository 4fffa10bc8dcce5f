"""amx -- MI355X-native mastering DSP hot path (host side).

Public surface:
  amx.engine.MasteringJob / master_array   GPU pipeline over libamx.so
  amx.settings.EQ_PRESETS                  audio_mastering_engine.py:32-38
  audio_mastering_engine.master_audio      drop-in for process_audio_with_ffmpeg_pipeline
"""
__all__ = ["capi", "design", "engine", "loudness", "chunking", "settings", "wavio", "synth"]
