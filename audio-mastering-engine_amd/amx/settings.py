"""Settings schema and constants of the reference's mastering path.

The ``settings`` dict is the API contract: the same keys
and defaults as the GUI (mastering_gui.py:119-130) and the engine
(audio_mastering_engine.py:172-223).
"""

# audio_mastering_engine.py:32-38
EQ_PRESETS = {
    "Vocal Clarity": {"bass_boost": -1.0, "mid_cut": 2.0, "presence_boost": 2.5, "treble_boost": 1.0},
    "Bass Punch": {"bass_boost": 2.5, "mid_cut": 1.0, "presence_boost": -1.0, "treble_boost": 0.5},
    "Vintage Warmth": {"bass_boost": 1.5, "mid_cut": 0.0, "presence_boost": -1.5, "treble_boost": -2.0},
    "Lo-Fi Haze": {"bass_boost": -2.0, "mid_cut": 3.0, "presence_boost": -2.0, "treble_boost": -4.0},
    "EDM Kick & Highs": {"bass_boost": 2.0, "mid_cut": 4.0, "presence_boost": 1.0, "treble_boost": 3.0},
}

# GUI defaults (mastering_gui.py:46-55)
GUI_DEFAULTS = {
    "analog_character": 0.0, "bass_boost": 0.0, "mid_cut": 0.0, "presence_boost": 0.0,
    "treble_boost": 0.0, "width": 1.0, "lufs": -14.0, "multiband": False,
    "low_thresh": -25.0, "low_ratio": 6.0, "mid_thresh": -20.0, "mid_ratio": 3.0,
    "high_thresh": -15.0, "high_ratio": 4.0, "art_prompt": "", "auto_generate_prompt": False,
    "create_mp3": True,
}

# hard-coded constants of the pipeline
SEGMENT_TIME_S = 30                     # ffmpeg -segment_time 30 (:178)
LOW_CROSSOVER, HIGH_CROSSOVER = 250, 4000   # :299
LOUDNORM_TP, LOUDNORM_LRA = -1.5, 11.0      # :229
ALIMITER = dict(level_in=1.0, level_out=1.0, limit=0.98, attack=5.0, release=50.0)  # :223


def apply_preset(settings, preset_name):
    """mastering_gui.py:165-168: a preset sets the four EQ gains ("None" zeroes them)."""
    s = dict(settings)
    if preset_name == "None":
        s.update(bass_boost=0, mid_cut=0, presence_boost=0, treble_boost=0)
        return s
    p = EQ_PRESETS.get(preset_name)
    if p:
        s.update(bass_boost=p.get("bass_boost", 0), mid_cut=p.get("mid_cut", 0),
                 presence_boost=p.get("presence_boost", 0), treble_boost=p.get("treble_boost", 0))
    return s
