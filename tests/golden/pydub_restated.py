"""Restatement of the parts of pydub 0.25.1 that the reference's hot path calls.

TEST INFRASTRUCTURE ONLY: used by ``make_golden.py`` to stand in for the
``pydub`` package (absent from this image) while the reference's own
``audio_mastering_engine.py`` functions are imported and run.

pydub is an upstream dependency of the reference (requirements.txt:2, unpinned);
it is NOT vendored in /root/reference, so this file restates its published
algorithm (pydub 0.25.1, ``pydub/audio_segment.py`` and ``pydub/effects.py``).
Only the members the reference touches are provided:

* ``AudioSegment``: constructor, ``channels``/``frame_rate``/``sample_width``,
  ``get_array_of_samples`` (audio_mastering_engine.py:251), ``_spawn`` (:257),
  ``set_channels`` (:190), ``frame_count``, ``get_sample_slice``, ``rms``,
  ``get_frame``, ``__len__``/``__getitem__`` (ms slicing) and ``overlay`` (:309).
* ``compress_dynamic_range`` (called at audio_mastering_engine.py:306-308).

All sample arithmetic goes through CPython's C ``audioop`` exactly as pydub does.
"""
import array
import audioop
from io import BytesIO
from math import log


def db_to_float(db, using_amplitude=True):
    db = float(db)
    if using_amplitude:
        return 10 ** (db / 20)
    return 10 ** (db / 10)


def ratio_to_db(ratio, val2=None, using_amplitude=True):
    ratio = float(ratio)
    if val2 is not None:
        ratio = ratio / val2
    if ratio == 0:
        return -float('inf')
    if using_amplitude:
        return 20 * log(ratio, 10)
    return 10 * log(ratio, 10)


class TooManyMissingFrames(Exception):
    pass


class AudioSegment(object):
    def __init__(self, data=None, sample_width=2, frame_rate=44100, channels=1):
        self.sample_width = sample_width
        self.frame_rate = frame_rate
        self.channels = channels
        self.frame_width = channels * sample_width
        if hasattr(data, 'read'):
            data.seek(0)
            data = data.read()
        self._data = bytes(data or b'')

    # --- construction helpers -------------------------------------------------
    def _spawn(self, data, overrides={}):
        if isinstance(data, list):
            data = b''.join(data)
        if isinstance(data, array.array):
            data = data.tobytes()
        if hasattr(data, 'read'):
            if hasattr(data, 'seek'):
                data.seek(0)
            data = data.read()
        meta = dict(sample_width=self.sample_width, frame_rate=self.frame_rate,
                    channels=self.channels)
        frame_width = overrides.pop('frame_width', None) if overrides else None
        meta.update(overrides)
        seg = AudioSegment(data=data, **meta)
        if frame_width is not None:
            seg.frame_width = frame_width
        return seg

    @classmethod
    def _sync(cls, *segs):
        channels = max(seg.channels for seg in segs)
        frame_rate = max(seg.frame_rate for seg in segs)
        sample_width = max(seg.sample_width for seg in segs)
        for seg in segs:
            assert (seg.channels, seg.frame_rate, seg.sample_width) == (channels, frame_rate, sample_width)
        return tuple(segs)

    # --- properties -----------------------------------------------------------
    @property
    def max_possible_amplitude(self):
        bits = self.sample_width * 8
        max_possible_val = (2 ** bits)
        return max_possible_val / 2

    @property
    def rms(self):
        return audioop.rms(self._data, self.sample_width)

    def get_array_of_samples(self, array_type_override=None):
        assert self.sample_width == 2
        return array.array('h', self._data)

    def frame_count(self, ms=None):
        if ms is not None:
            return ms * (self.frame_rate / 1000.0)
        return float(len(self._data) // self.frame_width)

    def get_frame(self, index):
        frame_start = index * self.frame_width
        frame_end = frame_start + self.frame_width
        return self._data[frame_start:frame_end]

    def get_sample_slice(self, start_sample=None, end_sample=None):
        max_val = int(self.frame_count())

        def bounded(val, default):
            if val is None:
                return default
            if val < 0:
                return 0
            if val > max_val:
                return max_val
            return val

        start_i = bounded(start_sample, 0) * self.frame_width
        end_i = bounded(end_sample, max_val) * self.frame_width
        return self._spawn(self._data[start_i:end_i])

    def set_channels(self, channels):
        if channels == self.channels:
            return self
        if channels == 2 and self.channels == 1:
            converted = audioop.tostereo(self._data, self.sample_width, 1, 1)
            return self._spawn(data=converted, overrides={'channels': channels,
                                                          'frame_width': self.frame_width * 2})
        raise NotImplementedError

    # --- millisecond slicing --------------------------------------------------
    def __len__(self):
        return round(1000 * (self.frame_count() / self.frame_rate))

    def _parse_position(self, val):
        if val < 0:
            val = len(self) - abs(val)
        val = self.frame_count(ms=len(self)) if val == float("inf") else \
            self.frame_count(ms=val)
        return int(val)

    def __getitem__(self, millisecond):
        if isinstance(millisecond, slice):
            assert not millisecond.step
            start = millisecond.start if millisecond.start is not None else 0
            end = millisecond.stop if millisecond.stop is not None else len(self)
            start = min(start, len(self))
            end = min(end, len(self))
        else:
            start = millisecond
            end = millisecond + 1
        start = self._parse_position(start) * self.frame_width
        end = self._parse_position(end) * self.frame_width
        data = self._data[start:end]
        expected_length = end - start
        missing_frames = (expected_length - len(data)) // self.frame_width
        if missing_frames:
            if missing_frames > self.frame_count(ms=2):
                raise TooManyMissingFrames("missing frames: %s" % missing_frames)
            silence = audioop.mul(data[:self.frame_width], self.sample_width, 0)
            data += (silence * missing_frames)
        return self._spawn(data)

    # --- mixing -----------------------------------------------------------------
    def overlay(self, seg, position=0, loop=False, times=None, gain_during_overlay=None):
        assert not loop and times is None and gain_during_overlay is None
        times = 1
        output = BytesIO()
        seg1, seg2 = AudioSegment._sync(self, seg)
        sample_width = seg1.sample_width
        spawn = seg1._spawn
        output.write(seg1[:position]._data)
        seg1 = seg1[position:]._data
        seg2 = seg2._data
        pos = 0
        seg1_len = len(seg1)
        seg2_len = len(seg2)
        while times:
            remaining = max(0, seg1_len - pos)
            if seg2_len >= remaining:
                seg2 = seg2[:remaining]
                seg2_len = remaining
                times = 1
            output.write(audioop.add(seg1[pos:pos + seg2_len], seg2, sample_width))
            pos += seg2_len
            times -= 1
        output.write(seg1[pos:])
        return spawn(data=output)


def compress_dynamic_range(seg, threshold=-20.0, ratio=4.0, attack=5.0, release=50.0):
    """pydub.effects.compress_dynamic_range (0.25.1), restated."""
    thresh_rms = seg.max_possible_amplitude * db_to_float(threshold)

    look_frames = int(seg.frame_count(ms=attack))

    def rms_at(frame_i):
        return seg.get_sample_slice(frame_i - look_frames, frame_i).rms

    def db_over_threshold(rms):
        if rms == 0:
            return 0.0
        db = ratio_to_db(rms / thresh_rms)
        return max(db, 0)

    output = []
    attenuation = 0.0
    attack_frames = seg.frame_count(ms=attack)
    release_frames = seg.frame_count(ms=release)
    for i in range(int(seg.frame_count())):
        rms_now = rms_at(i)
        max_attenuation = (1 - (1.0 / ratio)) * db_over_threshold(rms_now)
        attenuation_inc = max_attenuation / attack_frames
        attenuation_dec = max_attenuation / release_frames
        if rms_now > thresh_rms and attenuation <= max_attenuation:
            attenuation += attenuation_inc
            attenuation = min(attenuation, max_attenuation)
        else:
            attenuation -= attenuation_dec
            attenuation = max(attenuation, 0)
        frame = seg.get_frame(i)
        if attenuation != 0.0:
            frame = audioop.mul(frame, seg.sample_width, db_to_float(-attenuation))
        output.append(frame)
    return seg._spawn(data=b''.join(output))
