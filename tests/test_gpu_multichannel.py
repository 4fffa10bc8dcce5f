"""GPU: files with more than two channels (missing item 1).

The reference keeps a 3..8-channel chunk as ONE interleaved 1-D stream
(audio_segment_to_float_array reshapes only stereo, audio_mastering_engine.py:252):
analog character, EQ and crossover run along it (:264-265, :274, :303), width leaves it
alone (:268), pydub's compressor / overlay work on frames of C samples (:306-309).

* The chain (amx_mc_run_chunks through amx.engine.MultiChannelJob) is checked bit for bit
  against the golden vectors the reference's own chunk body made
  (tests/golden/mc*.npz, make_golden.py) and against the oracle's stream restatement on
  multi-chunk tracks.
* Loudness over C channels (libebur128's default channel map weights) and the C-channel
  alimiter are checked against the oracle's restatement (oracle/amx_oracle.c): parity
  unpinned against ffmpeg itself, like every ffmpeg stage."""
import glob
import json
import os
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

MC_GOLDEN = sorted(glob.glob(os.path.join(GOLDEN, "mc*.npz")))
MB = dict(multiband=True, low_thresh=-25.0, low_ratio=6.0, mid_thresh=-20.0, mid_ratio=3.0,
          high_thresh=-15.0, high_ratio=4.0)
VOCAL = dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0)
C3 = dict(VOCAL, lufs=-14.0, width=1.3, analog_character=40.0, **MB)


def _cmp(a, b, what, tol=0, exact_min=1.0):
    assert a.shape == b.shape, "%s: shape %s vs %s" % (what, a.shape, b.shape)
    if a.size == 0:
        return
    d = np.abs(a.astype(np.int32) - b.astype(np.int32))
    frac = float((d == 0).mean())
    assert d.max() <= tol, "%s: max |diff| %d LSB (exact %.7f)" % (what, d.max(), frac)
    assert frac >= exact_min, "%s: exact fraction %.7f" % (what, frac)


def _chain(x16, fs, settings, chunks, seg_frames=128):
    import torch
    from amx.engine import MultiChannelJob
    x16 = np.ascontiguousarray(x16, np.int16)
    job = MultiChannelJob(fs, x16.shape[1], settings, x16.shape[0], input_s16=True,
                          chunks=[(0, s, n) for s, n in chunks], seg_frames=seg_frames)
    job.run_chunks(torch.from_numpy(x16).cuda())
    torch.cuda.synchronize()
    out = job.out[:job.out_frames].cpu().numpy()
    job.close()
    return out


@pytest.mark.parametrize("path", MC_GOLDEN, ids=lambda p: os.path.basename(p)[:-4])
def test_golden_multichannel_chunk_bitexact(gpu, path):
    """the reference's own chunk body on a C-channel chunk (one interleaved stream)"""
    d = np.load(path)
    meta = json.loads(str(d["meta"]))
    out = _chain(d["x16"], meta["fs"], meta["settings"], [(0, d["x16"].shape[0])])
    _cmp(out, d["out16"], meta["name"])


@pytest.mark.parametrize("fs,C,settings,seconds", [
    (48000, 3, C3, 7.3), (48000, 6, dict(VOCAL, lufs=-14.0), 5.1), (44100, 6, dict(C3, treble_boost=-2.0), 4.0),
    (96000, 4, dict(MB), 3.1), (48000, 5, dict(bass_boost=-3.0, analog_character=100.0), 3.0),
    (48000, 8, dict(C3, bass_boost=0.0, mid_cut=0.0, presence_boost=0.0, treble_boost=0.0), 2.5),
])
@pytest.mark.parametrize("seg_frames", [128, 256])
def test_multichannel_chain_vs_oracle(gpu, oracle_mod, fs, C, settings, seconds, seg_frames):
    """three uneven chunks (state resets at chunk starts, :185-204): every chunk's output
    equals the oracle's stream chain (orc_chunk_mc, pinned to the reference goldens)"""
    from amx import synth
    n = int(fs * seconds)
    x16 = oracle_mod.quantize(synth.music_like(n, fs, C, seed=int(seconds * 10) + C, peak_dbfs=-3.0))
    assert x16.shape == (n, C)
    cuts = [0, n // 3 + 17, 2 * n // 3 - 5, n]
    chunks = [(cuts[i], cuts[i + 1] - cuts[i]) for i in range(3)]
    out = _chain(x16, fs, settings, chunks, seg_frames=seg_frames)
    ref = np.concatenate([oracle_mod.chunk_mc(x16[s:s + m], fs, settings) for s, m in chunks])
    # the IIR stages run from exact-up-to-rounding segment start states,
    # as in the stereo chain tests
    _cmp(out, ref, "mc chain fs=%d C=%d" % (fs, C), tol=3, exact_min=0.9999)


@pytest.mark.parametrize("C,settings,kind", [
    (6, C3, "mix"), (3, dict(VOCAL, lufs=-16.0), "mix"), (4, dict(lufs=None), "loud"),
    (5, dict(width=1.5), "loud"), (8, dict(C3, lufs=None), "mix"),
])
def test_multichannel_pipeline_vs_oracle(gpu, oracle_mod, C, settings, kind):
    """the whole path (:171-226) for C channels: chain, loudness over the channels with
    libebur128's weights (4: L R Ls Rs, 5: L R C Ls Rs, 6: L R C LFE Ls Rs -- the LFE
    unweighted, 8: channels 6, 7 unused), linear gain and the C-channel alimiter.
    "loud": a signal whose limiter engages (the peak signal's att trace carries it)"""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import master_array
    fs = 48000
    n = int(fs * 40.0)
    x = synth.mix_like(n, fs, C, seed=40 + C)
    if kind == "loud":
        x = np.clip(x * np.float32(2.5), -1.0, 1.0).astype(np.float32)
    y, rep = master_array(torch.from_numpy(x), fs, settings, quantum=512)
    y = y.cpu().numpy()
    x16 = oracle_mod.quantize(x)
    ref, info = oracle_mod.pipeline(x16, fs, settings, chunk_bounds(n, fs, 512))
    if settings.get("lufs") is not None:
        assert info["mode"] == "linear"
        assert rep["stats"][0] == info["stats"], (rep["stats"][0], info["stats"])
    if kind == "loud":
        assert not rep["limiter_fast"], "the limiter must engage"
    _cmp(y, ref, "mc pipeline C=%d" % C, tol=3, exact_min=0.9999)


@pytest.mark.parametrize("code,C", [("s16", 6), ("s24", 3), ("f32", 4)])
def test_master_audio_multichannel_file(gpu, oracle_mod, code, C):
    """master_audio on a C-channel WAV: same status / progress sequence as stereo, a
    C-channel 16-bit output equal to the oracle's pipeline"""
    import audio_mastering_engine as ame
    from amx import synth, wavio
    from amx.chunking import chunk_bounds, packet_frames
    fs = 48000
    n = int(fs * 35.0)
    x = synth.mix_like(n, fs, C, seed=90 + C)
    if code == "s16":
        nat = np.clip(np.round(x * 32767.0), -32768, 32767).astype(np.int16)
    elif code == "s24":
        nat = np.clip(np.round(x * 8388607.0), -8388608, 8388607).astype(np.int32)
    else:
        nat = x.astype(np.float32)
    settings = dict(C3)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "in.wav"), os.path.join(d, "out.wav")
        wavio.write_wav_pcm(src, nat, fs, code)
        st, pr = [], []
        out = ame.master_audio(dict(settings, input_file=src, output_file=dst), st.append,
                               lambda a, b: pr.append((a, b)))
        assert out == dst
        y, info = wavio.read_wav_native(dst)
        raw, winfo, _ = wavio.read_wav_raw(src)
        x16 = wavio.to_s16(wavio.read_wav_native(src)[0], winfo)
        bounds = chunk_bounds(n, fs, packet_frames(winfo.block_align))
    assert info.channels == C and info.bits == 16 and info.sample_rate == fs
    nb = len(bounds)
    assert st[:2] == ["Splitting audio into manageable chunks...", "Splitting complete."]
    assert st[-1] == "Applying final limiting and exporting..."
    assert pr[0] == (0, 100) and pr[-1] == (nb + 4, nb + 4)
    ref, rinfo = oracle_mod.pipeline(x16, fs, settings, bounds)
    _cmp(y, ref, "master_audio %s C=%d" % (code, C), tol=3, exact_min=0.9999)


def test_multichannel_refuses_dynamic_mode(gpu):
    """loudnorm's 192 kHz dynamic path runs on 1- and 2-channel files only: a C > 2 track
    that needs it raises DynamicModeUnsupported instead of writing a wrong file"""
    import torch
    from amx import synth
    from amx.engine import DynamicModeUnsupported, master_array
    fs = 48000
    n = fs * 12
    x = synth.mix_like(n, fs, 3, seed=5) * np.float32(0.12)
    rng = np.random.default_rng(5)
    for k in rng.integers(0, n - 200, 24):
        x[k:k + 50] += rng.uniform(-0.9, 0.9, (50, 3)).astype(np.float32)
    x = np.clip(x, -1.0, 1.0).astype(np.float32)
    with pytest.raises(DynamicModeUnsupported):
        master_array(torch.from_numpy(x), fs, dict(lufs=-14.0), quantum=512)
