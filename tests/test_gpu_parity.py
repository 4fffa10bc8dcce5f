"""GPU parity: the HIP path (through the C ABI) against the golden vectors made
from the reference and against the CPU oracle on seeded inputs.

Tolerance (north_star: +-1e-4 float32 of the reference chain): the reference's
output is 16-bit PCM, so 1e-4 is 3.3 LSB -> ``TOL_LSB = 3``.  Stages that are
integer/memory-less are expected bit-exact; the float64 IIR stages differ from
the sequential reference only by float64 rounding, which after the int16
quantisation is bit-exact in practice (``EXACT_MIN``)."""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

TOL_LSB = 3
EXACT_MIN = 0.9999

MB = dict(multiband=True, low_thresh=-25.0, low_ratio=6.0, mid_thresh=-20.0, mid_ratio=3.0,
          high_thresh=-15.0, high_ratio=4.0)
VOCAL = dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0)
C2 = dict(VOCAL, lufs=-14.0)
C3 = dict(VOCAL, lufs=-14.0, width=1.3, analog_character=40.0, **MB)


def _cmp(a, b, what, exact_min=EXACT_MIN, tol=TOL_LSB):
    assert a.shape == b.shape, "%s: shape %s vs %s" % (what, a.shape, b.shape)
    if a.size == 0:
        return
    d = np.abs(a.astype(np.int32) - b.astype(np.int32))
    frac = float((d == 0).mean())
    assert d.max() <= tol, "%s: max |diff| %d LSB (exact %.6f)" % (what, d.max(), frac)
    assert frac >= exact_min, "%s: exact fraction %.6f" % (what, frac)


def _chunk_chain(x16, fs, settings, chunks, seg_frames=256):
    import torch
    from amx.engine import MasteringJob
    x16 = np.ascontiguousarray(x16)
    ch = 1 if x16.ndim == 1 else x16.shape[1]
    job = MasteringJob(fs, ch, settings, [x16.shape[0]], input_s16=True,
                       chunks=[(0, s, n) for s, n in chunks], seg_frames=seg_frames)
    job.run_chunks(torch.from_numpy(x16).cuda())
    torch.cuda.synchronize()
    return job.out[:job.info.out_frames].cpu().numpy(), job


GOLDEN_2CH = [p for p in sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))) if not os.path.basename(p).startswith("mc")]


@pytest.mark.parametrize("path", GOLDEN_2CH, ids=lambda p: os.path.basename(p)[:-4])
def test_golden_chunk_bitexact(gpu, path):
    d = np.load(path)
    meta = json.loads(str(d["meta"]))
    x16 = d["x16"]
    out, _ = _chunk_chain(x16, meta["fs"], meta["settings"], [(0, x16.shape[0])], seg_frames=128)
    _cmp(out, d["out16"], meta["name"], exact_min=1.0, tol=0)


@pytest.mark.parametrize("fs,settings,seconds", [
    (48000, C2, 7.3), (48000, C3, 7.3), (44100, dict(bass_boost=3.0, treble_boost=3.0), 5.0),
    (96000, C3, 4.1), (48000, dict(VOCAL, analog_character=100.0, width=0.0), 3.0),
    (44100, dict(bass_boost=-2.0, treble_boost=-4.0, mid_cut=3.0, presence_boost=-2.0, **MB), 3.3),
    (192000, C3, 1.3), (32000, C3, 6.1),
])
@pytest.mark.parametrize("seg_frames", [128, 256, 1000])
def test_multichunk_chain_vs_oracle(gpu, oracle_mod, fs, settings, seconds, seg_frames):
    from amx import synth
    n = int(fs * seconds)
    x16 = oracle_mod.quantize(synth.music_like(n, fs, 2, seed=int(seconds * 10), peak_dbfs=-3.0))
    # three uneven chunks exercise state resets at chunk boundaries (:185-204)
    cuts = [0, n // 3 + 17, 2 * n // 3 - 5, n]
    chunks = [(cuts[i], cuts[i + 1] - cuts[i]) for i in range(3)]
    out, _ = _chunk_chain(x16, fs, settings, chunks, seg_frames=seg_frames)
    ref = np.concatenate([oracle_mod.chunk(x16[s:s + m], fs, settings) for s, m in chunks])
    _cmp(out, ref, "chain fs=%d" % fs)


@pytest.mark.parametrize("warm,rounds", [(0, 0), (0, 1), (64, 2), (-1, -1)])
@pytest.mark.parametrize("signal", ["music", "mix", "held"])
def test_compressor_fixup_paths(gpu, oracle_mod, warm, rounds, signal):
    """The envelope is exact however the work is split between speculation, the
    parallel fix-up rounds and the in-order walk (amx_dyn.hip): warm-up 0 and no
    rounds leaves everything to the walk; the music signal has long held-state
    (below-threshold) stretches between loud passages; "held" drops to -60 dB after
    2 s, so every band holds a non-zero attenuation over whole waves (the overlay's
    one-gain-per-lane path)."""
    from amx import synth
    fs = 48000
    n = int(fs * 9.7)
    if signal == "music":
        x = synth.music_like(n, fs, 2, seed=7, peak_dbfs=-3.0)
    elif signal == "held":
        x = synth.music_like(n, fs, 2, seed=9, peak_dbfs=-1.0)
        x[2 * fs:] *= 1e-3
    else:
        x = synth.mix_like(n, fs, 2, seed=7)
    x16 = oracle_mod.quantize(x)
    settings = dict(C3, _env_warm=warm, _env_rounds=rounds)
    chunks = [(0, n // 2 + 3), (n // 2 + 3, n - (n // 2 + 3))]
    out, _ = _chunk_chain(x16, fs, settings, chunks)
    ref = np.concatenate([oracle_mod.chunk(x16[s:s + m], fs, C3) for s, m in chunks])
    _cmp(out, ref, "compressor warm=%d rounds=%d %s" % (warm, rounds, signal), exact_min=1.0, tol=0)


@pytest.mark.parametrize("active", ["111", "110", "101", "010", "001", "000"])
def test_compressor_active_bands(gpu, oracle_mod, active):
    """Bands with no frame over their threshold (threshold 0 dBFS: no rms exceeds it) are
    skipped by the envelope kernels, and the active ones (threshold -40 dBFS) run on the
    segment table of their count (amx_dyn.hip env_bands, ChainDev::etab): bit-exact to
    the oracle for every pattern of active bands."""
    from amx import synth
    fs = 48000
    n = int(fs * 7.3)
    x16 = oracle_mod.quantize(synth.music_like(n, fs, 2, seed=11, peak_dbfs=-2.0))
    mb = dict(MB)
    for k, name in zip(active, ("low", "mid", "high")):
        mb[name + "_thresh"] = 0.0 if k == "0" else -40.0
    settings = dict(VOCAL, lufs=-14.0, width=1.3, analog_character=40.0, **mb)
    chunks = [(0, n // 3), (n // 3, n - n // 3)]
    out, _ = _chunk_chain(x16, fs, settings, chunks, seg_frames=128)
    ref = np.concatenate([oracle_mod.chunk(x16[s:s + m], fs, settings) for s, m in chunks])
    _cmp(out, ref, "compressor active bands %s" % active, exact_min=1.0, tol=0)


def test_mono_and_f32_quantise(gpu, oracle_mod):
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    fs = 44100
    x = synth.music_like(fs * 2, fs, 1, seed=3, peak_dbfs=0.5)   # clips: exercises A.1 clamp
    settings = dict(bass_boost=3.0, treble_boost=3.0)
    job = MasteringJob(fs, 1, settings, [x.shape[0]], chunks=[(0, 0, x.shape[0])])
    job.run_chunks(torch.from_numpy(np.ascontiguousarray(x)).cuda())
    out = job.out[:job.info.out_frames].cpu().numpy()
    ref = oracle_mod.chunk(oracle_mod.quantize(x), fs, settings)
    _cmp(out, ref, "mono f32")


def test_loudness_histograms_vs_oracle(gpu, oracle_mod):
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    fs = 48000
    n = fs * 12 + 1234
    x16 = oracle_mod.quantize(synth.music_like(n, fs, 2, seed=5, peak_dbfs=-9.0))
    job = MasteringJob(fs, 2, dict(lufs=-14.0), [n], input_s16=True, chunks=[(0, 0, n)])
    job.run_chunks(torch.from_numpy(x16).cuda())
    job.loudness_pass1()
    job.loudness_pass2(carry=False)
    job.histograms()
    hist = job.hist.cpu().numpy().view(np.uint64)[0]
    st = job.st_hist.cpu().numpy().view(np.uint64)[0]
    out = job.out[:n].cpu().numpy()
    # ffmpeg's pass 1 measures the track upsampled to 192 kHz
    oh, ost, opk, nb = oracle_mod.ebur128_192k(out, fs)
    assert hist.sum() == oh.sum() and st.sum() == ost.sum()
    # summation order differs (hop partials vs libebur128's ring sums): allow a
    # block to land in a neighbouring bin only when it sits on a boundary
    assert np.abs(hist.astype(np.int64) - oh.astype(np.int64)).sum() <= 2
    assert np.abs(st.astype(np.int64) - ost.astype(np.int64)).sum() <= 2
    pk = job.peak.cpu().numpy()[0]
    np.testing.assert_array_equal(pk[:2], opk)                      # 192 kHz sample peak, bit-exact
    np.testing.assert_array_equal(pk[2:], np.abs(out.astype(np.int32)).max(axis=0) / 32768.0)
    job.decide()
    assert job.fetch_report(raise_dynamic=False)["stats"][0] == oracle_mod.loudnorm_measure(out, fs)


@pytest.mark.parametrize("fs,settings,seconds,seed", [
    (48000, C2, 40.0, 1), (48000, C3, 31.0, 2), (44100, dict(bass_boost=3.0, treble_boost=3.0, lufs=-14.0), 35.0, 3),
    (96000, dict(C3, lufs=-16.0), 31.0, 4), (96000, C2, 12.0, 2),
])
def test_pipeline_vs_oracle(gpu, oracle_mod, fs, settings, seconds, seed):
    """Whole process_audio_with_ffmpeg_pipeline path, stage by stage: concatenated
    chunk chain, loudnorm histograms + pass-1 statistics, linear gain + alimiter."""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import master_array
    n = int(fs * seconds)
    x = synth.mix_like(n, fs, 2, seed=seed)
    y, rep = master_array(torch.from_numpy(x), fs, settings, quantum=512)
    job = rep["job"]
    ref, info = oracle_mod.pipeline(oracle_mod.quantize(x), fs, settings, chunk_bounds(n, fs, 512))
    _cmp(job.out[:job.info.out_frames].cpu().numpy(), info["concat"], "concat fs=%d" % fs)
    oh, ost, opk, _ = oracle_mod.ebur128_192k(info["concat"], fs)
    gh = job.hist.cpu().numpy().view(np.uint64)[0]
    gst = job.st_hist.cpu().numpy().view(np.uint64)[0]
    assert np.abs(gh.astype(np.int64) - oh.astype(np.int64)).sum() <= 2, np.nonzero(gh != oh)
    assert np.abs(gst.astype(np.int64) - ost.astype(np.int64)).sum() <= 2
    assert rep["stats"][0] == info["stats"], (rep["stats"], info["stats"])
    np.testing.assert_array_equal(job.peak.cpu().numpy()[0][:2], opk)
    assert rep["modes"] == ["linear"]
    _cmp(y.cpu().numpy(), ref, "pipeline fs=%d" % fs)


def test_batch_of_tracks_vs_oracle(gpu, oracle_mod):
    """C4 shape, scaled down: several tracks of different lengths in one plan (laid
    back to back), each with its own loudness statistics, gain and limiter; every
    track must equal the oracle's pipeline run on that track alone.  The silent
    track takes loudnorm's skip path (:238)."""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import MasteringJob
    fs = 48000
    xs = [synth.mix_like(int(fs * 31.0), fs, 2, seed=1),
          synth.music_like(int(fs * 12.3), fs, 2, seed=2, peak_dbfs=-3.0),
          np.zeros((int(fs * 5.0), 2), np.float32)]
    # -16 LUFS: the music track's crest factor (192 kHz TP - I = 12.54 dB) would put a
    # -14 LUFS target just past TP + offset = -1.5, i.e. into loudnorm's dynamic mode
    settings = dict(C3, lufs=-16.0)
    job = MasteringJob(fs, 2, settings, [x.shape[0] for x in xs], quantum=512)
    job.run(torch.from_numpy(np.ascontiguousarray(np.concatenate(xs))).cuda())
    rep = job.fetch_report()
    assert rep["modes"] == ["linear", "linear", "skip"], rep["modes"]
    for t, x in enumerate(xs):
        ref, info = oracle_mod.pipeline(oracle_mod.quantize(x), fs, settings, chunk_bounds(x.shape[0], fs, 512))
        if t < 2:
            assert rep["stats"][t] == info["stats"], (t, rep["stats"][t], info["stats"])
        _cmp(job.track_output(t).cpu().numpy(), ref, "batch track %d" % t)


def test_limiter_general_path(gpu, oracle_mod):
    """Loud square wave, no normalisation: alimiter engages (sequential kernel)."""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import master_array
    fs = 48000
    x = synth.square(fs * 3, fs, 2, freq=110.0, amp=1.0)
    settings = dict(bass_boost=6.0, lufs=None)
    y, rep = master_array(torch.from_numpy(x), fs, settings, quantum=512)
    assert rep["limiter_fast"] is False
    ref, _ = oracle_mod.pipeline(oracle_mod.quantize(x), fs, settings, chunk_bounds(len(x), fs, 512))
    _cmp(y.cpu().numpy(), ref, "limiter general", exact_min=1.0, tol=0)


def _bursts(n, fs, seed):
    """Quiet music with loud square bursts of random length (2 ms - 400 ms) at
    random places: limiting episodes of every length, some spanning segment
    boundaries, some back to back."""
    from amx import synth
    rng = np.random.default_rng(seed)
    x = synth.music_like(n, fs, 2, seed=seed, peak_dbfs=-12.0)
    t = 0
    while True:
        t += int(rng.integers(fs // 100, fs // 2))
        ln = int(rng.integers(fs // 500, fs * 2 // 5))
        if t + ln >= n:
            break
        x[t:t + ln] = synth.square(ln, fs, 2, freq=float(rng.uniform(60, 900)), amp=float(rng.uniform(0.9, 1.0)))
        t += ln
    return x


@pytest.mark.parametrize("fs,signal,seconds,lseg,warm", [
    (48000, "music", 20.0, 512, -1), (48000, "music", 20.0, 0, -1), (48000, "music", 20.0, 2048, 0),
    (48000, "bursts", 20.0, 512, -1), (48000, "bursts", 20.0, 4096, 0), (48000, "bursts", 20.0, 1024, 300),
    (96000, "bursts", 8.0, 512, -1), (96000, "bursts", 8.0, 1024, 0), (44100, "square", 2.0, 256, -1),
    (44100, "square", 2.0, 256, 0), (48000, "square", 0.3, 512, -1),
])
def test_limiter_segments_vs_oracle(gpu, oracle_mod, fs, signal, seconds, lseg, warm):
    """General alimiter (:223) run as warmed-up segments + in-order check and repair:
    bit-exact to the sequential oracle for loud music (frequent short episodes),
    square bursts (episodes of every length across segment boundaries), a
    continuous square (the limiter never rests) and a span shorter than one
    segment.  lseg 0 / warm -1 = the library defaults; warm 0 (segments guess the
    rest state at their first frame) and a short warm-up make most guesses wrong,
    so the walker's re-runs and state comparisons carry the result."""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import master_array
    n = int(fs * seconds)
    if signal == "music":
        x = synth.music_like(n, fs, 2, seed=7, peak_dbfs=3.0)
    elif signal == "square":
        x = synth.square(n, fs, 2, freq=110.0, amp=1.0)
    else:
        x = _bursts(n, fs, seed=int(seconds * 10) + fs)
    settings = dict(lufs=None)       # no EQ: the EQ shelves here pull the peaks under the limit
    y, rep = master_array(torch.from_numpy(x), fs, settings, quantum=512, limiter_seg_frames=lseg,
                          limiter_warm_frames=warm)
    assert rep["limiter_fast"] is False
    ref, _ = oracle_mod.pipeline(oracle_mod.quantize(x), fs, settings, chunk_bounds(n, fs, 512))
    _cmp(y.cpu().numpy(), ref, "limiter %s fs=%d lseg=%d warm=%d" % (signal, fs, lseg, warm),
         exact_min=1.0, tol=0)


def test_batch_general_limiter_vs_oracle(gpu, oracle_mod):
    """Several tracks in one plan with settings lufs None: two loud tracks of
    different lengths take the general limiter (per-track segment slots and
    counters in the same launch), a quiet one the idle path; each equals the
    oracle's pipeline on that track alone."""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import MasteringJob
    fs = 48000
    settings = dict(lufs=None)
    xs = [_bursts(int(fs * 9.0), fs, seed=5), synth.music_like(int(fs * 4.0), fs, 2, seed=6, peak_dbfs=-9.0),
          synth.music_like(int(fs * 13.7), fs, 2, seed=7, peak_dbfs=3.0)]
    job = MasteringJob(fs, 2, settings, [x.shape[0] for x in xs], quantum=512, limiter_seg_frames=2048)
    job.run(torch.from_numpy(np.ascontiguousarray(np.concatenate(xs))).cuda())
    rep = job.fetch_report()
    fast = [bool(int(v) & 1) for v in job.ctl.cpu().tolist()]
    assert fast == [False, True, False], fast
    for t, x in enumerate(xs):
        ref, _ = oracle_mod.pipeline(oracle_mod.quantize(x), fs, settings, chunk_bounds(x.shape[0], fs, 512))
        _cmp(job.track_output(t).cpu().numpy(), ref, "batch general limiter track %d" % t,
             exact_min=1.0, tol=0)


def test_silence_skips_normalisation(gpu, oracle_mod):
    import torch
    from amx.engine import master_array
    fs = 48000
    x = np.zeros((fs * 2, 2), np.float32)
    y, rep = master_array(torch.from_numpy(x), fs, dict(C3), quantum=512)
    assert rep["modes"] == ["skip"] and rep["stats"][0]["input_i"] == "-inf"
    assert int(np.abs(y.cpu().numpy()).max()) == 0


def test_short_and_edge_lengths(gpu, oracle_mod):
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    fs = 48000
    for n in (1, 7, 255, 256, 257, 241, 4799):
        x16 = oracle_mod.quantize(synth.music_like(n, fs, 2, seed=n))
        out, _ = _chunk_chain(x16, fs, C3, [(0, n)])
        _cmp(out, oracle_mod.chunk(x16, fs, C3), "n=%d" % n, exact_min=1.0, tol=0)


def test_deterministic(gpu):
    import torch
    from amx import synth
    from amx.engine import master_array
    fs = 48000
    x = torch.from_numpy(synth.music_like(fs * 5, fs, 2, seed=11, peak_dbfs=-3.0))
    a, _ = master_array(x, fs, dict(C3, lufs=None))
    b, _ = master_array(x, fs, dict(C3, lufs=None))
    assert torch.equal(a, b)


@pytest.mark.parametrize("settings", [C2, C3], ids=["c2", "c3"])
def test_graph_replay_matches_eager(gpu, oracle_mod, settings):
    """The captured hipGraph of the whole pipeline (MasteringJob.capture, used by
    bench.py) replays to the eager result and the oracle, also after the input
    buffer's contents change (the graph holds pointers, not values)."""
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    fs = 48000
    n = fs * 12
    xs = [synth.mix_like(n, fs, 2, seed=s) for s in (21, 22)]
    job = MasteringJob(fs, 2, settings, [n])
    d_in = torch.from_numpy(xs[0]).cuda()
    eager = job.run(d_in).cpu().numpy()
    job.capture(d_in)
    np.testing.assert_array_equal(job.replay().cpu().numpy(), eager)
    d_in.copy_(torch.from_numpy(xs[1]))
    y = job.replay().cpu().numpy()
    eager2 = MasteringJob(fs, 2, settings, [n]).run(torch.from_numpy(xs[1]).cuda()).cpu().numpy()
    np.testing.assert_array_equal(y, eager2)


@pytest.mark.slow
def test_full_size_c3_5min(gpu, oracle_mod):
    """BASELINE config 3 at full size (5 min stereo 48 kHz) against the oracle."""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import master_array
    fs = 48000
    n = fs * 300
    x = synth.mix_like(n, fs, 2, seed=5)
    y, rep = master_array(torch.from_numpy(x), fs, C3, quantum=512)
    ref, info = oracle_mod.pipeline(oracle_mod.quantize(x), fs, C3, chunk_bounds(n, fs, 512))
    assert rep["stats"][0] == info["stats"]
    _cmp(y.cpu().numpy(), ref, "C3 5 min")


@pytest.mark.parametrize("s16", [False, True])
def test_track_stream_matches_single_jobs(gpu, s16):
    """Double-buffered host pipeline (amx.stream_io.TrackStream, §8f row 2): five
    tracks through two resident jobs on three streams give, track by track, the
    output and loudnorm statistics of a single job run on that track alone."""
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    from amx.stream_io import TrackStream
    fs, n = 48000, 48000 * 7
    xs = [synth.mix_like(n, fs, 2, seed=40 + i) for i in range(5)]
    if s16:
        xs = [synth.to_s16(x) for x in xs]
    ts = TrackStream(fs, 2, C3, n, depth=2, input_s16=s16, quantum=512)
    h_ins = []
    for x in xs:
        h = ts.pinned_input()
        h.copy_(torch.from_numpy(x))
        h_ins.append(h)
    outs = [ts.pinned_output() for _ in xs]
    stats = [ts.pinned_stats() for _ in xs]
    ts.run(h_ins, outs, stats)
    for i, x in enumerate(xs):
        job = MasteringJob(fs, 2, C3, [n], quantum=512, input_s16=s16)
        y = job.run(torch.from_numpy(x).cuda())
        torch.cuda.synchronize()
        assert torch.equal(y.cpu(), outs[i]), "track %d output" % i
        assert torch.equal(job.stats.cpu(), stats[i]), "track %d stats" % i


@pytest.mark.parametrize("fs", [48000, 44100, 96000])
def test_tp_decision_at_192k(gpu, oracle_mod, fs):
    """The linear / dynamic decision (af_loudnorm, :240) on the 192 kHz input_tp: a
    square-ish signal has inter-sample peaks well above its samples, so targets a
    hair either side of TP + offset = -1.5 must flip the device's decision exactly
    where the oracle's does -- and where a native-rate measurement would not."""
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    n = int(fs * 12.0)
    x = synth.music_like(n, fs, 2, seed=17, peak_dbfs=-1.0)
    x = np.clip(x * 3.0, -0.5, 0.5).astype(np.float32)          # clipped: inter-sample overs
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    st_native = oracle_mod.loudnorm_measure(x16, fs, native=True)
    assert float(st["input_tp"]) > float(st_native["input_tp"])
    edge = -1.5 - float(st["input_tp"]) + float(st["input_i"])    # target where TP + offset = -1.5
    for target, want in ((edge - 0.01, "linear"), (edge, None), (edge + 0.01, "dynamic")):
        target = round(target, 2)
        job = MasteringJob(fs, 2, dict(lufs=target), [n], input_s16=True, chunks=[(0, 0, n)])
        job.run(torch.from_numpy(x16).cuda())
        rep = job.fetch_report(raise_dynamic=False)
        assert rep["stats"][0] == st, (rep["stats"][0], st)
        mode, _ = oracle_mod.loudnorm_linear_gain(st, target)
        assert (want is None or mode == want) and rep["modes"] == [mode], (target, mode, rep["modes"])


@pytest.mark.parametrize("env", [{}, {"AMX_F1": "2"}], ids=["split", "front1s"])
def test_front1_variants_vs_oracle(gpu, oracle_mod, monkeypatch, env):
    """both forms of the float32 analog + EQ front (amx_chain.hip front1s_t) give the
    oracle's result: k_analog_h (the odd tanh table's half in LDS) + k_gemv16, and
    k_front1s with the full table (the form a table that is not odd takes)"""
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    fs = 48000
    n = int(fs * 3.1)
    x16 = oracle_mod.quantize(synth.music_like(n, fs, 2, seed=31, peak_dbfs=-1.0))
    settings = dict(C3, analog_character=100.0)
    cuts = [(0, n // 2 + 3), (n // 2 + 3, n - n // 2 - 3)]
    # float32 input x16 / 32768: ffmpeg's quantisation gives x16 back exactly
    xf = np.ascontiguousarray(x16.astype(np.float32) / np.float32(32768.0))
    job = MasteringJob(fs, 2, settings, [n], chunks=[(0, s, m) for s, m in cuts], seg_frames=128)
    job.run_chunks(torch.from_numpy(xf).cuda())
    out = job.out[:job.info.out_frames].cpu().numpy()
    ref = np.concatenate([oracle_mod.chunk(x16[s:s + m], fs, settings) for s, m in cuts])
    _cmp(out, ref, "front1 %s" % env)


@pytest.mark.parametrize("fs,env", [
    (44100, {}), (44100, {"AMX_UP_POLY": "0"}), (88200, {}), (176400, {}), (32000, {}), (64000, {}),
    (24000, {}), (22050, {}), (11025, {}),
], ids=["44k1-poly", "44k1-slow", "88k2-poly", "176k4-poly", "32k-poly", "64k-poly", "24k-slow",
        "22k05-lin", "11k025-lin"])
def test_loudness_192k_rates_vs_oracle(gpu, oracle_mod, monkeypatch, fs, env):
    """the 192 kHz measurement at the rates without the unrolled k_up: k_up_poly's forms
    (amx_loud192.hip AMX_UP_POLY_FORMS) and k_up_slow (AMX_UP_POLY = 0, and 24 kHz, whose
    form is not built; 22.05 / 11.025 kHz with libswresample's 1024-phase interpolating
    kernel, swr_dot_lin) -- histograms, 192 kHz sample peaks bit for bit, the statistics"""
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n = fs * 7 + 1234
    x16 = oracle_mod.quantize(synth.music_like(n, fs, 2, seed=fs % 1000, peak_dbfs=-2.0))
    job = MasteringJob(fs, 2, dict(lufs=-14.0), [n], input_s16=True, chunks=[(0, 0, n)])
    job.run_chunks(torch.from_numpy(x16).cuda())
    job.loudness_pass1()
    job.loudness_pass2(carry=False)
    job.histograms()
    hist = job.hist.cpu().numpy().view(np.uint64)[0]
    st = job.st_hist.cpu().numpy().view(np.uint64)[0]
    out = job.out[:n].cpu().numpy()
    oh, ost, opk, _ = oracle_mod.ebur128_192k(out, fs)
    assert hist.sum() == oh.sum() and st.sum() == ost.sum()
    assert np.abs(hist.astype(np.int64) - oh.astype(np.int64)).sum() <= 2
    assert np.abs(st.astype(np.int64) - ost.astype(np.int64)).sum() <= 2
    np.testing.assert_array_equal(job.peak.cpu().numpy()[0][:2], opk)
    job.decide()
    assert job.fetch_report(raise_dynamic=False)["stats"][0] == oracle_mod.loudnorm_measure(out, fs)
