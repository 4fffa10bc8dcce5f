"""loudnorm dynamic mode (audio_mastering_engine.py:240 when the linear conditions fail)
on the GPU against the oracle's restatement of af_loudnorm (oracle/amx_oracle.c
orc_loudnorm; parity unpinned: no ffmpeg here).

* the filter alone (amx_loudnorm_192k) on a track with given pass-1 strings, against
  orc_loudnorm with the same options: 192 kHz resampler, 3 s / 100 ms framing, Gaussian
  AGC, true-peak limiter, final flush frame;
* the file-level drop-in (master_audio) on material that takes dynamic mode: pass 1's
  target_offset from its own filter run, pass 2, the alimiter at 192 kHz, a 192 kHz WAV;
* the < 3 s linear fallback and a silent intro (above_threshold starts at 0, so the
  output's short-term loudness steers the first frames).

The GPU statistics come from the 192 kHz hop energies (rounding-level differences from
libebur128's sequential sums) and device libm, so the outputs are compared within the
north_star's 3 LSB, with nearly every sample exact."""
import os
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dynamic_signal(seconds, fs, seed, intro=0.0):
    """quiet program with sparse full-scale transients: TP + offset > -1.5 dBTP"""
    from amx import synth
    n = int(fs * seconds)
    x = synth.mix_like(n, fs, 2, seed=seed) * 0.12
    rng = np.random.default_rng(seed)
    for k in rng.integers(0, n - 200, max(2, int(seconds * 2))):
        x[k:k + 50] += rng.uniform(-0.9, 0.9, (50, 2))
    if intro:
        x[:int(fs * intro)] = 0.0
    return np.clip(x, -1.0, 1.0).astype(np.float32)


def _cmp(y, ref, what, tol=3, exact_min=0.999):
    assert y.shape == ref.shape, (what, y.shape, ref.shape)
    d = np.abs(y.astype(np.int32) - ref.astype(np.int32))
    exact = float((d == 0).mean()) if d.size else 1.0
    print("%s: max |diff| %d LSB, exact fraction %.7f" % (what, d.max() if d.size else 0, exact))
    assert (d.max() if d.size else 0) <= tol and exact >= exact_min, (what, int(d.max()), exact)


@pytest.mark.parametrize("seconds,seed,intro", [(12.0, 3, 0.0), (7.3, 5, 0.0), (9.0, 8, 4.0)])
def test_filter_vs_oracle(gpu, oracle_mod, seconds, seed, intro):
    import torch
    from amx import capi
    from amx.engine import MasteringJob
    fs = 48000
    x = _dynamic_signal(seconds, fs, seed, intro)
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    # no chain: the job's d_out is the track itself; its pass-1 measurement feeds the filter
    job = MasteringJob(fs, 2, {"lufs": -14.0}, [x16.shape[0]], input_s16=True,
                       chunks=[(0, 0, x16.shape[0])], measure_only=True)
    job.out[:x16.shape[0]].copy_(torch.from_numpy(x16))
    job.loudness_pass1(tail=False)
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    rep = job.fetch_report(raise_dynamic=False)
    assert rep["stats"][0] == st, (rep["stats"][0], st)
    n192, job2, ws2, summ = job._job192(0)
    for measured, offset in ((None, 0.0), (st, 2.37)):
        d = capi.LoudnormDesc(-14.0, 11.0, -1.5, 0.0, 0.0, 99.0, -70.0, offset)
        if measured:
            d.measured_i, d.measured_lra = float(st["input_i"]), float(st["input_lra"])
            d.measured_tp, d.measured_thresh = float(st["input_tp"]), float(st["input_thresh"])
        job.loudnorm_192k(0, d, job2, ws2, summ)
        y = job2.out[:n192].cpu().numpy()
        ref, _ = oracle_mod.loudnorm(x16, fs, -14.0, measured=measured, offset=offset)
        _cmp(y, ref, "loudnorm filter %.1f s intro %.1f %s" % (seconds, intro, "pass 2" if measured else "pass 1"))


@pytest.mark.parametrize("seg,warm", [(1, 0), (2, 1), (7, 0), (4, 3)])
def test_parallel_splits_vs_oracle(gpu, oracle_mod, monkeypatch, seg, warm):
    """the parallel form under work splits that make most start guesses wrong (no
    warm-up, one-frame segments) on material that keeps the true-peak limiter busy
    (an offset of +9 dB): the walker's re-runs and the FINAL re-run carry the result,
    which must still be the oracle's"""
    import torch
    from amx import capi
    from amx.engine import MasteringJob
    monkeypatch.setenv("AMX_LN_SEG", str(seg))
    monkeypatch.setenv("AMX_LN_WARM", str(warm))
    fs = 48000
    x = _dynamic_signal(20.0, fs, 17)
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    job = MasteringJob(fs, 2, {"lufs": -14.0}, [x16.shape[0]], input_s16=True,
                       chunks=[(0, 0, x16.shape[0])], measure_only=True)
    job.out[:x16.shape[0]].copy_(torch.from_numpy(x16))
    job.loudness_pass1(tail=False)
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    n192, job2, ws2, summ = job._job192(0, cached=False)[0:4]
    for offset in (0.0, 9.0):
        d = capi.LoudnormDesc(-14.0, 11.0, -1.5, float(st["input_i"]), float(st["input_lra"]),
                              float(st["input_tp"]), float(st["input_thresh"]), offset)
        job.loudnorm_192k(0, d, job2, ws2, summ)
        s = summ.cpu().numpy()
        assert s[12] > 0 and s[13] == 0, s
        ref, _ = oracle_mod.loudnorm(x16, fs, -14.0, measured=st, offset=offset)
        print("split Fs=%d Wf=%d offset %.1f: %d segments, %d re-run, FINAL re-run %d" %
              (seg, warm, offset, s[12], s[10], s[11]))
        _cmp(job2.out[:n192].cpu().numpy(), ref, "parallel split Fs=%d Wf=%d offset %.1f" % (seg, warm, offset))


@pytest.mark.parametrize("seg,warm,intro", [(None, None, 0.0), (1, 0, 0.0), (None, None, 6.0), (2, 1, 12.5)])
def test_fill_prepass_equals_dense_form(gpu, oracle_mod, monkeypatch, seg, warm, intro):
    """k_lp_fill + the skipping peak scan + the sparse emit (the default) against the
    dense form (AMX_LP_FILL=0: every position's value loaded in the scans, every output
    written by k_lp_seg), bit for bit, on an output buffer poisoned before each run (a
    position neither form writes would show); quiet (+0 dB) and busy (+9 dB) limiters,
    one-frame segments without warm-up (re-runs), and quiet starts (the hand-over)"""
    import torch
    from amx import capi
    from amx.engine import MasteringJob
    if seg is not None:
        monkeypatch.setenv("AMX_LN_SEG", str(seg))
        monkeypatch.setenv("AMX_LN_WARM", str(warm))
    fs = 48000
    x = _dynamic_signal(24.0, fs, 23, intro)
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    job = MasteringJob(fs, 2, {"lufs": -14.0}, [x16.shape[0]], input_s16=True,
                       chunks=[(0, 0, x16.shape[0])], measure_only=True)
    job.out[:x16.shape[0]].copy_(torch.from_numpy(x16))
    job.loudness_pass1(tail=False)
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    n192, job2, ws2, summ = job._job192(0, cached=False)[0:4]
    for offset in (0.0, 9.0):
        d = capi.LoudnormDesc(-14.0, 11.0, -1.5, float(st["input_i"]), float(st["input_lra"]),
                              float(st["input_tp"]), float(st["input_thresh"]), offset)
        outs = []
        for fill in ("0", "1"):
            monkeypatch.setenv("AMX_LP_FILL", fill)
            job2.out.fill_(12345)
            job.loudnorm_192k(0, d, job2, ws2, summ)
            outs.append(job2.out[:n192].cpu().numpy())
        s = summ.cpu().numpy()
        print("fill pre-pass, offset %.1f: %d segments, %d re-run, FINAL re-run %d, handed over at %d" %
              (offset, s[12], s[10], s[11], s[14]))
        np.testing.assert_array_equal(outs[1], outs[0])
        ref, _ = oracle_mod.loudnorm(x16, fs, -14.0, measured=st, offset=offset)
        _cmp(outs[1], ref, "fill pre-pass offset %.1f" % offset)


@pytest.mark.parametrize("seg,warm,intro", [(4, 3, 6.0), (1, 0, 6.0), (4, 3, 12.5)])
def test_quiet_start_handover_vs_oracle(gpu, oracle_mod, monkeypatch, seg, warm, intro):
    """a quiet intro (the first 3 s below measured_thresh: above_threshold 0, so the
    output's own short-term loudness steers the gains) runs frame by frame in k_ln_dyn
    until the output reaches the target, then the state is handed to the parallel form at
    the next segment start (summary[14] = that frame); the whole output stays the
    oracle's"""
    import torch
    from amx import capi
    from amx.engine import MasteringJob
    monkeypatch.setenv("AMX_LN_SEG", str(seg))
    monkeypatch.setenv("AMX_LN_WARM", str(warm))
    fs = 48000
    x = _dynamic_signal(40.0, fs, 29, intro=intro)
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    job = MasteringJob(fs, 2, {"lufs": -14.0}, [x16.shape[0]], input_s16=True,
                       chunks=[(0, 0, x16.shape[0])], measure_only=True)
    job.out[:x16.shape[0]].copy_(torch.from_numpy(x16))
    job.loudness_pass1(tail=False)
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    n192, job2, ws2, summ = job._job192(0, cached=False)
    for offset in (8.0, 14.0):
        d = capi.LoudnormDesc(-14.0, 11.0, -1.5, float(st["input_i"]), float(st["input_lra"]),
                              float(st["input_tp"]), float(st["input_thresh"]), offset)
        job.loudnorm_192k(0, d, job2, ws2, summ)
        s = summ.cpu().numpy()
        ref, _ = oracle_mod.loudnorm(x16, fs, -14.0, measured=st, offset=offset)
        print("quiet start %.1f s, Fs=%d Wf=%d offset %.1f: hand-over at frame %d, %d segments, %d re-run" %
              (intro, seg, warm, offset, s[14], s[12], s[10]))
        assert s[12] > 0 and s[13] == 0 and s[14] > 0, s
        _cmp(job2.out[:n192].cpu().numpy(), ref, "quiet start %.1f s Fs=%d Wf=%d offset %.1f" % (intro, seg, warm, offset))


@pytest.mark.parametrize("warm", [3, 0])
def test_parallel_final_rerun_vs_oracle(gpu, oracle_mod, monkeypatch, warm):
    """a loud tail keeps the true-peak limiter busy across the FINAL flush frame's start,
    where af_loudnorm re-bases its ring with the limiter's envelope index still set: the
    walker runs FINAL itself from the true state"""
    import torch
    from amx import capi
    from amx.engine import MasteringJob
    monkeypatch.setenv("AMX_LN_WARM", str(warm))
    fs = 48000
    x = _dynamic_signal(14.0, fs, 23)
    n = x.shape[0]
    t = np.arange(n - 4 * fs, n) / fs
    # loud enough to keep the limiter busy under a +14 dB offset, not so loud that the
    # quiet start falls below the relative gate (that track would run frame by frame)
    x[n - 4 * fs:] = (0.25 * np.sin(2 * np.pi * 997.0 * t) * (1.0 + 0.3 * np.sin(2 * np.pi * 3.0 * t)))[:, None]
    x = np.clip(x, -1.0, 1.0).astype(np.float32)
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    job = MasteringJob(fs, 2, {"lufs": -14.0}, [x16.shape[0]], input_s16=True,
                       chunks=[(0, 0, x16.shape[0])], measure_only=True)
    job.out[:x16.shape[0]].copy_(torch.from_numpy(x16))
    job.loudness_pass1(tail=False)
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    n192, job2, ws2, summ = job._job192(0, cached=False)
    d = capi.LoudnormDesc(-14.0, 11.0, -1.5, float(st["input_i"]), float(st["input_lra"]),
                          float(st["input_tp"]), float(st["input_thresh"]), 14.0)
    job.loudnorm_192k(0, d, job2, ws2, summ)
    s = summ.cpu().numpy()
    ref, _ = oracle_mod.loudnorm(x16, fs, -14.0, measured=st, offset=14.0)
    print("loud tail Wf=%d: %d segments, %d re-run, FINAL re-run %d" % (warm, s[12], s[10], s[11]))
    assert s[12] > 0 and s[13] == 0 and s[11] == 1, s
    _cmp(job2.out[:n192].cpu().numpy(), ref, "loud tail, FINAL re-run, Wf=%d" % warm)


@pytest.mark.parametrize("dyn_graph", [False, True], ids=["eager_dynamic", "graph_dynamic"])
def test_graph_step_with_dynamic(gpu, oracle_mod, dyn_graph):
    """capture(dynamic=True): one hipGraph holds the whole step of a two-track batch, one
    track linear and one that loudnorm sends to dynamic mode; replays give the eager
    outputs bit for bit, and the dynamic track matches the oracle's pipeline.
    graph_dynamic: the dynamic path replayed from its own graph (it
    used to re-run walker segments the eager launches never did) -- every replay gives
    the eager run's output and the eager walker's counters"""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import MasteringJob
    fs = 48000
    settings = dict(mid_cut=2.0, lufs=-14.0)
    xa = synth.mix_like(fs * 10, fs, 2, seed=61)
    xb = _dynamic_signal(11.0, fs, 62)
    d_in = torch.from_numpy(np.ascontiguousarray(np.concatenate([xa, xb]))).cuda()
    eager = MasteringJob(fs, 2, settings, [xa.shape[0], xb.shape[0]], quantum=512)
    eager.run(d_in)
    rep = eager.fetch_report(raise_dynamic=False)
    assert rep["modes"] == ["linear", "dynamic"], rep["modes"]
    eager.finish_dynamic(rep)
    want = [eager.track_output(t).cpu().numpy() for t in range(2)]
    job = MasteringJob(fs, 2, settings, [xa.shape[0], xb.shape[0]], quantum=512)
    job.capture(d_in, dynamic=True, dyn_graph=dyn_graph)
    assert (job._dyn_graphs is not None) == dyn_graph
    for _ in range(4 if dyn_graph else 2):
        job.replay()
        torch.cuda.synchronize()
        rep2 = job.fetch_report(raise_dynamic=False)
        assert rep2["modes"] == ["linear", "dynamic"]
        assert job.dynamic_output(0) is None
        y1, info = job.dynamic_output(1)
        assert info["target_offset"] == eager.dyn_out[1][1]["target_offset"]
        assert info.get("pass2_parallel") == eager.dyn_out[1][1].get("pass2_parallel"), \
            (info.get("pass2_parallel"), eager.dyn_out[1][1].get("pass2_parallel"))
        assert np.array_equal(job.track_output(0).cpu().numpy(), want[0])
        assert np.array_equal(y1.cpu().numpy(), want[1])
    ref, rinfo = oracle_mod.pipeline(oracle_mod.quantize(xb), fs, settings, chunk_bounds(xb.shape[0], fs, 512))
    assert rinfo["mode"] == "dynamic"
    _cmp(want[1], ref, "graph step, dynamic track")


def test_graph_step_dynamic_gate_linear_batch(gpu):
    """capture(dynamic=True) on a batch whose tracks all stay linear: the dynamic path
    sits in a graph of its own that replay() launches only when a track's decision word
    (copied to pinned memory before the limiter kernel) says dynamic, so a linear step
    costs the dynamic=False graph and one host read that overlaps the limiter: within
    10 % of it (round 4: +130 %, ~25 gated nodes per track); the outputs are the same
    bit for bit"""
    import time
    import torch
    from amx import synth
    from amx.engine import MasteringJob
    fs = 48000
    settings = dict(mid_cut=2.0, lufs=-14.0)
    xs = [synth.mix_like(fs * 60, fs, 2, seed=70 + k) for k in range(2)]
    d_in = torch.from_numpy(np.ascontiguousarray(np.concatenate(xs))).cuda()
    n = [x.shape[0] for x in xs]
    times, outs = {}, {}
    for dyn in (False, True):
        job = MasteringJob(fs, 2, settings, n, quantum=512)
        job.capture(d_in, dynamic=dyn)
        for _ in range(3):
            job.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            job.replay()
        torch.cuda.synchronize()
        times[dyn] = (time.perf_counter() - t0) / 20
        assert job.fetch_report(raise_dynamic=False)["modes"] == ["linear", "linear"]
        outs[dyn] = job.y[:job.info.out_frames].cpu().numpy()
    print("linear batch step: dynamic=False %.3f ms, dynamic=True %.3f ms" % (times[False] * 1e3, times[True] * 1e3))
    assert np.array_equal(outs[False], outs[True])
    assert times[True] <= 1.10 * times[False], times


@pytest.mark.timeout(900)
def test_filter_300s_vs_oracle(gpu, oracle_mod):
    """a 5-minute track (the C2/C3 length) through the parallel form of dynamic mode
    (k_lp_stats / k_lp_seg / k_lp_walk) against orc_loudnorm, with pass 1's options and
    with pass 2's (the measured strings, an offset): every segment boundary checked, the
    FINAL flush frame, the whole 192 kHz output compared"""
    import time
    import torch
    from amx import capi
    from amx.engine import MasteringJob
    fs = 48000
    x = _dynamic_signal(300.0, fs, 3)
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    job = MasteringJob(fs, 2, {"lufs": -14.0}, [x16.shape[0]], input_s16=True,
                       chunks=[(0, 0, x16.shape[0])], measure_only=True)
    job.out[:x16.shape[0]].copy_(torch.from_numpy(x16))
    job.loudness_pass1(tail=False)
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    assert job.fetch_report(raise_dynamic=False)["stats"][0] == st
    n192, job2, ws2, summ = job._job192(0)
    for measured, offset in ((None, 0.0), (st, 2.37)):
        d = capi.LoudnormDesc(-14.0, 11.0, -1.5, 0.0, 0.0, 99.0, -70.0, offset)
        if measured:
            d.measured_i, d.measured_lra = float(st["input_i"]), float(st["input_lra"])
            d.measured_tp, d.measured_thresh = float(st["input_tp"]), float(st["input_thresh"])
        job.loudnorm_192k(0, d, job2, ws2, summ)           # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        job.loudnorm_192k(0, d, job2, ws2, summ)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        s = summ.cpu().numpy()
        assert s[12] > 0 and s[13] == 0, s            # the parallel form ran (no hand-over)
        y = job2.out[:n192].cpu().numpy()
        ref, _ = oracle_mod.loudnorm(x16, fs, -14.0, measured=measured, offset=offset)
        print("300 s filter %s: %.2f ms, %d segments, %d re-run, FINAL re-run %d" %
              ("pass 2" if measured else "pass 1", dt * 1e3, s[12], s[10], s[11]))
        _cmp(y, ref, "loudnorm filter 300 s %s" % ("pass 2" if measured else "pass 1"))


@pytest.mark.parametrize("seconds,intro,fs", [(12.0, 0.0, 48000), (30.0, 4.0, 44100), (9.0, 0.0, 96000)])
def test_dynamic_output_within_ceiling(gpu, oracle_mod, monkeypatch, seconds, intro, fs):
    """the 192 kHz alimiter's input bound is af_loudnorm's ceiling
    (engine.ln_output_bound) instead of a measurement -- exact only if EVERY sample of the
    filter's output, the FIRST frame, a quiet start's frames and the FINAL flush included,
    stays within it after s16 rounding.  Checked on the filter's whole 192 kHz output of
    both passes, and the final output equals the measured path's (AMX_LN_MEASURED_BOUND=1)"""
    import torch
    from amx.engine import MasteringJob, ln_output_bound
    x = _dynamic_signal(seconds, fs, 23, intro)
    settings = dict(bass_boost=1.0, lufs=-14.0)
    outs = {}
    for measured in ("0", "1"):
        monkeypatch.setenv("AMX_LN_MEASURED_BOUND", measured)
        job = MasteringJob(fs, 2, settings, [x.shape[0]], quantum=512)
        job.run(torch.from_numpy(x).cuda())
        rep = job.fetch_report(raise_dynamic=False)
        assert rep["modes"] == ["dynamic"], rep
        y, info = job.dynamic_track(0, rep["stats"][0])
        n192, job2 = job._j192[0][1], job._j192[1]
        filt = job2.out[:n192].cpu().numpy()          # pass 2's filter output (the alimiter's input)
        outs[measured] = y.cpu().numpy()
        bound = ln_output_bound(n192) if measured == "0" else None
        if measured == "0":
            assert bound is not None
            lim = int(round(bound * 32768))
            assert int(np.abs(filt.astype(np.int32)).max()) <= lim, (np.abs(filt.astype(np.int32)).max(), lim)
        job.close()
    np.testing.assert_array_equal(outs["0"], outs["1"])


@pytest.mark.parametrize("seconds,intro,fs", [(12.0, 0.0, 48000), (2.0, 0.0, 48000), (8.0, 3.5, 48000),
                                              (9.0, 0.0, 22050)])
def test_master_audio_dynamic(gpu, oracle_mod, seconds, intro, fs):
    """(22.05 kHz: the filter's 192 kHz input comes from libswresample's interpolating
    1024-phase kernel, k_ln_upsample's lin form)"""
    import audio_mastering_engine as ame
    from amx import wavio
    from amx.chunking import chunk_bounds, packet_frames
    x = _dynamic_signal(seconds, fs, 11, intro)
    settings = dict(bass_boost=1.0, lufs=-14.0)
    with tempfile.TemporaryDirectory() as dd:
        src, dst = os.path.join(dd, "in.wav"), os.path.join(dd, "out.wav")
        wavio.write_wav_f32(src, x, fs)
        out = ame.master_audio(dict(settings, input_file=src, output_file=dst))
        y, info = wavio.read_wav_native(dst)
        raw, winfo, _ = wavio.read_wav_raw(src)
        x16 = wavio.to_s16(wavio.read_wav_native(src)[0], winfo)
        bounds = chunk_bounds(x16.shape[0], fs, packet_frames(winfo.block_align))
    assert out == dst
    ref, rinfo = oracle_mod.pipeline(x16, fs, settings, bounds)
    assert rinfo["mode"] == "dynamic", rinfo.get("stats")
    assert info.sample_rate == 192000 == rinfo["sample_rate"]
    _cmp(y, ref, "master_audio dynamic %.1f s intro %.1f" % (seconds, intro))


def test_batch_linear_and_dynamic(gpu, oracle_mod):
    """one plan, two whole tracks (a C4-style batch): one stays linear, one takes dynamic
    mode; finish_dynamic replaces the dynamic track's slot with its 192 kHz output"""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import MasteringJob
    fs = 48000
    settings = dict(mid_cut=2.0, lufs=-16.0)
    xa = synth.mix_like(fs * 10, fs, 2, seed=21)
    xb = _dynamic_signal(9.0, fs, 22)
    job = MasteringJob(fs, 2, settings, [xa.shape[0], xb.shape[0]], quantum=512)
    d_in = torch.from_numpy(np.ascontiguousarray(np.concatenate([xa, xb]))).cuda()
    job.run(d_in)
    rep = job.fetch_report(raise_dynamic=False)
    assert rep["modes"] == ["linear", "dynamic"], rep["modes"]
    info = job.finish_dynamic(rep)
    assert list(info) == [1] and info[1]["sample_rate"] == 192000
    for t, x in enumerate((xa, xb)):
        x16 = oracle_mod.quantize(x)
        ref, rinfo = oracle_mod.pipeline(x16, fs, settings, chunk_bounds(x16.shape[0], fs, 512))
        _cmp(job.track_output(t).cpu().numpy(), ref, "batch track %d (%s)" % (t, rinfo["mode"]))


def test_trackstream_dynamic(gpu, oracle_mod):
    """pipelined TrackStream: a dynamic track raises by default; with dynamic={} it is
    stepped again and finished at 192 kHz, the linear tracks keep their slots"""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import DynamicModeUnsupported
    from amx.stream_io import TrackStream
    fs, n = 48000, 48000 * 6
    settings = dict(bass_boost=1.0, lufs=-14.0)
    xs = [synth.mix_like(n, fs, 2, seed=31), _dynamic_signal(6.0, fs, 32), synth.mix_like(n, fs, 2, seed=33)]
    ts = TrackStream(fs, 2, settings, n, depth=2, quantum=512)
    h_ins = [ts.pinned_input().copy_(torch.from_numpy(x)) for x in xs]
    h_outs = [ts.pinned_output() for _ in xs]
    with pytest.raises(DynamicModeUnsupported):
        ts.run(h_ins, h_outs)
    dyn = {}
    ts.run(h_ins, h_outs, dynamic=dyn)
    assert list(dyn) == [1] and dyn[1][1]["sample_rate"] == 192000
    for i, x in enumerate(xs):
        x16 = oracle_mod.quantize(x)
        ref, rinfo = oracle_mod.pipeline(x16, fs, settings, chunk_bounds(n, fs, 512))
        y = dyn[i][0] if i in dyn else h_outs[i]
        _cmp(y.numpy(), ref, "TrackStream track %d (%s)" % (i, rinfo["mode"]))


def test_sharded_batch_dynamic(gpu, oracle_mod):
    """ShardedBatch (C4 share, rank 0 of 2): finish_dynamic after the step, outputs by
    global track index"""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.dist import ShardedBatch
    fs = 48000
    settings = dict(bass_boost=1.0, lufs=-14.0)
    xs = [_dynamic_signal(5.0, fs, 41), synth.mix_like(fs * 4, fs, 2, seed=42),
          synth.mix_like(fs * 9, fs, 2, seed=43)]
    frames = [x.shape[0] for x in xs]
    b = ShardedBatch(fs, 2, settings, frames, rank=0, world=2, quantum=512)
    mine = [xs[k] for k in b.tracks]
    d_in = torch.from_numpy(np.ascontiguousarray(np.concatenate(mine))).cuda()
    b.step(d_in)
    info = b.finish_dynamic()
    assert 0 in b.tracks and list(info) == [0]
    for k in b.tracks:
        x16 = oracle_mod.quantize(xs[k])
        ref, rinfo = oracle_mod.pipeline(x16, fs, settings, chunk_bounds(frames[k], fs, 512))
        _cmp(b.track_output(k).cpu().numpy(), ref, "ShardedBatch track %d (%s)" % (k, rinfo["mode"]))


def test_batch_several_dynamic(gpu, oracle_mod):
    """finish_dynamic with several dynamic tracks runs them side by side (a stream and
    192 kHz scratch each); every track still matches its own oracle pipeline"""
    import torch
    from amx import synth
    from amx.chunking import chunk_bounds
    from amx.engine import MasteringJob
    fs = 48000
    settings = dict(bass_boost=1.0, lufs=-14.0)
    xs = [_dynamic_signal(6.0, fs, 51), synth.mix_like(fs * 5, fs, 2, seed=52),
          _dynamic_signal(7.5, fs, 53), _dynamic_signal(4.0, fs, 54, intro=1.5)]
    job = MasteringJob(fs, 2, settings, [x.shape[0] for x in xs], quantum=512)
    job.run(torch.from_numpy(np.ascontiguousarray(np.concatenate(xs))).cuda())
    rep = job.fetch_report(raise_dynamic=False)
    assert rep["modes"] == ["dynamic", "linear", "dynamic", "dynamic"], rep["modes"]
    info = job.finish_dynamic(rep)
    assert sorted(info) == [0, 2, 3] and all(v["sample_rate"] == 192000 for v in info.values())
    for t, x in enumerate(xs):
        x16 = oracle_mod.quantize(x)
        ref, rinfo = oracle_mod.pipeline(x16, fs, settings, chunk_bounds(x16.shape[0], fs, 512))
        _cmp(job.track_output(t).cpu().numpy(), ref, "several-dynamic batch track %d (%s)" % (t, rinfo["mode"]))


@pytest.mark.parametrize("ranks,seg,warm", [(3, None, None), (3, 1, 0), (2, 2, 1)])
def test_shard_parts_vs_oracle(gpu, oracle_mod, monkeypatch, ranks, seg, warm):
    """amx_loudnorm_192k_segments / amx_loudnorm_192k_shard through the C ABI, the
    ranks simulated in order in one process, each with its own scratch: part 0 (its
    192 kHz range + every frame's statistics), part 1 (its segments from guessed
    states), part 2 (its walk from the state record the previous one left).  The runs
    of the 192 kHz output, concatenated, must be the oracle's filter output -- with
    one-frame segments and no warm-up most guesses are wrong, so the records decide."""
    import ctypes
    import torch
    from amx import capi
    from amx.dist import shard_segments
    from amx.engine import MasteringJob
    if seg is not None:
        monkeypatch.setenv("AMX_LN_SEG", str(seg))
        monkeypatch.setenv("AMX_LN_WARM", str(warm))
    fs = 48000
    x = _dynamic_signal(20.0, fs, 17)
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    job = MasteringJob(fs, 2, {"lufs": -14.0}, [x16.shape[0]], input_s16=True,
                       chunks=[(0, 0, x16.shape[0])], measure_only=True)
    job.out[:x16.shape[0]].copy_(torch.from_numpy(x16))
    job.loudness_pass1(tail=False)
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    n192, job2, _, summ = job._job192(0, cached=False)[0:4]
    L = capi.load()
    K, kf, rd, co = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    capi.check(L.amx_loudnorm_192k_segments(job.plan.h, 0, None, 0, ctypes.byref(K), ctypes.byref(kf),
                                            ctypes.byref(rd), ctypes.byref(co)), "segments")
    starts = (ctypes.c_int64 * (K.value + 1))()
    capi.check(L.amx_loudnorm_192k_segments(job.plan.h, 0, starts, K.value + 1, ctypes.byref(K), None, None,
                                            None), "segments")
    starts = list(starts)
    assert starts[0] == 0 and starts[-1] == n192 and all(a < b for a, b in zip(starts, starts[1:]))
    assert 0 < kf.value <= K.value
    # a starts array too small is refused
    small = (ctypes.c_int64 * K.value)()
    assert L.amx_loudnorm_192k_segments(job.plan.h, 0, small, K.value, ctypes.byref(K), None, None, None) != 0
    ranges = shard_segments(K.value, kf.value, ranks)
    nb, wsb = ctypes.c_int64(), ctypes.c_int64()
    capi.check(L.amx_loudnorm_192k_size(job.plan.h, 0, ctypes.byref(nb), ctypes.byref(wsb)), "size")
    ws2s = [torch.empty(wsb.value, dtype=torch.uint8, device=job.device) for _ in range(ranks)]
    recs = [torch.zeros(rd.value, dtype=torch.float64, device=job.device) for _ in range(ranks)]
    for offset in (0.0, 9.0):
        d = capi.LoudnormDesc(-14.0, 11.0, -1.5, float(st["input_i"]), float(st["input_lra"]),
                              float(st["input_tp"]), float(st["input_thresh"]), offset)
        job2.out.zero_()
        for r, (kb, ke) in enumerate(ranges):
            for part in (0, 1, 2):
                sh = capi.LnShard(part, kb, ke, 0, -1, -1, capi.ptr(recs[r - 1]) if r > 0 else None,
                                  capi.ptr(recs[r]) if r < ranks - 1 else None)
                capi.check(L.amx_loudnorm_192k_shard(
                    job.plan.h, 0, ctypes.byref(d), None, None, ctypes.byref(sh), capi.ptr(job.out),
                    capi.ptr(job.hops), int(job.max_hops), capi.ptr(job.peak), capi.ptr(job2.out),
                    capi.ptr(summ), capi.ptr(ws2s[r]), None), "shard")
                ctl = int(ws2s[r][co.value:co.value + 4].view(torch.int32).item())
                assert ctl == 0, (r, part, ctl)          # the parallel form ran, no fallback
        ref, _ = oracle_mod.loudnorm(x16, fs, -14.0, measured=st, offset=offset)
        _cmp(job2.out[:n192].cpu().numpy(), ref, "shard parts x%d Fs=%s Wf=%s offset %.1f" % (ranks, seg, warm, offset))
    # a walk past the first segment without the previous state is refused
    sh = capi.LnShard(2, ranges[1][0], ranges[1][1], 0, -1, -1, None, None)
    assert L.amx_loudnorm_192k_shard(job.plan.h, 0, ctypes.byref(d), None, None, ctypes.byref(sh), capi.ptr(job.out),
                                     capi.ptr(job.hops), int(job.max_hops), capi.ptr(job.peak), capi.ptr(job2.out),
                                     capi.ptr(summ), capi.ptr(ws2s[1]), None) != 0


@pytest.mark.parametrize("ranks,seg,warm,fs", [(3, None, None, 48000), (3, 1, 0, 48000), (2, None, None, 44100)])
def test_shard_windows_vs_oracle(gpu, oracle_mod, monkeypatch, ranks, seg, warm, fs):
    """the windowed shard (amx_loudnorm_192k_shard_window + amx_ln_shard.windowed): each
    simulated rank holds ONLY its windows -- the chain frames its resampler reads, the
    192 kHz stream its segments read (a d_ws2 of the window's size) and the output
    positions they emit -- poisoned outside what it writes; the runs concatenated must be
    the oracle's filter output (within 3 LSB), and equal the whole-track shard's output"""
    import ctypes
    import torch
    from amx import capi
    from amx.dist import shard_segments
    from amx.engine import MasteringJob
    if seg is not None:
        monkeypatch.setenv("AMX_LN_SEG", str(seg))
        monkeypatch.setenv("AMX_LN_WARM", str(warm))
    x = _dynamic_signal(21.0, fs, 29)
    x16 = oracle_mod.quantize(x)
    st = oracle_mod.loudnorm_measure(x16, fs)
    n = x16.shape[0]
    job = MasteringJob(fs, 2, {"lufs": -14.0}, [n], input_s16=True, chunks=[(0, 0, n)], measure_only=True)
    job.out[:n].copy_(torch.from_numpy(x16))
    job.loudness_pass1(tail=False)
    job.loudness_pass2(carry=False)
    job.histograms()
    job.decide()
    n192, job2, ws2_whole, summ = job._job192(0, cached=False)[0:4]
    L = capi.load()
    K, kf, rd, co = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
    capi.check(L.amx_loudnorm_192k_segments(job.plan.h, 0, None, 0, ctypes.byref(K), ctypes.byref(kf),
                                            ctypes.byref(rd), ctypes.byref(co)), "segments")
    ranges = shard_segments(K.value, kf.value, ranks)
    dev = job.device
    wins, bufs = [], []
    for kb, ke in ranges:
        win, b = (ctypes.c_int64 * 9)(), ctypes.c_int64()
        capi.check(L.amx_loudnorm_192k_shard_window(job.plan.h, 0, kb, ke, win, ctypes.byref(b)), "window")
        x0, x1, u0, u1, y0, y1, ctl_off = list(win)[:7]
        assert 0 <= x0 < x1 <= n and 0 <= u0 < u1 <= n192 and u0 <= y0 < y1 <= u1
        xw = torch.from_numpy(np.ascontiguousarray(x16[x0:x1])).to(dev)
        bufs.append((xw, torch.empty(b.value, dtype=torch.uint8, device=dev),
                     torch.empty((y1 - y0, 2), dtype=torch.int16, device=dev)))
        wins.append((x0, x1, u0, u1, y0, y1, ctl_off))
    # a window of no segments is refused
    w0, b0 = (ctypes.c_int64 * 9)(), ctypes.c_int64()
    assert L.amx_loudnorm_192k_shard_window(job.plan.h, 0, 3, 3, w0, ctypes.byref(b0)) != 0
    recs = [torch.zeros(rd.value, dtype=torch.float64, device=dev) for _ in range(ranks)]
    for offset in (0.0, 9.0):
        d = capi.LoudnormDesc(-14.0, 11.0, -1.5, float(st["input_i"]), float(st["input_lra"]),
                              float(st["input_tp"]), float(st["input_thresh"]), offset)
        for r, (kb, ke) in enumerate(ranges):
            xw, ws2, yw = bufs[r]
            ws2.fill_(0xA5)
            yw.fill_(12345)
            for part in (0, 1, 2):
                sh = capi.LnShard(part, kb, ke, 1, -1, -1, capi.ptr(recs[r - 1]) if r > 0 else None,
                                  capi.ptr(recs[r]) if r < ranks - 1 else None)
                capi.check(L.amx_loudnorm_192k_shard(
                    job.plan.h, 0, ctypes.byref(d), None, None, ctypes.byref(sh), capi.ptr(xw),
                    capi.ptr(job.hops), int(job.max_hops), capi.ptr(job.peak), capi.ptr(yw),
                    capi.ptr(summ), capi.ptr(ws2), None), "shard windowed")
                c = wins[r][6]
                ctl = int(ws2[c:c + 4].view(torch.int32).item())
                assert ctl == 0, (r, part, ctl)
        y = np.concatenate([b[2].cpu().numpy() for b in bufs])
        assert y.shape[0] == n192
        ref, _ = oracle_mod.loudnorm(x16, fs, -14.0, measured=st, offset=offset)
        _cmp(y, ref, "shard windows x%d Fs=%s Wf=%s %d Hz offset %.1f" % (ranks, seg, warm, fs, offset))
        # the whole-track buffers' form: the same numbers
        job2.out.zero_()
        for r, (kb, ke) in enumerate(ranges):
            for part in (0, 1, 2):
                sh = capi.LnShard(part, kb, ke, 0, -1, -1, capi.ptr(recs[r - 1]) if r > 0 else None,
                                  capi.ptr(recs[r]) if r < ranks - 1 else None)
                capi.check(L.amx_loudnorm_192k_shard(
                    job.plan.h, 0, ctypes.byref(d), None, None, ctypes.byref(sh), capi.ptr(job.out),
                    capi.ptr(job.hops), int(job.max_hops), capi.ptr(job.peak), capi.ptr(job2.out),
                    capi.ptr(summ), capi.ptr(ws2_whole), None), "shard")
        np.testing.assert_array_equal(y, job2.out[:n192].cpu().numpy())
