"""GPU mastering engine: the host side of the drop-in path.

``MasteringJob`` owns one amx plan (tracks laid back to back, or one rank's
contiguous run of chunks of chunk-sharded tracks), torch-allocated device
buffers and the call sequence of process_audio_with_ffmpeg_pipeline
(audio_mastering_engine.py:171-226):

  chunk chain (:185-204) + concat (:205-214)    -> amx_run_chunks
  loudnorm pass 1 measurement (:229-237)         -> amx_loudness_pass1/pass2/histograms
                                                    + amx/loudness.py host arithmetic
  loudnorm pass 2 linear gain (:240) + alimiter (:223) -> amx_finalize

PyTorch only owns device memory and the stream; every per-sample operation is a
HIP kernel in libamx.so.  There is no CPU fallback: if the library or a GPU is
missing, construction raises.
"""
import math
import os

import numpy as np
import torch

from . import capi, design, loudness
from .chunking import plan_tracks, packet_frames
from .settings import ALIMITER, LOUDNORM_LRA, LOUDNORM_TP


class DynamicModeUnsupported(NotImplementedError):
    """loudnorm takes dynamic mode (192 kHz AGC) on a path that only finalises linear
    tracks (chunk-sharded N > 1, or TrackStream.run without ``dynamic=``): master_audio /
    master_array, MasteringJob.finish_dynamic, ShardedBatch.finish_dynamic and
    TrackStream.run(dynamic={}) run it through MasteringJob.dynamic_track."""


def final_desc(params=ALIMITER):
    fd = capi.FinalDesc()
    fd.limit = params["limit"]
    fd.attack_ms = params["attack"]
    fd.release_ms = params["release"]
    fd.level_in = params["level_in"]
    fd.level_out = params["level_out"]
    fd.auto_level = 1
    return fd


def ln_output_bound(n192):
    """The largest |sample| / 32768 of loudnorm's dynamic-mode output (int16 at 192 kHz):
    its true-peak limiter clamps every sample to the ceiling 10^(TP / 20) (af_loudnorm's
    final clamp), and the WAV muxer rounds to s16.  None for a track under 3 s, which
    takes the linear path (output = input x offset, unclamped).  AMX_LN_MEASURED_BOUND=1:
    None always (the 192 kHz alimiter's input is measured: A/B checks;
    tests/test_gpu_dynamic.py::test_dynamic_output_within_ceiling checks the bound)."""
    import math
    if n192 < 576000 or os.environ.get("AMX_LN_MEASURED_BOUND") == "1":
        return None                     # (< 3 s: frame_size(192000, 3000), the linear fallback)
    c = 10.0 ** (LOUDNORM_TP / 20.0)
    return min(math.floor(c * 32768.0 + 0.5), 32767) / 32768.0


def wait_host_word(ready, what, timeout_s=None):
    """Spin until ready() (a pinned-memory word the device stores, or an event query),
    for at most timeout_s seconds (AMX_WAIT_TIMEOUT_S, default 120): a faulted kernel
    or a hung collective then raises instead of spinning forever."""
    import time
    if ready():
        return
    if timeout_s is None:
        timeout_s = float(os.environ.get("AMX_WAIT_TIMEOUT_S", "120"))
    t_end = time.monotonic() + timeout_s
    n = 0
    while not ready():
        n += 1
        if n & 1023 == 0 and time.monotonic() > t_end:
            raise RuntimeError("amx: %s not ready after %.0f s (a device fault or a hung "
                               "collective?)" % (what, timeout_s))


class MasteringJob:
    def __init__(self, sample_rate, channels_in, settings, track_frames, *, quantum=None,
                 input_s16=False, seg_frames=128, device=None, chunks=None, track_frame0=None,
                 track_total=None, limiter=ALIMITER, limiter_seg_frames=0,
                 limiter_warm_frames=-1, measure_only=False):
        if not torch.cuda.is_available():
            raise RuntimeError("amx needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device or "cuda")
        self.fs = int(sample_rate)
        self.settings = dict(settings)
        self.channels_in = int(channels_in)
        self.input_s16 = bool(input_s16)
        self.desc, self._keep = design.chain_desc(self.fs, self.channels_in, self.settings)
        self.desc.input_s16 = 1 if input_s16 else 0
        self.desc.measure_only = 1 if measure_only else 0
        if quantum is None:
            quantum = packet_frames(self.channels_in * (2 if input_s16 else 4))
        self.track_frames = [int(n) for n in track_frames]
        self.chunks = chunks if chunks is not None else plan_tracks(self.track_frames, self.fs, quantum)
        self.plan = capi.Plan(self.desc, self.chunks, track_frame0, track_total, seg_frames)
        info = self.plan.info
        self.info = info
        self.n_tracks = info.n_tracks
        dev = self.device
        self.ws = torch.empty(max(1, info.workspace_bytes), dtype=torch.uint8, device=dev)
        self.out = torch.empty((max(1, info.out_frames), 2), dtype=torch.int16, device=dev)
        self.y = torch.empty_like(self.out)
        T = max(1, self.n_tracks)
        self.spans = [self.plan.span(t) for t in range(self.n_tracks)]
        self.hop = info.hop_frames                 # 100 ms of the 192 kHz measurement stream
        self.max_hops = max(1, int(info.max_hops))
        self.kw_tail = torch.zeros((T, 2, 4), dtype=torch.float64, device=dev)
        self.kw_carry = torch.zeros((T, 2, 4), dtype=torch.float64, device=dev)
        # per track: the measured (192 kHz) stream's sample peak L, R; d_out's own L, R
        self.peak = torch.zeros((T, 4), dtype=torch.float64, device=dev)
        # the 16 d_out frames before / after a span inside its track (chunk-sharded
        # ranks: the neighbours' frames the resampler window reaches); unused otherwise
        self.edge = torch.zeros((T, 2, capi.UP_EDGE, 2), dtype=torch.int16, device=dev)
        self.needs_edge = any(s.track_frame0 > 0 or s.track_frame0 + s.out_frames < s.track_frames_total
                              for s in self.spans)
        self.hops = torch.zeros((T, self.max_hops, 2), dtype=torch.float64, device=dev)
        self.hist = torch.zeros((T, 1000), dtype=torch.int64, device=dev)
        self.st_hist = torch.zeros((T, 1000), dtype=torch.int64, device=dev)
        self.gains = torch.full((T,), -1.0, dtype=torch.float64, device=dev)
        self.stats = torch.zeros((T, capi.STATS), dtype=torch.float64, device=dev)
        self.ctl = torch.zeros((T,), dtype=torch.int32, device=dev)
        self.dd = capi.DecideDesc()
        lufs = self.settings.get("lufs")
        self.dd.lufs_on = 0 if lufs is None else 1
        self.dd.target_i = 0.0 if lufs is None else float(lufs)
        self.dd.target_tp = LOUDNORM_TP
        self.dd.target_lra = LOUDNORM_LRA
        self.fd = final_desc(limiter)
        self.limit = limiter["limit"]
        self.bs, self.halo_frames, self.state_doubles = self.plan.limiter_geometry(self.fd)
        self.halo = torch.zeros((T, max(1, self.halo_frames), 2), dtype=torch.int16, device=dev)
        self.lim_state = torch.zeros((T, self.state_doubles), dtype=torch.float64, device=dev)
        # general-path limiter segments: allocated now, never inside a graph capture
        self.plan.limiter_prepare(self.fd, limiter_seg_frames, limiter_warm_frames)
        self._i_out = torch.zeros((T,), dtype=torch.float64, device=dev)   # pass 1's output I (dynamic)
        self._dyn_sides = None     # per track, the 192 kHz sets run() enqueues (prepare_dynamic)
        self._dyn_eager = False
        self.report = {}

    # ------------------------------------------------------------ device steps
    @staticmethod
    def _s(stream):
        import ctypes
        s = stream if stream is not None else torch.cuda.current_stream()
        return ctypes.c_void_p(s.cuda_stream)

    def run_chunks(self, d_in, stream=None):
        want = torch.int16 if self.input_s16 else torch.float32
        if d_in.dtype != want or not d_in.is_contiguous() or d_in.device.type != "cuda":
            raise TypeError("d_in must be a contiguous %s CUDA tensor" % want)
        need = max((off + n for (_, off, n) in self.chunks), default=0)
        if d_in.numel() < need * self.channels_in:
            raise ValueError("d_in holds %d samples, plan needs %d" % (d_in.numel(), need * self.channels_in))
        L = capi.load()
        ev = getattr(self, "stage_events", None)
        if ev is None:
            capi.check(L.amx_run_chunks(self.plan.h, capi.ptr(d_in), capi.ptr(self.out),
                                        capi.ptr(self.ws), self._s(stream)), "amx_run_chunks")
            return
        # per-stage timing: events recorded on the stream the kernels run on
        for s in range(len(capi.STAGES)):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record(stream)
            capi.check(L.amx_run_stage(self.plan.h, s, capi.ptr(d_in), capi.ptr(self.out),
                                       capi.ptr(self.ws), self._s(stream)), "amx_run_stage")
            b.record(stream)
            ev.append((capi.STAGES[s], a, b))

    def timed(self, name, fn, stream=None):
        """Run fn() between two HIP events on the launch stream when stage timing is on
        (self.stage_events is a list), else just run it."""
        ev = getattr(self, "stage_events", None)
        if ev is None:
            return fn()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(stream)
        r = fn()
        b.record(stream)
        ev.append((name, a, b))
        return r

    def loudness_pass1(self, stream=None, tail=True, part=None):
        """tail: also the K-filter end state from rest (only a chunk-sharded track's
        next rank needs it).  part 0 / 1: one of the two launches of the pass (the
        sample pass / peaks + scan), None: both."""
        for p in ((0, 1) if part is None else (part,)):
            capi.check(capi.load().amx_loudness_pass1_part(
                self.plan.h, p, capi.ptr(self.out), capi.ptr(self.edge) if self.needs_edge else None,
                capi.ptr(self.kw_tail) if tail else None, capi.ptr(self.peak), capi.ptr(self.ws),
                self._s(stream)), "amx_loudness_pass1_part")

    def loudness_pass2(self, stream=None, carry=True):
        capi.check(capi.load().amx_loudness_pass2(self.plan.h, capi.ptr(self.out),
                                                  capi.ptr(self.edge) if self.needs_edge else None,
                                                  capi.ptr(self.kw_carry) if carry else None,
                                                  capi.ptr(self.hops), int(self.max_hops),
                                                  capi.ptr(self.ws), self._s(stream)),
                   "amx_loudness_pass2")

    def histograms(self, stream=None):
        capi.check(capi.load().amx_loudness_histograms(self.plan.h, capi.ptr(self.hops), int(self.max_hops),
                                                       capi.ptr(self.hist), capi.ptr(self.st_hist),
                                                       capi.ptr(self.ws), self._s(stream)),
                   "amx_loudness_histograms")

    def decide(self, stream=None):
        """loudnorm statistics, mode, gain and limiter path on the device (no sync)."""
        lufs_on = self.dd.lufs_on
        capi.check(capi.load().amx_loudness_decide(
            self.plan.h, self.dd, self.fd, capi.ptr(self.hist) if lufs_on else None,
            capi.ptr(self.st_hist) if lufs_on else None, capi.ptr(self.peak), capi.ptr(self.stats),
            capi.ptr(self.gains), capi.ptr(self.ctl), self._s(stream)), "amx_loudness_decide")

    def publish_ctl(self, host, stream=None):
        """the tracks' decision words into the pinned host tensor `host` (amx_publish_ctl:
        device stores, no copy node), on the stream"""
        import ctypes
        capi.check(capi.load().amx_publish_ctl(capi.ptr(self.ctl), ctypes.c_void_p(host.data_ptr()),
                                               int(self.n_tracks), self._s(stream)), "amx_publish_ctl")

    def finalize(self, fast=None, stream=None, state=None, from_rest=False):
        """fast None: each track takes the limiter path amx_loudness_decide chose.
        state: the limiter state buffer (default self.lim_state): read as the state
        entering the span, and the span's end state written back to it.  from_rest:
        the entering state is not read -- every span starts from rest with its halo
        (amx_final_desc.from_rest: the speculative first run of the rank-to-rank
        hand-off, with no zero fill before it)."""
        ctl = capi.ptr(self.ctl) if fast is None else None
        st = self.lim_state if state is None else state
        fd = self.fd
        if from_rest:
            fd = capi.FinalDesc.from_buffer_copy(self.fd)
            fd.from_rest = 1
        capi.check(capi.load().amx_finalize(self.plan.h, fd, capi.ptr(self.out), capi.ptr(self.gains),
                                            ctl, 1 if fast else 0, capi.ptr(self.halo), capi.ptr(self.y),
                                            capi.ptr(st), capi.ptr(self.ws), self._s(stream)),
                   "amx_finalize")

    def env_counters(self):
        """Compressor fix-up diagnostics of the last step (amx_env_counters): segments
        re-run by the chain walkers, the longest walk (segments re-run one after
        another by one wave), chains, and the segments of the optimistic parallel
        pass before them.  Synchronous."""
        import ctypes
        n = 16 * 4
        buf = (ctypes.c_int32 * n)()
        capi.check(capi.load().amx_env_counters(self.plan.h, capi.ptr(self.ws), buf, n), "amx_env_counters")
        rows = [list(buf[4 * r:4 * r + 4]) for r in range(16)]
        keys = ("reruns", "max_chain", "chains", "wide")
        return [dict(zip(keys, r)) for r in rows if any(r)]

    # --------------------------------------------- loudnorm dynamic mode (192 kHz)
    def _job192(self, t, cached=True):
        """the 192 kHz side of track t: a measure-only plan at 192 kHz holding the
        filter's output (its loudness measurement gives pass 1's target_offset; its
        alimiter is the reference's :223 on the 192 kHz file) + amx_loudnorm_192k's
        scratch.  cached: kept for the next call on the same track (one at a time);
        else a fresh set, so several tracks can run at once (finish_dynamic)."""
        import ctypes
        n192, wsb = ctypes.c_int64(), ctypes.c_int64()
        capi.check(capi.load().amx_loudnorm_192k_size(self.plan.h, t, ctypes.byref(n192), ctypes.byref(wsb)),
                   "amx_loudnorm_192k_size")
        key = (t, n192.value)
        if not cached or getattr(self, "_j192", None) is None or self._j192[0] != key:
            job2 = MasteringJob(192000, 2, {"lufs": self.settings.get("lufs")}, [n192.value],
                                input_s16=True, chunks=[(0, 0, n192.value)], device=self.device,
                                measure_only=True, seg_frames=1024)   # the K scan's window at 192 kHz
            ws2 = torch.empty(max(1, wsb.value), dtype=torch.uint8, device=self.device)
            summ = torch.zeros(16, dtype=torch.float64, device=self.device)
            if not cached:
                return n192.value, job2, ws2, summ
            self._j192 = (key, job2, ws2, summ)
        return n192.value, self._j192[1], self._j192[2], self._j192[3]

    def loudnorm_192k(self, t, desc, job2, ws2, summ, stream=None, measured=None, offset_i=None, gate=None):
        """amx_loudnorm_192k_ex: measured / offset_i / gate are device rows (None: desc's
        host values, no gate) -- see include/amx.h"""
        import ctypes
        capi.check(capi.load().amx_loudnorm_192k_ex(
            self.plan.h, t, ctypes.byref(desc), capi.ptr(measured), capi.ptr(offset_i), capi.ptr(gate),
            capi.ptr(self.out), capi.ptr(self.hops), int(self.max_hops), capi.ptr(self.peak), capi.ptr(job2.out),
            capi.ptr(summ), capi.ptr(ws2), self._s(stream)), "amx_loudnorm_192k")

    def dynamic_track(self, t, stats=None, stream=None, filt=None):
        """loudnorm's dynamic mode for track t (:240 when the linear conditions fail), as
        the reference's two ffmpeg passes run it: pass 1's filter with the measured_*
        defaults, whose output loudness gives target_offset; pass 2's filter with the
        pass-1 strings; then the alimiter (:223) at 192 kHz.  Returns (int16 [n192, 2] at
        192 kHz, info).  Every step is on the device, without a host round trip (the
        "%.2f" strings pass 2 parses are formed there); the host reads the result."""
        run = self._dyn_enqueue(t, self._job192(t, cached=True), stream, filt=filt)
        return self._dyn_result(run, stream)

    def _dyn_enqueue(self, t, side, stream, gate=False, filt=None):
        """Both passes of the dynamic path for track t, enqueued on `stream`: pass 1's
        filter with the measured_* defaults and the 192 kHz measurement of its output
        (its integrated loudness is pass 1's target_offset); pass 2's filter with the
        track's own pass-1 statistics (k_decide's "%.2f" values) and that offset; the
        192 kHz measurement of its output (the alimiter's input bound) and the alimiter.
        side: the 192 kHz set of _job192 (made beforehand: a plan's creation synchronises
        the device).  gate: every loudnorm kernel first checks the track's control word
        and returns unless it says dynamic (a captured step holds the path for whichever
        tracks need it).  filt(desc, measured, offset_i): the filter run in place of
        amx_loudnorm_192k_ex (ShardedTrack's segment-sharded run)."""
        n192, job2, ws2, summ = side
        reuse = filt is None
        if filt is None:
            def filt(desc, measured, offset_i):
                self.loudnorm_192k(t, desc, job2, ws2, summ, stream, measured=measured, offset_i=offset_i,
                                   gate=g)
        target = float(self.settings["lufs"])
        g = self.ctl[t:t + 1] if gate else None
        d1 = capi.LoudnormDesc(target, LOUDNORM_LRA, LOUDNORM_TP, 0.0, 0.0, 99.0, -70.0, 0.0)
        self.timed("ln_filter1", lambda: filt(d1, None, None), stream)

        def measure1():
            job2.loudness_pass1(stream, tail=False)
            job2.loudness_pass2(stream, carry=False)
            job2.histograms(stream)
            job2.dd.lufs_on = 1
            job2.decide(stream)
            with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream()):
                self._i_out[t:t + 1].copy_(job2.stats[0, 0:1])       # pass 1's output loudness
        self.timed("ln_measure1", measure1, stream)
        d2 = capi.LoudnormDesc(target, LOUDNORM_LRA, LOUDNORM_TP, 0.0, 0.0, 99.0, -70.0, 0.0)
        # pass 2 filters the same input on the same scratch: pass 1's 192 kHz stream stands
        d2.reuse_stream = 1 if reuse else 0
        self.timed("ln_filter2", lambda: filt(d2, self.stats[t], self._i_out[t:t + 1]), stream)

        def limit():
            # the limiter's input bound: af_loudnorm clamps every limited output sample to
            # its ceiling, so that is the bound without a pass over the 192 kHz samples
            # (a track under 3 s takes the unlimited linear path: measured)
            bound = ln_output_bound(n192)
            if bound is not None:
                with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream()):
                    job2.peak.fill_(bound)
            else:
                job2.loudness_pass1(stream, tail=False)
            job2.dd.lufs_on = 0
            job2.decide(stream)
            job2.finalize(None, stream)
        self.timed("ln_limit192", limit, stream)
        return {"t": t, "n192": n192, "job2": job2, "ws2": ws2, "summ": summ}

    def _dyn_result(self, run, stream):
        with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream()):
            prof = run["summ"].cpu().numpy()
            i_out = float(self._i_out[run["t"]].item())
        target = float(self.settings["lufs"])
        info = {"target_offset": loudness._fmt(target - i_out), "pass1_output_i": i_out,
                "sample_rate": 192000}
        if prof[12] > 0 and prof[13] == 0:
            # the parallel form (amx_loudnorm.hip k_lp_*): its walker's diagnostics
            info["pass2_parallel"] = {"segments": int(prof[12]), "reruns": int(prof[10]),
                                      "final_rerun": bool(prof[11])}
        else:
            info["pass2_cycles"] = {k: float(prof[i]) for i, k in enumerate(
                ("fill", "detect", "envelope", "output", "stats", "r128_out",
                 "detect_calls", "serial_chunks"), start=2)}
        return run["job2"].y[:run["n192"]], info

    # ------------------------------------------------------------ report
    def fetch_report(self, raise_dynamic=True):
        """Synchronise and read the device decision back: loudnorm statistics as the
        JSON strings ffmpeg prints, mode, gain, limiter path.  Raises
        DynamicModeUnsupported when loudnorm would have used dynamic mode."""
        st = self.stats.cpu().numpy()
        stats, modes, gains, fast = [], [], [], []
        for t in range(self.n_tracks):
            row = st[t]
            mode = capi.MODES[int(row[8])]
            modes.append(mode)
            gains.append(float(row[9]))
            fast.append(bool(row[10]))
            if self.dd.lufs_on:
                stats.append({"input_i": loudness._fmt(row[4]), "input_tp": loudness._fmt(row[5]),
                              "input_lra": loudness._fmt(row[6]), "input_thresh": loudness._fmt(row[7])})
            if mode == "dynamic" and raise_dynamic:
                raise DynamicModeUnsupported(
                    "loudnorm takes dynamic mode for these measurements %s: finish the track "
                    "with dynamic_track() (master_audio / master_array do)" % (stats[-1],))
        self.report.update({"stats": stats if self.dd.lufs_on else None, "modes": modes,
                            "gains": gains, "limiter_fast": all(fast)})
        return self.report

    def run(self, d_in, stream=None, dyn=True, ctl_to=None):
        """Whole pipeline for whole tracks on this GPU, fully on the stream (no host
        round trip); returns y (int16 [frames, 2]).  fetch_report() reads the
        loudness decision afterwards.  dyn False: without the gated dynamic path
        (capture puts it in a graph of its own); ctl_to: a pinned host tensor the
        decision words are copied to as soon as they are made (before the limiter)."""
        self.run_chunks(d_in, stream)
        self.timed("up", lambda: self.loudness_pass1(stream, tail=False, part=0), stream)
        self.timed("loud1", lambda: self.loudness_pass1(stream, tail=False, part=1), stream)
        if self.dd.lufs_on:
            self.timed("loud2", lambda: self.loudness_pass2(stream, carry=False), stream)
            self.timed("hist", lambda: self.histograms(stream), stream)
        self.timed("decide", lambda: self.decide(stream), stream)
        if ctl_to is not None:
            self.publish_ctl(ctl_to, stream)
        self.timed("final", lambda: self.finalize(None, stream), stream)
        if self._dyn_sides and dyn:
            # the dynamic path of every track, gated on the device by the track's decision
            # (a linear track's kernels return at once): the step needs no host round trip
            # whichever mode loudnorm takes
            for t, side in enumerate(self._dyn_sides):
                self._dyn_enqueue(t, side, stream, gate=True)
        self.report = {"chunks": len(self.chunks), "segments": self.info.n_segments}
        return self.y[:self.info.out_frames]

    def prepare_dynamic(self):
        """Make run() (and a graph captured from it) hold loudnorm's dynamic path for every
        track, gated on the device: the 192 kHz plans and scratch are made here, outside
        any capture.  Afterwards dynamic_output(t) is track t's 192 kHz result when the
        step's decision was dynamic."""
        if self.dd.lufs_on and self._dyn_sides is None:
            self._dyn_sides = [self._job192(t, cached=False) for t in range(self.n_tracks)]
            # the side plan's 192 kHz measurement passes and alimiter return at once for a
            # track whose decision is not dynamic (a linear batch paid them)
            for t, (_, job2, _, _) in enumerate(self._dyn_sides):
                job2.plan.set_gate(self.ctl[t:t + 1])

    def dynamic_output(self, t, stream=None):
        """after a step with prepare_dynamic(): (int16 [n192, 2], info) of track t if its
        loudnorm took dynamic mode, else None (synchronises the stream)"""
        if not self._dyn_sides:
            return None
        mode = capi.MODES[int(self.stats[t, 8].item())]
        if mode != "dynamic":
            return None
        n192, job2, ws2, summ = self._dyn_sides[t]
        return self._dyn_result({"t": t, "n192": n192, "job2": job2, "ws2": ws2, "summ": summ}, stream)

    def capture(self, d_in, dynamic=False, dyn_graph=None):
        """Record run(d_in) as one hipGraph (torch.cuda.CUDAGraph over the HIP stream
        capture): replay() then re-issues the whole pipeline -- every kernel, same
        buffers -- with one launch, so the host's per-kernel launch cost is off the
        critical path.  run() has no host round trip, so the captured graph is the
        complete step.  dynamic: the step also holds loudnorm's dynamic path
        (prepare_dynamic), so a track that takes it is finished inside the step too --
        enqueued by replay() after the graph, for the tracks whose published decision
        word says dynamic (AMX_DYN_INLINE=1: gated inside the graph instead).
        dyn_graph (default AMX_DYN_GRAPH, off): that path of each track is captured into
        a graph of its own as well, and replay() launches the track's graph instead of
        the ~35 eager launches.  (Round 5 measured such a graph 10-20x slower with walker
        re-runs: a captured hipMemsetAsync's fill node left the filter's boundary
        counters full of garbage on some replays.  The library zeroes with kernels since
        round 6, and the graph then equals the eager launches bit for bit and in time,
        profiles/r06c_dyn_graph_probe_zero_kernel.log.)"""
        self._dyn_eager = False
        self._dyn_graphs = None
        if dyn_graph is None:
            dyn_graph = os.environ.get("AMX_DYN_GRAPH") == "1"
        if dynamic:
            self.prepare_dynamic()
        dyn = bool(self._dyn_sides)
        if os.environ.get("AMX_DYN_INLINE") == "1":
            dyn = False      # (diagnostics: the gated dynamic path inside the step's graph)
        if dyn:
            # k_decide stores the decision words here as well (amx_plan_set_publish): the
            # host reads them while the limiter kernel still runs
            self._ctl_pin = torch.full((max(1, self.n_tracks),), -1, dtype=torch.int32).pin_memory()
            self.plan.set_publish(self._ctl_pin)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self.run(d_in)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # thread_local: other threads (a process group's watchdog) may query events meanwhile
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self.run(d_in, dyn=not dyn)
        self._graph = g
        self._dyn_eager = dyn
        if dyn and dyn_graph:
            # the gated dynamic path of each track as a graph of its own (warmed up on
            # the side stream first, as torch's capture wants)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for t in range(self.n_tracks):
                    self._dyn_enqueue(t, self._dyn_sides[t], None, gate=True)
            torch.cuda.current_stream().wait_stream(s)
            self._dyn_graphs = []
            for t in range(self.n_tracks):
                gt = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gt, capture_error_mode="thread_local"):
                    self._dyn_enqueue(t, self._dyn_sides[t], None, gate=True)
                self._dyn_graphs.append(gt)
        return g

    def replay(self):
        """One step from the captured graph.  With the dynamic path (capture(dynamic=True))
        the graph publishes the decision words to pinned memory before its limiter kernel
        (device stores: they land while that kernel still runs); the host then enqueues
        the gated dynamic path, eagerly, only for a track whose word says dynamic, so a
        linear step pays none of its ~35 launches per track.  (A graph of its own for
        that path replayed 10-20x slower than the same launches made eagerly, with
        walker re-runs: profiles/r05_dyn_graph.txt.)"""
        if not getattr(self, "_dyn_eager", False):
            self._graph.replay()
            return self.y[:self.info.out_frames]
        h = self._ctl_pin
        h.fill_(-1)                 # (the previous step's words were read: its decide has run)
        self._graph.replay()
        hv = h.numpy()[:self.n_tracks]
        wait_host_word(lambda: not (hv == -1).any(), "the step's decision words")
        dyn = [t for t in range(self.n_tracks) if (int(hv[t]) >> 4) & 15 == 3]   # k_decide mode 3
        for t in dyn:
            if self._dyn_graphs is not None:
                self._dyn_graphs[t].replay()
            else:
                self._dyn_enqueue(t, self._dyn_sides[t], None, gate=True)
        return self.y[:self.info.out_frames]

    def finish_dynamic(self, report=None):
        """After a step of whole tracks: every track loudnorm sends to dynamic mode is
        finished by dynamic_track (its 192 kHz output replaces the slot the step wrote);
        returns {track: info}."""
        rep = report if report is not None else self.fetch_report(raise_dynamic=False)
        self.dyn_out = {}
        dyn = [t for t, mode in enumerate(rep["modes"]) if mode == "dynamic"]
        if len(dyn) == 1:
            y, info = self.dynamic_track(dyn[0], rep["stats"][dyn[0]])
            self.dyn_out[dyn[0]] = (y.clone(), info)
        elif dyn:
            # Several tracks: each on a stream of its own with its own 192 kHz scratch.  A
            # filter run is one workgroup working in order, so the tracks' runs go side by
            # side on different CUs instead of one after another.  Pass 2 of a track is
            # enqueued as soon as its own pass 1 has been read back.
            # The 192 kHz plans are made first: creating one synchronises the device.
            sides = [self._job192(t, cached=False) for t in dyn]
            cur = torch.cuda.current_stream(self.device)
            runs = []
            for t, side in zip(dyn, sides):
                st = torch.cuda.Stream(device=self.device)   # (HIP spreads streams over its hardware queues)
                st.wait_stream(cur)
                runs.append((st, self._dyn_enqueue(t, side, st)))
            for st, run in runs:
                y, info = self._dyn_result(run, st)
                cur.wait_stream(st)
                self.dyn_out[run["t"]] = (y.clone(), info)
        return {t: v[1] for t, v in self.dyn_out.items()}

    def close(self):
        """Release what the job holds on the device, the captured graph first (its nodes
        use the plan's tables and the job's buffers), then the 192 kHz side jobs and the
        plan.  Idempotent; the job is unusable afterwards.  `with MasteringJob(...) as
        job:` calls it."""
        if getattr(self, "_closed", False):
            return
        self._closed = True
        torch.cuda.synchronize(self.device)
        self._graph = None
        self._dyn_graphs = None
        self._dyn_eager = False
        side_jobs = [side[1] for side in (self._dyn_sides or [])]     # (n192, job2, ws2, summ)
        j192 = getattr(self, "_j192", None)                            # (key, job2, ws2, summ)
        if j192 is not None:
            side_jobs.append(j192[1])
        self._dyn_sides = self._j192 = None
        for job2 in side_jobs:
            job2.close()
        if getattr(self, "_ctl_pin", None) is not None and self.plan.h:
            self.plan.set_publish(None)
        self.plan.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def track_output(self, t):
        """track t's output: its slot of y, or its 192 kHz output after finish_dynamic"""
        dyn = getattr(self, "dyn_out", None)
        if dyn and t in dyn:
            return dyn[t][0]
        s = self.spans[t]
        return self.y[s.out_offset:s.out_offset + s.out_frames]


class MultiChannelJob:
    """One whole track with 3..8 channels (missing item 1).

    The reference keeps such a chunk as ONE interleaved 1-D stream
    (audio_segment_to_float_array reshapes only stereo, :252): analog character, EQ and
    crossover run along it (:264-265, :274, :303), width leaves it alone (:268), and
    pydub's compressor and overlay work on frames of C samples (:306-309); then ffmpeg
    concatenates, measures loudness over the C channels (libebur128's default channel
    map) and limits them together (:216-223).  On the GPU:
      amx_mc_run_chunks      -- the chain (stream sub-plans + C-sample compressor);
      amx_mc_split_pairs     -- the output's channel pairs as the tracks of a stereo
                                measure plan (loudness pass 1 / 2 per channel);
      amx_mc_loudness_combine -- one track's hop energies with the channel weights, and
                                its peaks; histograms and the decision on a one-track plan;
      amx_mc_peak_pick + amx_finalize (att trace) + amx_mc_limiter_out -- the alimiter:
                                its state depends only on each frame's largest |sample|.
    Loudnorm's dynamic mode (:240 when the linear conditions fail) is not run for C > 2:
    finish() raises DynamicModeUnsupported.  Parity: the chain is pinned bit-exact to the
    reference's own chunk body (tests/golden/mc*.npz); the measurement's channel weights
    and the C-channel alimiter are parity unpinned (ffmpeg is absent), checked against
    the oracle's restatement (oracle/amx_oracle.c)."""

    def __init__(self, sample_rate, channels, settings, frames, *, quantum=None, input_s16=False,
                 seg_frames=128, device=None, chunks=None, limiter=ALIMITER):
        if not torch.cuda.is_available():
            raise RuntimeError("amx needs a ROCm GPU (torch.cuda.is_available() is False)")
        C = int(channels)
        if not 3 <= C <= 8:
            raise ValueError("MultiChannelJob takes 3..8 channels (%d): MasteringJob takes 1 or 2" % C)
        self.device = torch.device(device or "cuda")
        self.fs, self.C = int(sample_rate), C
        self.settings = dict(settings)
        self.input_s16 = bool(input_s16)
        self.desc, self._keep = design.chain_desc(self.fs, C, self.settings)
        self.desc.input_s16 = 1 if input_s16 else 0
        if quantum is None:
            quantum = packet_frames(C * (2 if input_s16 else 4))
        self.frames = int(frames)
        self.chunks = chunks if chunks is not None else plan_tracks([self.frames], self.fs, quantum)
        self.plan = capi.McPlan(self.desc, self.chunks, seg_frames)
        n = self.out_frames = int(self.plan.out_frames)
        dev = self.device
        self.ws = torch.empty(max(1, self.plan.workspace_bytes), dtype=torch.uint8, device=dev)
        self.out = torch.empty((max(1, n), C), dtype=torch.int16, device=dev)
        self.y = torch.empty_like(self.out)
        P = (C + 1) // 2
        lufs = self.settings.get("lufs")
        m = max(1, n)
        self.meas = MasteringJob(self.fs, 2, {"lufs": lufs}, [m] * P, input_s16=True,
                                 chunks=[(p, p * m, m) for p in range(P)], device=dev, measure_only=True,
                                 limiter=limiter)
        self.one = MasteringJob(self.fs, 2, {"lufs": lufs}, [m], input_s16=True, chunks=[(0, 0, m)],
                                device=dev, measure_only=True, limiter=limiter)
        assert self.meas.max_hops == self.one.max_hops
        self.att = torch.ones(m, dtype=torch.float64, device=dev)
        capi.check(capi.load().amx_plan_set_limiter_trace(self.one.plan.h, capi.ptr(self.att)),
                   "amx_plan_set_limiter_trace")
        self.report = {}

    _s = staticmethod(MasteringJob._s)

    def run_chunks(self, d_in, stream=None):
        """:185-214 -- every chunk's chain, the concat in self.out [out_frames, C]"""
        want = torch.int16 if self.input_s16 else torch.float32
        if d_in.dtype != want or not d_in.is_contiguous() or d_in.device.type != "cuda":
            raise TypeError("d_in must be a contiguous %s CUDA tensor" % want)
        need = max((off + k for (_, off, k) in self.chunks), default=0)
        if d_in.numel() < need * self.C:
            raise ValueError("d_in holds %d samples, plan needs %d" % (d_in.numel(), need * self.C))
        capi.check(capi.load().amx_mc_run_chunks(self.plan.h, capi.ptr(d_in), capi.ptr(self.out),
                                                 capi.ptr(self.ws), self._s(stream)), "amx_mc_run_chunks")

    def measure(self, stream=None, lufs_on=None):
        """loudnorm pass 1's measurement (:229) over the C channels: every channel's 192 kHz
        K-weighted hop energies and peaks (the pairs as tracks), combined with the channel
        weights into the one-track plan; its histograms (lufs on) and decision"""
        L = capi.load()
        s = self._s(stream)
        n = self.out_frames
        one, meas = self.one, self.meas
        if lufs_on is None:
            lufs_on = one.dd.lufs_on
        one.dd.lufs_on = 1 if lufs_on else 0
        capi.check(L.amx_mc_split_pairs(capi.ptr(self.out), n, self.C, capi.ptr(meas.out), s),
                   "amx_mc_split_pairs")
        meas.loudness_pass1(stream, tail=False)
        if lufs_on:
            meas.loudness_pass2(stream, carry=False)
        capi.check(L.amx_mc_loudness_combine(capi.ptr(meas.hops), int(meas.max_hops), capi.ptr(meas.peak),
                                             self.C, capi.ptr(one.hops), capi.ptr(one.peak), s),
                   "amx_mc_loudness_combine")
        if lufs_on:
            one.histograms(stream)
        one.decide(stream)

    def finalize(self, stream=None):
        """:240's linear gain and :223's alimiter on the C channels -> self.y"""
        L = capi.load()
        s = self._s(stream)
        one = self.one
        capi.check(L.amx_mc_peak_pick(capi.ptr(self.out), self.out_frames, self.C, capi.ptr(one.gains),
                                      capi.ptr(one.out), s), "amx_mc_peak_pick")
        one.finalize(None, stream)
        capi.check(L.amx_mc_limiter_out(one.plan.h, one.fd, capi.ptr(self.out), self.C, capi.ptr(one.gains),
                                        capi.ptr(one.ctl), capi.ptr(self.att), capi.ptr(self.y), s),
                   "amx_mc_limiter_out")
        return self.y[:self.out_frames]

    def fetch_report(self, raise_dynamic=True):
        rep = self.one.fetch_report(raise_dynamic=False)
        if raise_dynamic and rep["modes"] and rep["modes"][0] == "dynamic":
            raise DynamicModeUnsupported(
                "loudnorm takes dynamic mode for these measurements %s; the 192 kHz dynamic path "
                "runs on 1- and 2-channel files only" % (rep["stats"],))
        self.report = dict(rep, channels=self.C)
        return self.report

    def run(self, d_in, stream=None):
        """the whole pipeline (:171-226) on the stream; returns y int16 [frames, C]"""
        self.run_chunks(d_in, stream)
        self.measure(stream)
        return self.finalize(stream)

    def close(self):
        if getattr(self, "_closed", False):
            return
        self._closed = True
        torch.cuda.synchronize(self.device)
        self.meas.close()
        self.one.close()
        self.plan.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False


def master_array(x, sample_rate, settings, *, quantum=None, seg_frames=128, limiter_seg_frames=0,
                 limiter_warm_frames=-1):
    """In-memory twin of master_audio: float32 [frames, C] (C = 1/2,
    any device) -> int16 [frames', 2] CUDA tensor (the 16-bit WAV the reference
    writes) and a report dict."""
    x = torch.as_tensor(x)
    if x.dim() == 1:
        x = x.reshape(-1, 1)
    if x.dtype == torch.int16:
        s16 = True
    else:
        s16 = False
        x = x.to(torch.float32)
    x = x.contiguous().to("cuda")
    if x.shape[1] > 2:
        # 3..8 channels: one interleaved stream through the chain (:252)
        job = MultiChannelJob(sample_rate, x.shape[1], settings, x.shape[0], quantum=quantum,
                              input_s16=s16, seg_frames=seg_frames)
        y = job.run(x)
        job.fetch_report(raise_dynamic=True)
        job.report.update(sample_rate=job.fs, job=job)
        return y, job.report
    job = MasteringJob(sample_rate, x.shape[1], settings, [x.shape[0]], quantum=quantum,
                       input_s16=s16, seg_frames=seg_frames, limiter_seg_frames=limiter_seg_frames,
                       limiter_warm_frames=limiter_warm_frames)
    y = job.run(x)
    rep = job.fetch_report(raise_dynamic=False)
    if rep["modes"] and rep["modes"][0] == "dynamic":
        # loudnorm pass 2 in dynamic mode (:240): the 192 kHz path replaces the linear
        # step's output (run() finalised the track without a gain; it is recomputed here)
        y, info = job.dynamic_track(0, rep["stats"][0])
        job.report.update(dynamic=info, sample_rate=info["sample_rate"])
    else:
        job.report["sample_rate"] = job.fs
    job.report["job"] = job
    return y, job.report
