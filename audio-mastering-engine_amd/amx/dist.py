"""Chunk-sharded multi-GPU mastering: one process per GPU, torch.distributed
(backend "nccl" = RCCL over xGMI on ROCm; "gloo" for CPU tests).

A track is cut into ~30 s chunks exactly as on one GPU (the ffmpeg segment rule,
audio_mastering_engine.py:178); rank r owns a contiguous run of chunks.  The chunk
chain needs no communication (all DSP state resets per chunk, :185-204).  The
exchange steps are the track-level ones:

0. Edges: the loudness measurement resamples the track to 192 kHz (ffmpeg's
   pass 1), whose 32-tap window reaches 16 frames into each neighbour's span, and
   the alimiter's look-ahead needs the previous rank's last B - 1 frames: one
   all-gather of every rank's first and last frames, right after the chunk chain.
1. K-filter carry (loudnorm measurement is continuous over the concatenated
   track): all-gather each rank's zero-start tail state (8 doubles), then
   carry(r) = sum_{q<r} A^{frames between span q and span r} tail(q) on the device
   (amx_kw_carry; the transition matrices are host-computed once per job).
2. Loudness partials: RCCL all-reduce(SUM) of the whole-track 100 ms hop energy
   array (a hop spanning a rank boundary gets exactly two non-zero addends, so the
   sum is order-independent and bit-identical for any world size) and
   all-reduce(MAX) of the sample peaks.  Every rank then derives the same
   histograms, statistics and gain.
3. Limiter: all-gather of each rank's last B-1 frames (the look-ahead halo).  If
   the limiter can engage (peaks above the limit) its state is handed rank to rank
   with send/recv (sequential, rare path).

Everything before the limiter runs on the stream without a host round trip; at
N > 1 the host reads the one-word limiter decision (identical on every rank, it is
computed from all-reduced data) to choose between the idle path and the
sequential rank-to-rank chain -- or loudnorm's dynamic mode (ShardedTrack.dynamic).
"""
import numpy as np
import torch
import torch.distributed as dist

from .chunking import chunk_bounds, packet_frames
from .engine import MasteringJob, wait_host_word


def overlay_len(n, fs):
    ms = round(1000 * (n / fs))
    return int(ms * (fs / 1000.0))


def chunk_out_frames(n, fs, multiband):
    if not multiband or n == 0:
        return n
    return overlay_len(overlay_len(n, fs), fs)


def shard_ranges(n_chunks, world):
    """Contiguous chunk ranges [(c0, c1)] per rank; the first n % world get one more."""
    base, extra = divmod(n_chunks, world)
    out, c = [], 0
    for r in range(world):
        k = base + (1 if r < extra else 0)
        out.append((c, c + k))
        c += k
    return out


def shard_tracks(track_frames, world):
    """A batch of whole tracks (C4: 64 tracks on 8 GPUs) split into contiguous runs,
    one per rank, balanced by frames: [(t0, t1)].  Whole tracks need no exchange at
    all -- loudness and the limiter are per track -- so each rank runs one
    MasteringJob over its tracks."""
    n = len(track_frames)
    if n < world:
        raise ValueError("%d tracks for %d ranks" % (n, world))
    total = float(sum(track_frames))
    out, t, acc = [], 0, 0.0
    for r in range(world):
        t0 = t
        goal = total * (r + 1) / world
        # take tracks while the next one's midpoint stays within this rank's share,
        # leaving at least one track for every later rank
        while t < n - (world - 1 - r) and (t == t0 or acc + track_frames[t] / 2.0 <= goal):
            acc += track_frames[t]
            t += 1
        out.append((t0, t))
    out[-1] = (out[-1][0], n)
    return out


def carry_from_tails(tails, span_frames, rank, propagate):
    """K-filter state entering `rank`'s span: c_0 = 0, c_{q+1} = A^{len_q} c_q + tail_q.

    tails: [world][8] zero-start end states; propagate(frames, state8) -> A^frames state8."""
    c = np.zeros(8)
    for q in range(rank):
        c = propagate(span_frames[q], c) + np.asarray(tails[q], np.float64).reshape(8)
    return c


# ------------------------------------------------------------------ collectives
# Device-agnostic (CUDA tensors over RCCL on the GPU path, CPU tensors over gloo in
# tests/test_dist.py), so the exchange steps are tested exactly as they run.

def _staged(group, *ts):
    """gloo with device tensors (multi-rank rehearsal on one GPU): host copies."""
    if dist.get_backend(group) == "gloo" and any(t.is_cuda for t in ts):
        return [t.cpu() for t in ts], True
    return list(ts), False


def gather_tails(tail, tails_all, group=None):
    """Step 1: every rank's zero-start K-filter end state [2, 4] -> tails_all[world, 2, 4]
    (rank order)."""
    (a, b), st = _staged(group, tails_all, tail.reshape(1, 2, 4).contiguous())
    dist.all_gather_into_tensor(a, b, group=group)
    if st:
        tails_all.copy_(a)
    return tails_all


def reduce_loudness(hops, peak, group=None):
    """Step 2: whole-track hop energies summed over ranks (each hop has at most two
    non-zero addends), sample peaks max-reduced.  hops None: loudnorm off."""
    for t, op in ((hops, dist.ReduceOp.SUM), (peak, dist.ReduceOp.MAX)):
        if t is None:
            continue
        (h,), st = _staged(group, t)
        dist.all_reduce(h, op=op, group=group)
        if st:
            t.copy_(h)


def gather_halo(out, n, h, rank, world, group=None):
    """Step 3: every rank's last h frames of its span out[:n] (zero-padded in front when
    the span is shorter) are all-gathered; returns the previous rank's (None on rank 0)."""
    mine = out[max(0, n - h):n]
    if mine.shape[0] < h:
        mine = torch.cat([torch.zeros((h - mine.shape[0], 2), dtype=mine.dtype, device=mine.device), mine])
    # one int32 word per stereo int16 frame: neither RCCL nor gloo reduces/gathers int16
    (mine,), st = _staged(group, mine.contiguous().view(torch.int32))
    allh = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allh, mine, group=group)
    if rank == 0:
        return None
    prev = allh[rank - 1].view(torch.int16)
    return prev.to(out.device) if st else prev


def chain_state(state, run, rank, world, group=None):
    """Sequential limiter path: receive the state from rank - 1, run(), pass it on."""
    (s,), st = _staged(group, state)
    if rank > 0:
        dist.recv(s, src=rank - 1, group=group)
        if st:
            state.copy_(s)
    run()
    if rank < world - 1:
        if st:
            s.copy_(state)
        dist.send(s, dst=rank + 1, group=group)


def is_rest_state(s, bs):
    """The alimiter's rest state in the hand-off layout (amx_final.hip): att = 1,
    delta = 0, empty list (nextiter = nextlen = 0, nextpos[0] = -1), valid.  s: one
    track's state ([state_doubles] or [1, state_doubles])."""
    s = s.detach().reshape(-1).cpu()
    return bool(s[5] == 1.0 and s[0] == 1.0 and s[1] == 0.0 and s[3] == 0.0 and s[4] == 0.0
                and s[8 + 2 * bs] == -1.0)


def chain_state_speculative(state, run, is_rest, rank, world, group=None, first_run_done=False):
    """Limiter hand-off with the ranks' work in parallel.  Every rank first runs its
    span from the rest state (state zeroed = nothing carried: the span's ring comes
    from the halo and the limiter is assumed at rest), all at once.  Then the true
    end states travel rank to rank: a rank whose received state is the rest state
    already has its exact output and end state; otherwise it re-runs from the
    received state.  Only the small state messages stay sequential.
    first_run_done: the from-rest run already happened (the N > 1 graph runs it on
    the device's own decision), so only the hand-off and re-runs remain."""
    if not first_run_done:
        state.zero_()
        run()
    if world == 1:
        return
    (s,), st = _staged(group, state)
    if rank > 0:
        incoming = torch.empty_like(s)
        dist.recv(incoming, src=rank - 1, group=group)
        if not is_rest(incoming):
            state.copy_(incoming)
            run()
    if rank < world - 1:
        if st:
            s.copy_(state)
        dist.send(s, dst=rank + 1, group=group)


def is_dynamic(ctl):
    """the device's mode word (k_decide, bits 4..7; 3 = dynamic): loudnorm's pass 2 runs
    the 192 kHz filter (:240 when the linear conditions fail)"""
    return (ctl >> 4) & 15 == 3


def shard_segments(K, k_fin, world):
    """The parallel loudnorm filter's segments (amx_loudnorm_192k_segments) split over
    the ranks for the sharded dynamic mode: contiguous [(kb, ke)], [0, k_fin) in near
    equal runs (the first k_fin % world one longer) and the last rank also takes the
    FINAL flush frame's segments [k_fin, K) (FINAL re-bases the ring: its walk cannot
    cross ranks).  None when there are fewer pre-FINAL segments than ranks."""
    if world < 1 or k_fin < world or K < k_fin:
        return None
    out = shard_ranges(k_fin, world)
    out[-1] = (out[-1][0], K)
    return out


def gather_track(out, n, span_frames, world, group=None):
    """every rank's span out[:n] (int16 [frames, 2]) all-gathered into the whole track
    [sum(span_frames), 2] on every rank (spans padded to the longest: one
    all_gather_into_tensor, one int32 word per stereo frame)"""
    mx = max(span_frames)
    buf = torch.zeros((mx, 2), dtype=torch.int16, device=out.device)
    if n > 0:
        buf[:n].copy_(out[:n])
    (w,), st = _staged(group, buf.view(torch.int32).reshape(-1))
    allw = torch.empty(world * mx, dtype=torch.int32, device=w.device)
    dist.all_gather_into_tensor(allw, w, group=group)
    allw = allw.view(world, mx)
    whole = torch.cat([allw[q, :span_frames[q]] for q in range(world)]).view(torch.int16).reshape(-1, 2)
    return whole.to(out.device) if st else whole


class ShardedTrack:
    """This rank's part of one chunk-sharded track.

    A step has three exchanges (every one a single collective over all ranks):
      1. edges: each rank's first 80 and last max(80, B - 1) output frames, all-gathered
         as raw bytes -- the 192 kHz resampler window of the loudness measurement
         reaches up to 80 frames into both neighbours (16 for the 32-tap filter, more
         for the downsampling filter above 192 kHz), and the alimiter's look-ahead ring
         needs the previous rank's last B - 1 frames;
      2. K-filter tails (8 doubles) and sample peaks (4 doubles), all-gathered: every
         rank builds its incoming K-filter state (amx_kw_carry) and the track's peaks;
      3. hop energies, all-reduced (SUM).
    """

    def __init__(self, sample_rate, channels_in, settings, track_frames, rank, world, *,
                 quantum=None, input_s16=False, seg_frames=128, group=None, force_exchange=False,
                 dynamic=False):
        self.rank, self.world, self.group = rank, world, group
        # dynamic: at one rank, hold loudnorm's dynamic path in the step (prepare_dynamic:
        # gated on the device) and return the 192 kHz output when the track takes it; at
        # N > 1 the step always handles it (dynamic())
        self.dyn = bool(dynamic)
        # force_exchange: run the N > 1 step (graph segments, every collective, the
        # carry kernels) even at world 1 -- an RCCL rehearsal on one GPU, since RCCL
        # refuses two ranks on one device; the output must equal the bypass path's
        self.xchg = world > 1 or bool(force_exchange)
        fs = int(sample_rate)
        if quantum is None:
            quantum = packet_frames(channels_in * (2 if input_s16 else 4))
        self.bounds = chunk_bounds(track_frames, fs, quantum)
        if len(self.bounds) < world:
            raise ValueError("track has %d chunks for %d ranks" % (len(self.bounds), world))
        mb = bool(settings.get("multiband"))
        self.out_n = [chunk_out_frames(n, fs, mb) for _, n in self.bounds]
        self.ranges = shard_ranges(len(self.bounds), world)
        c0, c1 = self.ranges[rank]
        self.in0 = self.bounds[c0][0]
        self.local_frames = sum(n for _, n in self.bounds[c0:c1])
        self.span_frames = [sum(self.out_n[a:b]) for a, b in self.ranges]
        self.tframe0 = sum(self.out_n[:c0])
        self.ttotal = sum(self.out_n)
        chunks = [(0, s - self.in0, n) for s, n in self.bounds[c0:c1]]
        self._job_args = ((fs, channels_in, settings, [self.local_frames]),
                          dict(chunks=chunks, track_frame0=[self.tframe0], track_total=[self.ttotal],
                               input_s16=input_s16, seg_frames=seg_frames))
        self.job = MasteringJob(*self._job_args[0], **self._job_args[1])
        self._slots = None         # the pipelined replay's two buffer sets (capture)
        self._pending = None
        if self.xchg:
            self._setup_exchange()

    def _setup_exchange(self):
        """the K-filter carry transitions and the exchange buffers of the N > 1 step.
        The exchange moves whole buffers with one gather kernel each, and the all-gathers
        run in place (each rank's input is its own row of the output): the K-filter tail
        and the peaks ARE that row (the job's kw_tail / peak are views of it), the edge
        frames are one index_select out of the span into it and one out of the gathered
        rows into a buffer the job's resampler edges and limiter halo are views of"""
        rank, world = self.rank, self.world
        job = self.job
        frames_after = [sum(self.span_frames[q + 1:rank]) for q in range(rank)]
        job.plan.kw_carry_setup(frames_after)
        dev = job.device
        from . import capi
        self.ne = capi.UP_EDGE                                  # frames after the span start
        self.nl = max(capi.UP_EDGE, job.halo_frames)            # frames before the span end
        W = self.ne + self.nl                                   # one int32 word per frame
        # the gathered words, and one zero word after them (the source of a missing
        # neighbour); this rank's words are its own row: the all-gathers run in place
        # (no local copy, none at all at world 1)
        self._eall = torch.zeros(world * W + 1, dtype=torch.int32, device=dev)
        self._ebuf = self._eall[rank * W:(rank + 1) * W]
        E, h = capi.UP_EDGE, max(1, job.halo_frames)
        self._edst = torch.zeros(2 * E + h, dtype=torch.int32, device=dev)
        job.edge = self._edst[:2 * E].view(torch.int16).reshape(1, 2, E, 2)
        job.halo = self._edst[2 * E:].view(torch.int16).reshape(1, h, 2)
        zero = world * W
        src = [zero] * (2 * E + h)
        if rank > 0:
            for i in range(E):
                src[i] = (rank - 1) * W + self.ne + self.nl - E + i
            for i in range(job.halo_frames):
                src[2 * E + i] = (rank - 1) * W + self.ne + self.nl - job.halo_frames + i
        if rank < world - 1:
            for i in range(E):
                src[E + i] = (rank + 1) * W + i
        self._eidx = torch.tensor(src, dtype=torch.int64, device=dev)
        n = self.span_frames[rank]
        self._pidx = None
        if n >= max(self.ne, self.nl):
            self._pidx = torch.tensor(list(range(self.ne)) + list(range(n - self.nl, n)), dtype=torch.int64,
                                      device=dev)
        self._xall = torch.zeros(world * 12, dtype=torch.float64, device=dev)
        self._xbuf = self._xall[rank * 12:(rank + 1) * 12]
        job.kw_tail = self._xbuf[0:8].view(1, 2, 4)
        job.peak = self._xbuf[8:12].view(1, 4)

    # -------------------------------------------------------------- exchanges
    def _all_gather(self, out, inp):
        (a, b), st = _staged(self.group, out, inp)
        dist.all_gather_into_tensor(a, b, group=self.group)
        if st:
            out.copy_(a)

    def _pack_edges(self):
        """This span's first ne and last nl output frames (zero-padded when shorter)."""
        job, n = self.job, self.span_frames[self.rank]
        out32 = job.out.view(torch.int32).reshape(-1)
        if self._pidx is not None:
            torch.index_select(out32, 0, self._pidx, out=self._ebuf)
            return
        b = self._ebuf
        b.zero_()
        m = min(self.ne, n)
        if m > 0:
            b[:m].copy_(out32[:m])
        m = min(self.nl, n)
        if m > 0:
            o = self.ne + self.nl - m
            b[o:o + m].copy_(out32[n - m:n])

    def _unpack_edges(self):
        """Previous rank's last frames -> the resampler's low edge and the limiter halo;
        next rank's first frames -> the resampler's high edge (one gather)."""
        torch.index_select(self._eall, 0, self._eidx, out=self._edst)

    def exchange_edges(self):
        self._pack_edges()
        self._all_gather(self._eall[:-1], self._ebuf)
        self._unpack_edges()

    def _pack_x(self):
        """(nothing to move: the job's kw_tail and peak live in the all-gather's input)"""

    def _unpack_x(self):
        from . import capi
        job = self.job
        # the K-filter carry from the previous ranks' tails and the track's peaks (max over
        # the ranks) straight from the gathered rows: one kernel
        capi.check(capi.load().amx_kw_carry_rows(job.plan.h, capi.ptr(self._xall), self.world, 12,
                                                 capi.ptr(job.kw_carry), capi.ptr(job.peak), job._s(None)),
                   "amx_kw_carry_rows")

    def exchange_carry_peaks(self):
        self._pack_x()
        self._all_gather(self._xall, self._xbuf)
        self._unpack_x()

    def limiter_sequential(self):
        job = self.job
        chain_state_speculative(job.lim_state, lambda: job.finalize(False),
                                lambda v: is_rest_state(v, job.bs), self.rank, self.world, self.group)

    # ------------------------------------------------- loudnorm dynamic mode
    def m192(self, f):
        """the 192 kHz stream position of chain frame f of the track (ceil(f L / M):
        the first output whose window is centred at or after f)"""
        import math
        g = math.gcd(self.job.fs, 192000)
        L, M = 192000 // g, self.job.fs // g
        return (f * L + M - 1) // M

    def dynamic_range(self, rank=None):
        """[P0, P1): the 192 kHz output frames rank `rank` returns in dynamic mode -- the
        outputs made from its span's chain frames, so the ranks' outputs concatenate to
        the track's"""
        r = self.rank if rank is None else rank
        f0 = sum(self.span_frames[:r])
        return self.m192(f0), self.m192(f0 + self.span_frames[r])

    def _ln_split(self, W):
        """the filter's segments, this rank's share and the hand-off buffers (once per
        whole-track plan): None when the track has too few segments to split"""
        import ctypes
        from . import capi
        L = capi.load()
        K, kf, rd, co = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        capi.check(L.amx_loudnorm_192k_segments(W.plan.h, 0, None, 0, ctypes.byref(K), ctypes.byref(kf),
                                                ctypes.byref(rd), ctypes.byref(co)), "amx_loudnorm_192k_segments")
        starts = (ctypes.c_int64 * (K.value + 1))()
        capi.check(L.amx_loudnorm_192k_segments(W.plan.h, 0, starts, K.value + 1, ctypes.byref(K), None, None,
                                                None), "amx_loudnorm_192k_segments")
        ranges = shard_segments(K.value, kf.value, self.world)
        if ranges is None:
            return None
        dev = W.device
        return {"starts": list(starts), "ranges": ranges, "ctl": co.value,
                "rec_in": torch.zeros(rd.value, dtype=torch.float64, device=dev),
                "rec_out": torch.zeros(rd.value, dtype=torch.float64, device=dev),
                "flag": torch.zeros(1, dtype=torch.int32, device=dev)}

    def _filter_sharded(self, W, side, desc, measured, offset_i):
        """one dynamic-mode filter run of the track, its segments sharded over the ranks
        (amx_loudnorm_192k_shard): part 0 (this rank's 192 kHz stream, every frame's
        statistics), part 1 (gains, the segments [kb, ke) from guessed states), then the
        walks in rank order: each rank receives the true limiter state at kb from
        rank - 1 (one record), walks its boundaries and sends the state at ke on.  This
        rank's output: job2.out[start(kb), start(ke)).
        A quiet start or a walk that cannot go on (the frame-by-frame path: one
        sequence over the whole track) runs the whole filter on every rank instead;
        every rank takes the same branch (the control word comes from the same hop
        energies; the walk's fallback is all-reduced)."""
        import ctypes
        from . import capi
        n192, job2, ws2, summ = side
        L = capi.load()
        sp = self._split

        def whole():
            W.loudnorm_192k(0, desc, job2, ws2, summ, measured=measured, offset_i=offset_i)
            self._forms.append("replicated")

        kb, ke = sp["ranges"][self.rank]
        rank, world = self.rank, self.world

        def part(p):
            sh = capi.LnShard(p, kb, ke, 0, -1, -1, capi.ptr(sp["rec_in"]) if rank > 0 else None,
                              capi.ptr(sp["rec_out"]) if rank < world - 1 else None)
            capi.check(L.amx_loudnorm_192k_shard(
                W.plan.h, 0, ctypes.byref(desc), capi.ptr(measured), capi.ptr(offset_i), ctypes.byref(sh),
                capi.ptr(W.out), capi.ptr(W.hops), int(W.max_hops), capi.ptr(W.peak), capi.ptr(job2.out),
                capi.ptr(summ), capi.ptr(ws2), W._s(None)), "amx_loudnorm_192k_shard")

        ctl = ws2[sp["ctl"]:sp["ctl"] + 4].view(torch.int32)
        part(0)
        if int(ctl.item()) != 0:
            return whole()
        part(1)
        if rank > 0:
            (s,), st = _staged(self.group, sp["rec_in"])
            dist.recv(s, src=rank - 1, group=self.group)
            if st:
                sp["rec_in"].copy_(s)
        part(2)
        if rank < world - 1:
            (s,), _ = _staged(self.group, sp["rec_out"])
            dist.send(s, dst=rank + 1, group=self.group)
        flag = sp["flag"]
        flag.copy_(ctl[0:1] == 2)
        (f,), st = _staged(self.group, flag)
        dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
        if int(f.item()) != 0:
            return whole()
        self._forms.append("sharded")

    def _dynamic_sharded(self, W):
        """_dyn_enqueue's sequence with the 192 kHz stream split over the ranks by the
        filter's segments: filter pass 1 (sharded), the loudness of its output measured
        from the ranks' runs (Span192: K-filter carry, hop energies all-reduced) ->
        target_offset, filter pass 2 (sharded), its peaks (max over ranks) and the
        alimiter over the runs (halo + state hand-off).  Returns (this rank's run of the
        192 kHz output, info)."""
        from . import capi, loudness
        from .settings import LOUDNORM_LRA, LOUDNORM_TP
        sp = self._split
        side = W._job192(0, cached=True)
        job2 = side[1]
        kb, ke = sp["ranges"][self.rank]
        starts = sp["starts"]
        s0, s1 = starts[kb], starts[ke]
        S = sp.get("span")
        if S is None:
            lens = [starts[b] - starts[a] for a, b in sp["ranges"]]
            S = sp["span"] = Span192(lens, self.rank, self.world, self.group, W.settings.get("lufs"), W.device)
        target = float(W.settings["lufs"])
        d1 = capi.LoudnormDesc(target, LOUDNORM_LRA, LOUDNORM_TP, 0.0, 0.0, 99.0, -70.0, 0.0)
        self._filter_sharded(W, side, d1, None, None)
        S.job.out[:s1 - s0].copy_(job2.out[s0:s1])
        S.measure(True)
        W._i_out[0:1].copy_(S.job.stats[0, 0:1])             # pass 1's output loudness
        d2 = capi.LoudnormDesc(target, LOUDNORM_LRA, LOUDNORM_TP, 0.0, 0.0, 99.0, -70.0, 0.0)
        self._filter_sharded(W, side, d2, W.stats[0], W._i_out[0:1])
        S.job.out[:s1 - s0].copy_(job2.out[s0:s1])
        S.measure(False)                                     # the limiter's input bound
        y = S.limit()
        i_out = float(W._i_out[0].item())
        info = {"target_offset": loudness._fmt(target - i_out), "pass1_output_i": i_out,
                "sample_rate": 192000, "limiter_fast": S.fast}
        return y, info

    def dynamic(self, sharded=True):
        """loudnorm's dynamic mode on the chunk-sharded track (:240 when the linear
        conditions fail; :223's alimiter then runs on the 192 kHz stream).

        Windowed form (the default at N > 1, _dynamic_windowed): every rank keeps its own
        part -- the filter's gains come from the step's own all-reduced hop energies and
        decision, the filter segments are split at the ranks' span boundaries, and a
        rank holds only its span plus a halo of the neighbours' edge frames (one
        all-gather), the 192 kHz stream and output of its own segments; the limiter
        state record goes rank to rank; the 192 kHz measurement and the alimiter run
        over the ranks' runs (Span192).  Per-rank memory and traffic scale as 1 / N.
        Replicated form (a track too short to split, a quiet start or a walk fallback
        -- one sequence over the whole track --, or sharded=False): the spans are
        all-gathered and every rank runs the whole 192 kHz path.
        Returns int16 [P1 - P0, 2]: this rank's run of the 192 kHz output."""
        job = self.job
        self._forms = []
        y = info = None
        if sharded and self.world > 1:
            wd = self._windows()
            if wd is not None:
                r = self._dynamic_windowed(wd)
                if r is not None:
                    y, info = r
                    self.dyn_range = wd["y"][self.rank]
        if y is None:
            y, info = self._dynamic_replicated(sharded)
        fs_ = self._forms or ["replicated"]
        form = fs_[0] if all(f == fs_[0] for f in fs_) else "+".join(fs_)
        self.dyn_info = dict(info, form=form)
        job.report.update(dynamic=self.dyn_info, sample_rate=192000)
        return y

    def _dynamic_replicated(self, sharded):
        """the spans all-gathered into a whole-track plan on every rank, measured again,
        and the 192 kHz path run whole (MasteringJob.dynamic_track), or with the filter's
        segments split evenly over the ranks (_dynamic_sharded)"""
        job = self.job
        whole = gather_track(job.out, self.span_frames[self.rank], self.span_frames, self.world, self.group)
        W = getattr(self, "_whole", None)
        if W is None:
            W = MasteringJob(job.fs, 2, {"lufs": job.settings.get("lufs")}, [self.ttotal], input_s16=True,
                             chunks=[(0, 0, self.ttotal)], device=job.device, measure_only=True)
            self._whole = W
            self._split = self._ln_split(W) if self.world > 1 else None
        W.out[:self.ttotal].copy_(whole)
        W.loudness_pass1(tail=False)
        W.loudness_pass2(carry=False)
        W.histograms()
        W.decide()
        if sharded and self._split is not None:
            y, info = self._dynamic_sharded(W)
            kb, ke = self._split["ranges"][self.rank]
            self.dyn_range = (self._split["starts"][kb], self._split["starts"][ke])
        else:
            y, info = W.dynamic_track(0)
            self.dyn_range = self.dynamic_range()
            y = y[self.dyn_range[0]:self.dyn_range[1]]
            self._forms.append("replicated")
        return y, info

    # ------------------------------------------- dynamic mode, windowed (N > 1)
    def _windows(self):
        """(once per track) the filter's segments split at the ranks' span boundaries and
        each rank's windows (amx_loudnorm_192k_shard_window): chain frames x, 192 kHz
        stream u, output positions y; the halo sizes of the edge exchange.  None when the
        track cannot be split so (spans shorter than a halo, a rank without a segment,
        FINAL not on the last rank)."""
        if hasattr(self, "_wd"):
            return self._wd
        import ctypes
        from . import capi, design
        L = capi.load()
        job, world = self.job, self.world
        desc, keep = design.chain_desc(job.fs, 2, {"lufs": job.settings.get("lufs")})
        desc.input_s16 = 1
        desc.measure_only = 1
        plan = capi.Plan(desc, [(0, 0, self.ttotal)], None, None, 128)   # geometry only
        K, kf, rd, co = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        capi.check(L.amx_loudnorm_192k_segments(plan.h, 0, None, 0, ctypes.byref(K), ctypes.byref(kf),
                                                ctypes.byref(rd), ctypes.byref(co)), "amx_loudnorm_192k_segments")
        starts = (ctypes.c_int64 * (K.value + 1))()
        capi.check(L.amx_loudnorm_192k_segments(plan.h, 0, starts, K.value + 1, ctypes.byref(K), None, None, None),
                   "amx_loudnorm_192k_segments")
        starts = list(starts)
        F = [sum(self.span_frames[:q]) for q in range(world + 1)]
        kbs = [0]
        for q in range(1, world):
            p = self.m192(F[q])
            kbs.append(next((k for k in range(K.value) if starts[k] >= p), K.value))
        kbs.append(K.value)
        self._wd = None
        if any(kbs[q] >= kbs[q + 1] for q in range(world)) or kbs[world - 1] > kf.value:
            return None
        xs, us, ys, wsb, ctl, doff = [], [], [], [], [], []
        for q in range(world):
            win = (ctypes.c_int64 * 9)()
            b = ctypes.c_int64()
            capi.check(L.amx_loudnorm_192k_shard_window(plan.h, 0, kbs[q], kbs[q + 1], win, ctypes.byref(b)),
                       "amx_loudnorm_192k_shard_window")
            xs.append((win[0], win[1]))
            us.append((win[2], win[3]))
            ys.append((win[4], win[5]))
            wsb.append(b.value)
            ctl.append(win[6])
            doff.append((win[7], win[8]))
        before = [max(0, F[q] - xs[q][0]) for q in range(world)]
        after = [max(0, xs[q][1] - F[q + 1]) for q in range(world)]
        if any(before[q] > (self.span_frames[q - 1] if q > 0 else 0) for q in range(world)) or \
                any(after[q] > (self.span_frames[q + 1] if q + 1 < world else 0) for q in range(world)):
            return None
        r = self.rank
        dev = job.device
        Hb, Ha = max(before), max(after)
        wd = {"plan": plan, "keep": keep, "K": K.value, "kb": kbs[r], "ke": kbs[r + 1], "x": xs[r], "u": us[r],
              "y": ys, "F": F, "Hb": Hb, "Ha": Ha, "ctl": ctl[r], "rec_doubles": rd.value,
              "d_off": doff[r][0], "T": doff[r][1],
              "qbuf": torch.zeros(3 + max(1, doff[r][1]), dtype=torch.float64, device=dev),
              "ws2": torch.empty(max(1, wsb[r]), dtype=torch.uint8, device=dev),
              "xwin": torch.zeros((max(1, xs[r][1] - xs[r][0]), 2), dtype=torch.int16, device=dev),
              "summ": torch.zeros(16, dtype=torch.float64, device=dev),
              "i_out": torch.zeros(1, dtype=torch.float64, device=dev),
              "rec_in": torch.zeros(rd.value, dtype=torch.float64, device=dev),
              "rec_out": torch.zeros(rd.value, dtype=torch.float64, device=dev),
              "flag": torch.zeros(1, dtype=torch.int32, device=dev),
              "ebuf": torch.zeros(max(1, Ha + Hb), dtype=torch.int32, device=dev),
              "eall": torch.zeros(world * max(1, Ha + Hb), dtype=torch.int32, device=dev)}
        # the 192 kHz runs as a chunk-sharded measure-only track: its output buffer is the
        # filter's windowed output (no copy)
        wd["span"] = Span192([y1 - y0 for y0, y1 in ys], r, world, self.group, job.settings.get("lufs"), dev)
        self._wd = wd
        return wd

    def _fill_window(self, wd):
        """the chain frames [x_lo, x_hi) this rank's resampler reads: the previous rank's
        last frames, its own span, the next rank's first frames (one all-gather of every
        rank's first Ha and last Hb frames)"""
        job, r, world = self.job, self.rank, self.world
        Ha, Hb, F = wd["Ha"], wd["Hb"], wd["F"]
        n = self.span_frames[r]
        out32 = job.out[:n].view(torch.int32).reshape(-1)
        eb = wd["ebuf"]
        if Ha + Hb > 0:
            eb.zero_()
            m = min(Ha, n)
            eb[:m].copy_(out32[:m])
            m = min(Hb, n)
            eb[Ha + Hb - m:Ha + Hb].copy_(out32[n - m:n])
            self._all_gather(wd["eall"], eb)
        ea = wd["eall"].view(world, -1)
        x0, x1 = wd["x"]
        xw = wd["xwin"].view(torch.int32).reshape(-1)
        # [x0, F_r): the previous rank's last frames
        if x0 < F[r]:
            k = F[r] - x0
            xw[:k].copy_(ea[r - 1][Ha + Hb - k:Ha + Hb])
        a, b = max(x0, F[r]), min(x1, F[r + 1])
        if b > a:
            xw[a - x0:b - x0].copy_(out32[a - F[r]:b - F[r]])
        if x1 > F[r + 1]:
            k = x1 - F[r + 1]
            xw[x1 - x0 - k:].copy_(ea[r + 1][:k])

    def _filter_windowed(self, wd, desc, measured, offset_i):
        """one filter run over this rank's segments [kb, ke) in its windows
        (amx_loudnorm_192k_shard, windowed): part 0 (the 192 kHz stream over the u
        window, every frame's statistics from the all-reduced hop energies), part 1
        (gains, the fill pre-pass, the segments from guessed states), then the walks in
        rank order with the one-record hand-off.  A quiet start runs split first
        (_quiet_start: rank 0's frames in order up to the hand-over).  False: the parallel
        form cannot run this track (a walk fallback, a start still quiet past rank 0's
        segments) -- every rank takes the same branch."""
        import ctypes
        from . import capi
        L = capi.load()
        job, rank, world = self.job, self.rank, self.world
        kb, ke = wd["kb"], wd["ke"]
        y_out = wd["span"].job.out

        def part(p):
            sh = capi.LnShard(p, kb, ke, 1, -1, -1, capi.ptr(wd["rec_in"]) if rank > 0 else None,
                              capi.ptr(wd["rec_out"]) if rank < world - 1 else None)
            capi.check(L.amx_loudnorm_192k_shard(
                wd["plan"].h, 0, ctypes.byref(desc), capi.ptr(measured), capi.ptr(offset_i), ctypes.byref(sh),
                capi.ptr(wd["xwin"]), capi.ptr(job.hops), int(job.max_hops), capi.ptr(job.peak), capi.ptr(y_out),
                capi.ptr(wd["summ"]), capi.ptr(wd["ws2"]), job._s(None)), "amx_loudnorm_192k_shard")

        ctl = wd["ws2"][wd["ctl"]:wd["ctl"] + 4].view(torch.int32)
        part(0)
        c0 = int(ctl.item())
        if c0 == 1 and not self._quiet_start(wd, part):
            return False
        if c0 not in (0, 1):
            return False
        part(1)
        if rank > 0:
            (s,), st = _staged(self.group, wd["rec_in"])
            dist.recv(s, src=rank - 1, group=self.group)
            if st:
                wd["rec_in"].copy_(s)
        part(2)
        if rank < world - 1:
            (s,), _ = _staged(self.group, wd["rec_out"])
            dist.send(s, dst=rank + 1, group=self.group)
        flag = wd["flag"]
        flag.copy_(ctl[0:1] == 2)
        (f,), st = _staged(self.group, flag)
        dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
        return int(f.item()) == 0

    def _quiet_start(self, wd, part):
        """A track whose first 3 s are below measured_thresh (control word 1 on every rank,
        the same hop energies): af_loudnorm's gains there follow its own output (a feedback
        loop, k_ln_dyn frame by frame).  Rank 0 holds the track's start: it runs those frames
        in order up to the hand-over segment (amx_ln_shard part 3) and broadcasts the control
        words and the deltas written so far; every rank then runs its own segments as for a
        loud start (rank 0 from the hand-over record).  False -- the track is still quiet past
        rank 0's last segment, or a rank's first segment would precede the hand-over: the
        replicated form, on every rank alike (the words come from the broadcast)."""
        w = wd["ws2"]
        ctl = w[wd["ctl"]:wd["ctl"] + 24].view(torch.int32)
        T, d_off = int(wd["T"]), int(wd["d_off"])
        D = w[d_off:d_off + 8 * T].view(torch.float64)
        q = wd["qbuf"]
        if self.rank == 0:
            part(3)
            q[0:3].copy_(ctl[torch.tensor([0, 4, 5], device=ctl.device)].to(torch.float64))
            q[3:3 + T].copy_(D)
        (b,), st = _staged(self.group, q)
        dist.broadcast(b, src=0, group=self.group)
        if st:
            q.copy_(b)
        words = [int(v) for v in q[0:3].tolist()]
        if words[0] != 4:             # (the same words on every rank: one branch for all)
            return False
        # part 3 hands over at a segment below rank 0's last (amx_ln_shard.part 3), so every
        # other rank's segments start after it
        if self.rank > 0:
            ctl[0] = 4
            ctl[4] = words[1]
            ctl[5] = words[2]
            t0 = max(0, words[2] - 1)
            D[:t0].copy_(q[3:3 + t0])
        return True

    def _dynamic_windowed(self, wd):
        """the reference's two loudnorm passes in dynamic mode (:229 / :240) and the
        alimiter (:223) over the ranks' windows: filter pass 1 -> the loudness of its
        output measured over the runs (Span192) -> target_offset; filter pass 2 with the
        step's own statistics row; its peaks and the alimiter over the runs.  None: the
        parallel form cannot run this track (the replicated form takes it)."""
        from . import capi, loudness
        from .settings import LOUDNORM_LRA, LOUDNORM_TP
        job = self.job
        S = wd["span"]
        self._fill_window(wd)
        target = float(job.settings["lufs"])
        d1 = capi.LoudnormDesc(target, LOUDNORM_LRA, LOUDNORM_TP, 0.0, 0.0, 99.0, -70.0, 0.0)
        if not self._filter_windowed(wd, d1, None, None):
            return None
        S.measure(True)
        wd["i_out"].copy_(S.job.stats[0, 0:1])                    # pass 1's output loudness
        d2 = capi.LoudnormDesc(target, LOUDNORM_LRA, LOUDNORM_TP, 0.0, 0.0, 99.0, -70.0, 0.0)
        d2.reuse_stream = 1          # the same windows: pass 1's stream over u stands
        if not self._filter_windowed(wd, d2, job.stats[0], wd["i_out"]):
            return None
        S.measure(False)                                     # the limiter's input bound
        y = S.limit()
        i_out = float(wd["i_out"][0].item())
        self._forms.append("windowed")
        info = {"target_offset": loudness._fmt(target - i_out), "pass1_output_i": i_out,
                "sample_rate": 192000, "limiter_fast": S.fast}
        return y, info

    # -------------------------------------------------------------- the step
    def capture(self, d_in):
        """Record the step's device work as hipGraphs (torch.cuda.CUDAGraph over HIP
        stream capture).  One rank: the whole step (MasteringJob.capture).  N ranks over
        RCCL: the whole step as ONE graph with its three collectives captured as nodes:
          chunk chain, packing the span's edge frames;
          all-gather of the edges;
          unpacking them, loudness pass 1 (GEMV + scan from rest + tail + peaks),
          packing tail and peaks;
          all-gather of tails and peaks;
          carry (amx_kw_carry), peak = max over ranks, loudness pass 2;
          all-reduce(SUM) of the hop energies (loudnorm on);
          histograms + decision + the limiter on the device's decision, and the
          decision word copied to pinned host memory;
        then the host reads the decision and, only if the limiter can engage, hands
        its state rank to rank.  Over gloo (host-staged collectives) the four stretches
        between the collectives are four graphs and the collectives run eagerly."""
        if not self.xchg:
            return self.job.capture(d_in, dynamic=self.dyn)
        job = self.job
        lufs_on = job.dd.lufs_on

        def seg(*fns):
            g = torch.cuda.CUDAGraph()
            # thread_local: the process group's watchdog thread polls the events of
            # finished collectives; in the default (global) mode that poll invalidates a
            # capture running at the same time
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                for fn in fns:
                    fn()
            return g

        # the limiter runs from rest in the graph, so when the device picks the general
        # limiter the in-graph run IS the speculative from-rest run of
        # chain_state_speculative: replay() then only hands the end states along
        def fin():
            job.finalize(None, from_rest=True)

        torch.cuda.synchronize()
        if dist.get_backend(self.group) == "nccl":
            return self._capture_pipelined(d_in, seg)
        self._ctl_host = torch.zeros(1, dtype=torch.int32).pin_memory()
        self._ctl_ev = torch.cuda.Event()
        # gloo (the N-rank rehearsal on one GPU) stages every collective through host
        # copies, which a graph cannot hold: the stretches between them are the graphs
        g1 = seg(lambda: job.run_chunks(d_in), self._pack_edges)
        g2 = seg(self._unpack_edges, lambda: job.loudness_pass1(tail=True), self._pack_x)
        g3 = seg(self._unpack_x, lambda: job.loudness_pass2(carry=True)) if lufs_on else seg(self._unpack_x)
        g4 = seg(job.histograms, job.decide, fin) if lufs_on else seg(job.decide, fin)
        self._g = [g1, g2, g3, g4]
        return self._g

    # the pipelined replay's per-slot state: a MasteringJob, its exchange buffers, the
    # pinned decision word and its event, its graph
    # (every tensor a slot's graph reads or writes stays referenced here: one replaced by
    # the other slot's _setup_exchange and freed would be re-used while the graph holds
    # its address -- r05f's index_select fault on the freed gather indices)
    _SLOT_KEYS = ("job", "_ebuf", "_eall", "_edst", "_eidx", "_pidx", "_xbuf", "_xall", "_ctl_host",
                  "_ctl_ev", "_g")

    def _use(self, k):
        for key, v in self._slots[k].items():
            setattr(self, key, v)

    def _capture_pipelined(self, d_in, seg):
        """Two buffer sets (slots), each with its own job, exchange buffers and graph: the
        whole step as ONE graph with its RCCL collectives captured as nodes
        (scripts/rccl_capture_probe.py), the decision word copied to pinned memory at
        its end.  replay() alternates them, so step k + 1 is enqueued before the host
        reads step k's word: the host never stalls the device, and a step whose limiter
        needs the rank-to-rank hand-off (or dynamic mode) is finished on its own slot,
        in stream order after step k + 1 (which touches only the other slot's
        buffers).  Every rank takes the same branch (the word comes from all-reduced
        data), so RCCL operations stay in the same order on every rank."""
        lufs_on = self.job.dd.lufs_on
        slots = []
        for k in range(2):
            if k == 1:
                self.job = MasteringJob(*self._job_args[0], **self._job_args[1])
                self._setup_exchange()
                self.step(d_in)                  # the new buffers' first (eager) step
                torch.cuda.synchronize()
            job = self.job
            self._ctl_host = torch.zeros(1, dtype=torch.int32).pin_memory()
            self._ctl_ev = torch.cuda.Event()
            job.plan.set_publish(self._ctl_host)

            def whole(job=job):
                job.run_chunks(d_in)
                self._pack_edges()
                self._all_gather(self._eall[:-1], self._ebuf)
                self._unpack_edges()
                job.loudness_pass1(tail=True)
                self._pack_x()
                self._all_gather(self._xall, self._xbuf)
                self._unpack_x()
                if lufs_on:
                    job.loudness_pass2(carry=True)
                    reduce_loudness(job.hops, None, self.group)
                    job.histograms()
                job.decide()                   # (k_decide also stores the word to _ctl_host)
                # the in-graph limiter run from rest on the device's decision (see fin):
                # from_rest ignores the carried state, and the span's end state lands in
                # this slot's own job.lim_state, which _resolve hands to the next rank
                # (a shared zero buffer was overwritten by the first engaged
                # step, and lim_state was never written in the graph)
                job.finalize(None, from_rest=True)
            self._g = [seg(whole)]
            slots.append({key: getattr(self, key) for key in self._SLOT_KEYS})
        self._slots = slots
        self._slot = 0
        self._pending = None
        self._use(0)
        return [sl["_g"][0] for sl in slots]

    def _resolve(self, k):
        """finish the step that ran on slot k: wait for its decision word and, if the
        limiter can engage, hand its state along; dynamic mode runs the 192 kHz path.
        Returns the step's output."""
        from . import capi
        cur = {key: getattr(self, key) for key in self._SLOT_KEYS}
        self._use(k)
        try:
            job = self.job
            wait_host_word(self._ctl_ev.query, "the step's end event")
            hv = self._ctl_host.numpy()
            # (the device's store lands with the step's end)
            wait_host_word(lambda: hv[0] != -1, "the step's decision word")
            ctl = int(hv[0])
            if is_dynamic(ctl):
                return self.dynamic()
            if not (ctl & capi.CTL_FAST):
                chain_state_speculative(job.lim_state, lambda: job.finalize(False),
                                        lambda v: is_rest_state(v, job.bs), self.rank, self.world,
                                        self.group, first_run_done=True)
            return job.y[:job.info.out_frames]
        finally:
            for key, v in cur.items():
                setattr(self, key, v)

    def flush(self):
        """The output of the last replay(), final (the pipelined replay resolves a step
        when the next one has been enqueued; call this before reading the last output).
        None when nothing is pending."""
        if self._slots is None or self._pending is None:
            return getattr(self, "_last_out", None)
        k, self._pending = self._pending, None
        self._last_out = self._resolve(k)
        return self._last_out

    def _one_rank_dynamic(self, y):
        d = self.job.dynamic_output(0) if self.dyn else None
        if d is None:
            return y
        self.dyn_info = dict(d[1], form="one rank")
        return d[0]

    def replay(self):
        """One step from the captured graph(s).  Pipelined (N > 1 over RCCL): enqueues
        the step on the next slot, then resolves the previous step (its decision word,
        and the rare hand-off / dynamic path on its own slot); returns this step's
        linear output buffer.  That buffer is final only after the next replay() or
        flush(), and only if the step stayed linear: a step that turns out dynamic has its
        192 kHz output in what flush() returns -- callers that keep a
        step's output take it from flush() (or the next replay()'s _last_out)."""
        if not self.xchg:
            self._last_out = self._one_rank_dynamic(self.job.replay())
            return self._last_out
        from . import capi
        if self._slots is not None:
            k = self._slot
            self._use(k)
            self._ctl_host.fill_(-1)            # (this slot's previous word was read)
            self._g[0].replay()                 # the whole step, collectives included
            self._ctl_ev.record()
            prev, self._pending, self._slot = self._pending, k, k ^ 1
            if prev is not None:
                self._last_out = self._resolve(prev)
            out = self.job.y[:self.job.info.out_frames]
            self._use(0)            # (step(), dynamic() and callers see slot 0's buffers)
            return out
        job = self.job
        if len(self._g) == 4:
            g1, g2, g3, g4 = self._g
            g1.replay()
            self._all_gather(self._eall[:-1], self._ebuf)
            g2.replay()
            self._all_gather(self._xall, self._xbuf)
            g3.replay()
            if job.dd.lufs_on:
                reduce_loudness(job.hops, None, self.group)
            g4.replay()
            self._ctl_host.copy_(job.ctl[:1], non_blocking=True)
        # The one host read of the step: RCCL operations are enqueued by the host, so
        # only the host can decide whether the limiter's rank-to-rank hand-off runs.
        # The word is the same on every rank (computed from all-reduced data); when it
        # says "idle" (the common case) the step is already complete on the device.
        # Only this 4-byte copy is waited for: an event on the launch stream, polled
        # (a blocking event wait sleeps and wakes late)
        self._ctl_ev.record()
        wait_host_word(self._ctl_ev.query, "the decision word's copy")
        if is_dynamic(int(self._ctl_host[0])):
            self._last_out = self.dynamic()
            return self._last_out
        if not (int(self._ctl_host[0]) & capi.CTL_FAST):
            chain_state_speculative(job.lim_state, lambda: job.finalize(False),
                                    lambda v: is_rest_state(v, job.bs), self.rank, self.world,
                                    self.group, first_run_done=True)
        self._last_out = job.y[:job.info.out_frames]
        return self._last_out

    def close(self):
        """Free what this rank's step holds, graphs first: the captured graphs (at N > 1
        over RCCL their nodes use the process group's communicator), then the slots'
        jobs, the dynamic-mode side jobs and plans.  Call it before
        dist.destroy_process_group -- or use `with ShardedTrack(...) as tr:` -- so no
        graph holding RCCL nodes outlives its communicator (the round-5 hipGraphLaunch
        segfault's suspect: such graphs freed at a later garbage collection).
        Idempotent; the object is unusable afterwards."""
        import gc
        if getattr(self, "_closed", False):
            return
        self._closed = True
        torch.cuda.synchronize()
        self._pending = None
        jobs = [self.job]
        for sl in (self._slots or []):
            sl["_g"] = None
            jobs.append(sl["job"])
        self._slots = None
        self._g = None
        wd = getattr(self, "_wd", None)
        if wd:
            jobs.append(wd["span"].job)
            wd["plan"].close()
        sp = getattr(self, "_split", None)
        if sp and sp.get("span") is not None:
            jobs.append(sp["span"].job)
        if getattr(self, "_whole", None) is not None:
            jobs.append(self._whole)
        seen = set()
        for j in jobs:
            if id(j) not in seen:
                seen.add(id(j))
                j.close()
        gc.collect()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def step(self, d_in):
        """One pass of the whole path over this rank's chunks (input resident)."""
        from . import capi
        if self._slots is not None and self._pending is not None:
            self.flush()            # a pipelined step still pending: resolve it first
        job = self.job
        if not self.xchg:
            if self.dyn:
                job.prepare_dynamic()
            return self._one_rank_dynamic(job.run(d_in))
        job.run_chunks(d_in)
        self.exchange_edges()
        job.timed("up", lambda: job.loudness_pass1(tail=True, part=0))
        job.timed("loud1", lambda: job.loudness_pass1(tail=True, part=1))
        self.exchange_carry_peaks()
        lufs_on = job.dd.lufs_on
        if lufs_on:
            job.timed("loud2", lambda: job.loudness_pass2(carry=True))
            reduce_loudness(job.hops, None, self.group)
            job.timed("hist", job.histograms)
        job.timed("decide", job.decide)
        ctl = int(job.ctl[0].item())
        job.report = {"chunks": len(job.chunks), "segments": job.info.n_segments}
        if is_dynamic(ctl):
            return self.dynamic()
        fast = bool(ctl & capi.CTL_FAST)
        if fast:
            job.timed("final", lambda: job.finalize(True))
        else:
            job.lim_state.zero_()
            self.limiter_sequential()
        return job.y[:job.info.out_frames]


class Span192(ShardedTrack):
    """This rank's run of a chunk-sharded track's 192 kHz stream in loudnorm's dynamic
    mode (ShardedTrack._dynamic_sharded): a measure-only job over the frames of its
    filter segments with ShardedTrack's exchanges -- edges (the alimiter's halo),
    K-filter tails + sample peaks (all-gather), hop energies (all-reduce), the
    alimiter's state hand-off (chain_state_speculative).  Only those exchange methods
    and measure() / limit() are used on it: it has no chunks, so ShardedTrack's
    step / capture / replay do not apply."""

    def __init__(self, spans, rank, world, group, lufs, device):
        self.rank, self.world, self.group = rank, world, group
        self.xchg, self.dyn = True, False
        self.span_frames = [int(v) for v in spans]
        self.tframe0 = sum(self.span_frames[:rank])
        self.ttotal = sum(self.span_frames)
        n = self.span_frames[rank]
        self.job = MasteringJob(192000, 2, {"lufs": lufs}, [n], input_s16=True, chunks=[(0, 0, n)],
                                track_frame0=[self.tframe0], track_total=[self.ttotal], device=device,
                                measure_only=True, seg_frames=1024)    # the K scan's window at 192 kHz
        self.fast = None
        self._setup_exchange()

    def measure(self, lufs_on):
        """the stream's loudness (lufs_on) and peaks from the runs, as ShardedTrack.step
        measures the chain output: every rank ends with the same statistics row.  Without
        the loudness only the limiter's input bound is needed: the filter's ceiling
        (engine.ln_output_bound), the same on every rank"""
        from .engine import ln_output_bound
        job = self.job
        self.exchange_edges()
        bound = None if lufs_on else ln_output_bound(self.ttotal)
        if bound is not None:
            job.peak.fill_(bound)
        else:
            job.loudness_pass1(tail=True)
            self.exchange_carry_peaks()
        job.dd.lufs_on = 1 if lufs_on else 0
        if lufs_on:
            job.loudness_pass2(carry=True)
            reduce_loudness(job.hops, None, self.group)
            job.histograms()
        job.decide()

    def limit(self):
        """the alimiter (:223) over the runs: the device's decision (the same on every
        rank) picks the idle path or the rank-to-rank state hand-off"""
        from . import capi
        job = self.job
        self.fast = bool(int(job.ctl[0].item()) & capi.CTL_FAST)
        if self.fast:
            job.finalize(True)
        else:
            job.lim_state.zero_()
            self.limiter_sequential()
        return job.y[:self.span_frames[self.rank]]


class ShardedBatch:
    """This rank's share of a batch of whole tracks (BASELINE configs[3], C4: 64 tracks
    over 8 GPUs).  Tracks are dealt to ranks as contiguous runs balanced by frames
    (shard_tracks); loudness and the limiter are per track, so a batch needs no
    exchange at all: each rank runs one MasteringJob over its tracks, laid back to
    back in its input buffer, every track chunked exactly as on its own
    (audio_mastering_engine.py:178)."""

    def __init__(self, sample_rate, channels_in, settings, track_frames, rank, world, *,
                 quantum=None, input_s16=False, seg_frames=128):
        self.rank, self.world = rank, world
        fs = int(sample_rate)
        if quantum is None:
            quantum = packet_frames(channels_in * (2 if input_s16 else 4))
        self.track_frames = [int(n) for n in track_frames]
        self.ranges = shard_tracks(self.track_frames, world)
        t0, t1 = self.ranges[rank]
        self.tracks = list(range(t0, t1))
        mine = self.track_frames[t0:t1]
        self.local_frames = sum(mine)
        self.in0 = sum(self.track_frames[:t0])
        mb = bool(settings.get("multiband"))
        self.track_bounds = [chunk_bounds(n, fs, quantum) for n in self.track_frames]
        out_t = [sum(chunk_out_frames(n, fs, mb) for _, n in b) for b in self.track_bounds]
        self.span_frames = [sum(out_t[a:b]) for a, b in self.ranges]
        self.job = MasteringJob(fs, channels_in, settings, mine, quantum=quantum,
                                input_s16=input_s16, seg_frames=seg_frames)

    def step(self, d_in):
        """One pass of the whole path over this rank's tracks (input resident)."""
        y = self.job.run(d_in)
        self.job.report = {"chunks": len(self.job.chunks), "segments": self.job.info.n_segments,
                           "tracks": len(self.tracks)}
        return y

    def capture(self, d_in):
        return self.job.capture(d_in)

    def replay(self):
        return self.job.replay()

    def flush(self):
        """ShardedTrack's interface: a batch step needs no host resolution"""
        return None

    def close(self):
        """MasteringJob.close on this rank's job (graph first, then the plan)"""
        self.job.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def finish_dynamic(self):
        """After a step: finish this rank's tracks that loudnorm sends to dynamic mode
        (MasteringJob.finish_dynamic); returns {global track index: info}."""
        info = self.job.finish_dynamic()
        return {self.tracks[t]: v for t, v in info.items()}

    def track_output(self, k):
        """global track k's output (192 kHz after finish_dynamic if it took dynamic mode)"""
        return self.job.track_output(self.tracks.index(k))
