"""Host <-> device streaming of many tracks ("pinned-memory
H2D/D2H double-buffering, so end-to-end throughput approaches the kernel
throughput").

The reference masters one file at a time, serially: read, process, write
(audio_mastering_engine.py:171-226).  A file-to-file job here is bound by PCIe,
not by the kernels: one 5-minute f32 track is 115 MB in and 58 MB out against a
0.35 ms device step.  ``TrackStream`` keeps ``depth`` complete mastering jobs
resident, each with its own device buffers and its own captured hipGraph, and
moves batches through three HIP streams:

    copy-in stream   H2D of track i + 1 (pinned host -> slot (i + 1) % depth)
    compute stream   graph replay of track i (chunk chain .. limiter)
    copy-out stream  D2H of track i - 1's int16 output and loudnorm statistics

Events order each slot's reuse: a slot's input is rewritten only after its
previous step consumed it, and its output is recomputed only after the previous
D2H of it finished.  H2D and D2H use the two directions of the link at once, so
the steady-state time per track is max(H2D, D2H, step) instead of their sum.
"""
import torch

from .engine import MasteringJob


class TrackStream:
    """``depth`` resident jobs for tracks of ``frames`` frames each (same settings)."""

    def __init__(self, sample_rate, channels_in, settings, frames, *, depth=2, input_s16=False,
                 quantum=None, seg_frames=128):
        if depth < 2:
            raise ValueError("TrackStream needs depth >= 2 to overlap copies with compute")
        self.depth = int(depth)
        self.frames = int(frames)
        self.channels_in = int(channels_in)
        self.input_s16 = bool(input_s16)
        dt = torch.int16 if input_s16 else torch.float32
        self.jobs, self.d_in = [], []
        for _ in range(self.depth):
            job = MasteringJob(sample_rate, channels_in, settings, [self.frames], quantum=quantum,
                               input_s16=input_s16, seg_frames=seg_frames)
            d_in = torch.zeros((self.frames, self.channels_in), dtype=dt, device=job.device)
            job.capture(d_in)
            self.jobs.append(job)
            self.d_in.append(d_in)
        self.out_frames = self.jobs[0].info.out_frames
        self.s_in = torch.cuda.Stream()
        self.s_comp = torch.cuda.Stream()
        self.s_out = torch.cuda.Stream()
        torch.cuda.synchronize()

    def pinned_input(self):
        dt = torch.int16 if self.input_s16 else torch.float32
        return torch.empty((self.frames, self.channels_in), dtype=dt).pin_memory()

    def pinned_output(self):
        return torch.empty((self.out_frames, 2), dtype=torch.int16).pin_memory()

    def pinned_stats(self):
        return torch.empty(self.jobs[0].stats.shape, dtype=torch.float64).pin_memory()

    def run(self, h_ins, h_outs, h_stats=None, dynamic=None):
        """Master every pinned input in ``h_ins`` into the pinned output at the same index
        (and its loudnorm statistics row into ``h_stats``); returns when all are done.

        A track loudnorm sends to dynamic mode has a 192 kHz output that does not fit its
        48 kHz slot: with ``dynamic=None`` that raises DynamicModeUnsupported; with a dict,
        each such track is stepped again after the pipeline drains and finished by
        MasteringJob.dynamic_track, and ``dynamic[i] = (int16 [n192, 2] host tensor, info)``
        (its ``h_outs[i]`` is left as the linear path wrote it)."""
        if len(h_outs) != len(h_ins) or (h_stats is not None and len(h_stats) != len(h_ins)):
            raise ValueError("h_ins, h_outs (and h_stats) must have the same length")
        for h in h_ins:
            if not h.is_pinned() or tuple(h.shape) != (self.frames, self.channels_in):
                raise ValueError("inputs must be pinned [%d, %d] tensors" % (self.frames, self.channels_in))
        for h in h_outs:
            if not h.is_pinned() or tuple(h.shape) != (self.out_frames, 2) or h.dtype != torch.int16:
                raise ValueError("outputs must be pinned int16 [%d, 2] tensors" % self.out_frames)
        if h_stats is None:
            # statistics rows always come back: the mode word is checked below
            shape = (len(h_ins),) + tuple(self.jobs[0].stats.shape)
            if getattr(self, "_rows", None) is None or self._rows.shape[0] < shape[0]:
                self._rows = torch.empty(shape, dtype=torch.float64).pin_memory()
            h_stats = [self._rows[i] for i in range(len(h_ins))]
        cur = torch.cuda.current_stream()
        for s in (self.s_in, self.s_comp, self.s_out):
            s.wait_stream(cur)
        consumed = [None] * self.depth     # step done reading slot's input
        drained = [None] * self.depth      # D2H done reading slot's output
        for i, h in enumerate(h_ins):
            k = i % self.depth
            job = self.jobs[k]
            with torch.cuda.stream(self.s_in):
                if consumed[k] is not None:
                    self.s_in.wait_event(consumed[k])
                self.d_in[k].copy_(h, non_blocking=True)
                loaded = torch.cuda.Event()
                loaded.record(self.s_in)
            with torch.cuda.stream(self.s_comp):
                self.s_comp.wait_event(loaded)
                if drained[k] is not None:
                    self.s_comp.wait_event(drained[k])
                job.replay()
                consumed[k] = torch.cuda.Event()
                consumed[k].record(self.s_comp)
            with torch.cuda.stream(self.s_out):
                self.s_out.wait_event(consumed[k])
                h_outs[i].copy_(job.y[:self.out_frames], non_blocking=True)
                if h_stats is not None:
                    h_stats[i].copy_(job.stats, non_blocking=True)
                drained[k] = torch.cuda.Event()
                drained[k].record(self.s_out)
        for s in (self.s_in, self.s_comp, self.s_out):
            cur.wait_stream(s)
        torch.cuda.synchronize()
        # the device decided each track's loudnorm mode; a track that needs dynamic mode
        # must not pass as mastered (its gain would silently be "none")
        dyn = [i for i, r in enumerate(h_stats) if int(r.reshape(-1, r.shape[-1])[:, 8].max()) == 3]
        if dyn and dynamic is None:
            from .engine import DynamicModeUnsupported
            raise DynamicModeUnsupported("track %d: loudnorm would use dynamic mode" % dyn[0])
        for i in dyn:
            job = self.jobs[0]
            self.d_in[0].copy_(h_ins[i])
            job.replay()
            rep = job.fetch_report(raise_dynamic=False)
            y, info = job.dynamic_track(0, rep["stats"][0])
            dynamic[i] = (y.cpu(), info)
        return h_outs
