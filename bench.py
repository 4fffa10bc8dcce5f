"""Benchmark: mastered Msamples/s (48 kHz stereo f32) at N GPUs + HBM roofline.

Workload (default configs[2], C3 -- the north_star's "fused EQ -> multiband-comp ->
LUFS chain"): per rank a 5-minute stereo 48 kHz float32 program (synthetic, seeded),
mastered with the "Vocal Clarity" EQ preset, width 1.3, analog character 40 %, the
3-band multiband compressor (GUI default thresholds / ratios) and loudness
normalisation to -14 LUFS, i.e. the whole process_audio_with_ffmpeg_pipeline path
(audio_mastering_engine.py:171-226): chunk chain + concat, loudnorm measurement +
linear gain, alimiter.  At N GPUs the job is ONE track of N x 5 min, chunk-sharded
over the ranks (weak scaling) with the RCCL all-reduce of the loudness partials.
Input is resident in HBM before timing; the output (16-bit PCM, what the reference
writes) stays in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5] [--strong]

--gpus N > 1 without a launcher starts the N ranks itself (a child
`python -m torch.distributed.run --nproc-per-node N`, one process per GPU); under a
launcher WORLD_SIZE must equal N (else exit 2).

c2 = configs[1] (EQ + loudnorm + alimiter), c4 = configs[3] (8 whole 4-minute tracks
per GPU, track-sharded, no exchange), c5 = configs[4] (60 min at 96 kHz per GPU).
--strong: ONE track of the config's length split over the N ranks (configs[4] as
BASELINE.json states it: one 60-min 96 kHz track chunk-sharded over 8 GPUs).
At N = 1 the default run also times C2, C4 and C5 on the GPU (``other_configs``:
hipGraph replays, no CPU leg), so every config has a number from the driver's run.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFS = 78.6           # MI355X fp64 vector, spec (half the 157.3 TF fp32 rate); measured 68
FP32_PEAK_TFS = 157.3          # MI355X fp32 vector, spec
CHAIN_BYTES = 8                # 4 B f32 read + 4 B write per channel-sample (chain)
E2E_BYTES = 16                 # + the gain / limiter pass

VOCAL = dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0)
MB = dict(multiband=True, low_thresh=-25.0, low_ratio=6.0, mid_thresh=-20.0, mid_ratio=3.0,
          high_thresh=-15.0, high_ratio=4.0)
C3 = dict(VOCAL, lufs=-14.0, width=1.3, analog_character=40.0, **MB)
CONFIGS = {
    "c2": dict(VOCAL, lufs=-14.0),
    "c3": C3,
    "c4": C3,
    "c5": C3,
}
# sample rate, seconds per track, tracks per GPU (BASELINE.json configs)
CONFIG_FS = {"c2": 48000, "c3": 48000, "c4": 48000, "c5": 96000}
CONFIG_SECONDS = {"c2": 300.0, "c3": 300.0, "c4": 240.0, "c5": 3600.0}
CONFIG_TRACKS = {"c2": 1, "c3": 1, "c4": 8, "c5": 1}
WORKLOAD = {
    "c2": "configs[1]: 5 min stereo 48 kHz f32 per GPU, EQ 'Vocal Clarity' + loudnorm -14 LUFS "
          "(linear) + alimiter; N GPUs = one N x 5 min track, chunk-sharded",
    "c3": "configs[2]: 5 min stereo 48 kHz f32 per GPU, C2 + multiband compressor (3-band "
          "crossover, GUI thresholds/ratios) + width 1.3 + analog character 40; N GPUs = one "
          "N x 5 min track, chunk-sharded",
    "c4": "configs[3]: batch of 4 min stereo 48 kHz f32 tracks, 8 per GPU (64 at N = 8), C3 "
          "settings, whole tracks sharded over the ranks (no exchange)",
    "c5": "configs[4]: 60 min stereo 96 kHz f32 per GPU, C3 settings, hipGraph-captured step",
}
# --strong: the total work is fixed, one track split over the N ranks (configs[4] as stated)
WORKLOAD_STRONG = {
    "c5": "configs[4]: ONE 60 min stereo 96 kHz f32 track, C3 settings, chunk-sharded over the N "
          "GPUs (strong scaling: the same track at every N)",
    "c3": "configs[2] settings: ONE 5 min stereo 48 kHz f32 track chunk-sharded over the N GPUs "
          "(strong scaling)",
    "c2": "configs[1] settings: ONE 5 min stereo 48 kHz f32 track chunk-sharded over the N GPUs "
          "(strong scaling)",
}
# the reference's own Python chain, 1 core (measured in the survey container):
# context for the C oracle's rate, which is ~50-90x faster than the reference
REF_PY = {"c2": (20.9, "EQ only (the C2 chain's scipy part; ffmpeg stages not measurable)"),
          "c3": (0.42, "EQ + analog + width + multiband (crossover + 3 pydub compressors)")}


def stage_bytes(stage, frames, ch_in):
    """Per-kernel byte MODEL: what each stage's kernel must read and
    write per stereo frame, x frames.  int16 stereo frame = 4 B; f32 stereo = 8 B.
    Reported beside the §8(d) roofline, not as it."""
    fin = 4 * ch_in
    per = {
        "front1": fin + 4,              # f32 input -> s16 chain input
        "front2": 4 + 4,                # s16 chain input -> s16 chunk output / P
        "up": 4,                        # 192 kHz sample pass (k_up): reads the track once
        "loud1": 0,                     # peaks + scan: per-segment states only
        "loud2": 4,                     # K-filter recursion: reads the track once
        "final": 4 + 4,                 # gain + limiter: track in -> output
        "xover": 4 + 12,                # P -> 3 bands
        "rms": 12 + 6,                  # 3 bands -> 3 x u16 rms index r (m = table[r])
        "env": 6 + 1.5,                 # r once -> 3 x f64 checkpoint per 16 frames
        "apply": 12 + 6 + 1.5 + 4,      # bands + r + checkpoints -> output
    }
    return per.get(stage, 0) * frames


def front2_flops(frames, settings, mb):
    """fp64 FLOPs of one k_front2 launch, per channel-frame:
    a 2nd-order section in DF-II-T is 9 (3 FMA + 1 mul + 1 FMA); a shelf adds its
    3-op mix (:286-289), a peak is 4 sections + its 2-op mix (:290-298); the fused
    GEMV is 2 D (K filter D = 4, crossover D = 8)."""
    per = 0
    for key, kind in (("bass_boost", "shelf"), ("mid_cut", "peak"), ("presence_boost", "peak"),
                      ("treble_boost", "shelf")):
        if float(settings.get(key, 0.0)) != 0.0:
            per += 12 if kind == "shelf" else 38
    per += 16 if mb else 8
    return per * 2 * frames


# the one kernel of each single-kernel stage (rocprofv3 short names)
STAGE_KERNEL = {"front1": "k_front1s", "front2": "k_front2", "xover": "k_xover2", "rms": "k_rms",
                "env": "k_env0", "apply": "k_gain_overlay", "final": "k_final", "up": "k_up"}
# launches per step of kernels that run more than once (the envelope fix rounds)
PER_STEP = {}   # kernels launched more than once per step (none since round 5)
# the pipeline's kernels (runtime copy / torch helper kernels excluded from step traffic)
PIPELINE_PREFIX = "k_"


def synth_generator(frames, fs):
    """the generator synth_input uses for this length (named in the bench line's data)"""
    return "amx.synth.mix_tiled(block_seconds=60)" if frames > 600 * fs else "amx.synth.mix_like"


def synth_input(frames, fs, seed, kind="mix"):
    """the seeded synthetic program; inputs longer than 10 minutes repeat a 60 s block
    (amx.synth.mix_tiled: mix_like costs ~1 s of host time per 20 s of audio).
    kind "dynamic": the programme at -18 dB with two 50-frame full-scale bursts per
    second -- true peak + offset above -1.5 dBTP, so loudnorm takes dynamic mode"""
    import numpy as np
    from amx import synth
    if frames > 600 * fs:
        x = synth.mix_tiled(frames, fs, 2, seed=seed)
    else:
        x = synth.mix_like(frames, fs, 2, seed=seed)
    if kind == "dynamic":
        x *= np.float32(0.12)
        rng = np.random.default_rng(seed + 11)
        for k in rng.integers(0, max(1, frames - 200), max(2, int(frames / fs * 2))):
            x[k:k + 50] += rng.uniform(-0.9, 0.9, (min(50, frames - k), 2)).astype(np.float32)
        np.clip(x, -1.0, 1.0, out=x)
    return x


def load_flops(config):
    """Per-launch FLOPs from the committed PMC summary (profiles/flops_<config>.json,
    scripts/gpu_flops.sh: rocprofv3 SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_{F64,F32}, one pass)."""
    path = os.path.join(ROOT, "profiles", "flops_%s.json" % config)
    try:
        return json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return None


def time_graph(runner, d_in, warmup, soak_s, min_s):
    """warm-up steps, capture, soak, then >= min_s seconds of replays; ms per step"""
    import torch
    for _ in range(warmup):
        runner.step(d_in)
    runner.capture(d_in)
    runner.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < soak_s or n < 2:
        runner.replay()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    t_est = (time.perf_counter() - t0) / n
    steps = max(5, int(math.ceil(min_s / t_est)))
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.replay()
    if hasattr(runner, "flush"):
        runner.flush()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps, steps


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    return oracle


def _threads():
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1, 16))


def oracle_tracks(tracks, fs, settings, ex):
    """The C oracle's whole pipeline (:171-226) over [(x16 track, chunk bounds)]: chunk
    chains on the thread pool `ex` (ctypes drops the GIL), loudness + alimiter serial per
    track as in the reference, the tracks themselves side by side.  Test infrastructure:
    the checker of the GPU output, never the thing measured."""
    import numpy as np
    oracle = _oracle()

    def one(xb):
        xt, bounds = xb
        outs = [oracle.chunk(xt[s:s + n], fs, settings) for s, n in bounds] if len(tracks) > 1 else \
            list(ex.map(lambda sn: oracle.chunk(xt[sn[0]:sn[0] + sn[1]], fs, settings), bounds))
        cat = np.concatenate(outs, axis=0)
        yy = cat
        if settings.get("lufs") is not None:
            mode, g = oracle.loudnorm_linear_gain(oracle.loudnorm_measure(cat, fs), float(settings["lufs"]))
            if mode == "linear":
                yy = oracle.linear_gain(cat, g)
        return oracle.alimiter(yy, fs)
    if len(tracks) == 1:
        return [one(tracks[0])]
    return list(ex.map(one, tracks))


def parity(ys, refs, what):
    """max |diff| (LSB) and the exact fraction of the GPU outputs against the oracle's"""
    import numpy as np
    mx, ex_n, n_all = 0, 0, 0
    for t, (y, ref) in enumerate(zip(ys, refs)):
        if y.shape != ref.shape:
            return {"shape_mismatch": [list(y.shape), list(ref.shape)], "track": t}
        d = np.abs(y.astype(np.int32) - ref.astype(np.int32))
        mx = max(mx, int(d.max()) if d.size else 0)
        ex_n += int((d == 0).sum())
        n_all += d.size
    return {"max_abs_lsb": mx, "exact_frac": ex_n / max(1, n_all), "tracks": len(refs), "what": what}


def other_configs(args):
    """C2, C4, C5 on this GPU (N = 1): the same step as their own bench lines (hipGraph
    replay of the whole pipeline on HBM-resident synthetic input), timed over >= 1 s;
    then each config's whole workload through the C oracle (thread pool), compared with
    the GPU output bit for bit (parity_vs_oracle); no per-stage events"""
    import gc
    from concurrent.futures import ThreadPoolExecutor
    import torch
    from amx.dist import ShardedBatch, ShardedTrack
    oracle = _oracle()
    out = {}
    for cfg in ("c2", "c4", "c5"):
        fs = CONFIG_FS[cfg]
        per_track = int(CONFIG_SECONDS[cfg] * fs)
        if cfg == "c4":
            frames = [per_track] * CONFIG_TRACKS[cfg]
            runner = ShardedBatch(fs, 2, CONFIGS[cfg], frames, 0, 1, quantum=512, seg_frames=args.seg_frames)
            xs = [synth_input(frames[t], fs, 1000 + t) for t in runner.tracks]
            x = np.concatenate(xs, axis=0)
        else:
            runner = ShardedTrack(fs, 2, CONFIGS[cfg], per_track, 0, 1, quantum=512, seg_frames=args.seg_frames)
            x = synth_input(runner.local_frames, fs, 0)
            xs = [x]
        d_in = torch.from_numpy(x).cuda()
        del x
        ms, steps = time_graph(runner, d_in, 2, 0.5, 1.0)
        samples = sum(runner.span_frames) * 2
        rep = runner.job.fetch_report()
        o = {"workload": WORKLOAD[cfg], "ms_per_step": round(ms, 4), "steps": steps,
             "data": synth_generator(per_track, fs),
             "value": round(samples / (ms / 1e3) / 1e6, 3), "unit": "Msamples/s",
             "chain_frac": round(CHAIN_BYTES * samples / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
             "loudnorm_mode": rep.get("modes"), "limiter_fast": rep.get("limiter_fast")}
        if not args.no_cpu_baseline:
            if cfg == "c4":
                ys = [runner.job.track_output(t).cpu().numpy() for t in range(len(runner.tracks))]
                tracks = [(oracle.quantize(xt), runner.track_bounds[t]) for xt, t in zip(xs, runner.tracks)]
            else:
                ys = [runner.job.y[:runner.job.info.out_frames].cpu().numpy()]
                tracks = [(oracle.quantize(xs[0]), [(s - runner.in0, n) for s, n in runner.bounds])]
            del xs
            t0 = time.perf_counter()
            with ThreadPoolExecutor(_threads()) as ex:
                refs = oracle_tracks(tracks, fs, CONFIGS[cfg], ex)
            o["parity_vs_oracle"] = dict(parity(ys, refs, "whole workload, bit for bit"),
                                         oracle_seconds=round(time.perf_counter() - t0, 2))
            del ys, refs, tracks
        if cfg == "c4":
            # the same batch captured with loudnorm's dynamic path held for every track
            # (MasteringJob.capture(dynamic=True): launched only for a track whose decision
            # says dynamic -- none here): what a product batch pays to finish loud tracks
            # in the step
            job = runner.job
            job.capture(d_in, dynamic=True)
            for _ in range(3):
                job.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            nd = 0
            while time.perf_counter() - t0 < 1.0 or nd < 5:
                job.replay()
                nd += 1
            torch.cuda.synchronize()
            msd = (time.perf_counter() - t0) * 1e3 / nd
            o["dynamic_capture"] = {"ms_per_step": round(msd, 4), "steps": nd,
                                    "overhead": round(msd / ms - 1.0, 4),
                                    "what": "capture(dynamic=True): the dynamic path held for every track"}
        out[cfg] = o
        runner.close()
        del runner, d_in
        gc.collect()
        torch.cuda.empty_cache()
    return out


def other_inputs(args):
    """loudnorm's dynamic mode (:240 when the linear conditions fail: the 192 kHz AGC,
    true-peak limiter and the alimiter at 192 kHz) on the default bench's own step: a
    quiet programme with full-scale bursts (synth_input kind "dynamic").  C3 settings on
    one 5-min 48 kHz track (per-stage times, and the whole 192 kHz output against the C
    oracle's pipeline) and C5 strong (one 60-min 96 kHz track).  The step is the same
    captured graph with the dynamic path gated on the device, replayed; the host reads
    the decision and the 192 kHz output's size back each step."""
    import gc
    import torch
    from amx.chunking import chunk_bounds
    from amx.dist import ShardedTrack
    out = {}
    for cfg, fs, seconds in (("c3", 48000, 300.0), ("c5_strong", 96000, 3600.0)):
        settings = CONFIGS["c3"]
        n = int(seconds * fs)
        runner = ShardedTrack(fs, 2, settings, n, 0, 1, quantum=512, seg_frames=args.seg_frames, dynamic=True)
        x = synth_input(runner.local_frames, fs, 0, "dynamic")
        d_in = torch.from_numpy(x).cuda()
        ms, steps = time_graph(runner, d_in, 1, 0.5, 1.0)
        y = runner.replay()
        info = dict(getattr(runner, "dyn_info", None) or {})
        o = {"settings": "c3", "sample_rate": fs, "seconds": seconds, "ms_per_step": round(ms, 4), "steps": steps,
             "value": round(2 * n / (ms / 1e3) / 1e6, 3), "unit": "Msamples/s (input rate)",
             "output_sample_rate": info.get("sample_rate"), "dynamic": info,
             "data": "synthetic: %s at -18 dB with two 50-frame full-scale bursts per second" %
                     synth_generator(n, fs)}
        job = runner.job
        if cfg == "c3":
            job.stage_events = []
            for _ in range(3):
                runner.step(d_in)
            torch.cuda.synchronize()
            st = {}
            for name, a, b in job.stage_events:
                st[name] = st.get(name, 0.0) + a.elapsed_time(b) / 3
            job.stage_events = None
            o["stages_ms"] = {k: round(v, 4) for k, v in st.items()}
            if not args.no_cpu_baseline:
                oracle = _oracle()
                y = runner.replay().cpu().numpy()
                t0 = time.perf_counter()
                ref, rinfo = oracle.pipeline(oracle.quantize(x), fs, settings, chunk_bounds(n, fs, 512))
                o["parity_vs_oracle"] = dict(parity([y], [ref], "the whole 192 kHz output, bit for bit"),
                                             oracle_mode=rinfo.get("mode"),
                                             oracle_seconds=round(time.perf_counter() - t0, 2))
        out[cfg] = o
        runner.close()
        del runner, d_in, x, y
        gc.collect()
        torch.cuda.empty_cache()
    return out


def other_rates(args):
    """C3 settings on one 5-minute track at 44.1 kHz: the rate whose 192 kHz measurement
    takes k_up_poly (M > 1) instead of k_up<4> -- not a BASELINE config, reported beside
    them; the same captured-graph step, timed over >= 1 s"""
    import gc
    import torch
    from amx.dist import ShardedTrack
    out = {}
    for fs in (44100,):
        n = int(CONFIG_SECONDS["c3"] * fs)
        runner = ShardedTrack(fs, 2, CONFIGS["c3"], n, 0, 1, quantum=512, seg_frames=args.seg_frames)
        d_in = torch.from_numpy(synth_input(runner.local_frames, fs, 0)).cuda()
        ms, steps = time_graph(runner, d_in, 2, 0.5, 1.0)
        out[str(fs)] = {"settings": "c3", "seconds": CONFIG_SECONDS["c3"], "ms_per_step": round(ms, 4),
                        "steps": steps, "value": round(2 * n / (ms / 1e3) / 1e6, 3), "unit": "Msamples/s"}
        runner.close()
        del runner, d_in
        gc.collect()
        torch.cuda.empty_cache()
    return out


def load_traffic(config):
    """Per-launch HBM bytes from the committed PMC summary (profiles/traffic_<config>.json,
    scripts/gpu_traffic.sh: rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE, separate passes)."""
    path = os.path.join(ROOT, "profiles", "traffic_%s.json" % config)
    try:
        return json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return None


def launch_plan(gpus, env, argv=None, port=None):
    """How this invocation runs its --gpus N ranks (decided before any GPU call):
      ("run", None)       -- one process per rank already: WORLD_SIZE == --gpus (a launcher
                             started us), or N = 1 with no launcher;
      ("spawn", cmd)      -- N > 1 and no launcher: start N ranks as a child
                             `python -m torch.distributed.run --nproc-per-node N` on
                             127.0.0.1 with the same arguments, and exit with its code;
      ("refuse", message) -- a launcher's WORLD_SIZE disagrees with --gpus, or N < 1.
    A bare `python bench.py --gpus 8` therefore measures 8 ranks, never one rank labelled
    n_gpus 1."""
    if gpus < 1:
        return ("refuse", "--gpus must be >= 1 (got %d)" % gpus)
    world = env.get("WORLD_SIZE")
    if world is not None:
        try:
            w = int(world)
        except ValueError:
            return ("refuse", "WORLD_SIZE=%r is not an integer" % world)
        if w != gpus:
            return ("refuse", "launched with WORLD_SIZE=%d but --gpus %d: the world size must equal "
                              "--gpus" % (w, gpus))
        return ("run", None)
    if gpus == 1:
        return ("run", None)
    if port is None:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + argv
    return ("spawn", cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: enough for a >= 2 s timed region)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--soak", type=float, default=2.0,
                    help="seconds of untimed graph replays after the warm-up, so the GPU is "
                         "visibly busy before the timed region")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--seconds", type=float, default=None, help="per track (default: the config's)")
    ap.add_argument("--tracks", type=int, default=None, help="tracks per GPU (c4; default 8)")
    ap.add_argument("--seg-frames", type=int, default=128)
    ap.add_argument("--env-warm", type=int, default=None,
                    help="compressor envelope warm-up frames (default: the plan's, 2048)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the double-buffered host rate")
    ap.add_argument("--eager", action="store_true", help="launch every kernel from the host")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: one track of the config's length split over the ranks")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="skip the GPU-only timings of the other configs (N = 1 default run)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on cuda:0 (rehearsal with --dist-backend gloo)")
    ap.add_argument("--input", default="mix", choices=("mix", "dynamic"),
                    help="dynamic: a quiet programme with full-scale bursts, so loudnorm takes "
                         "dynamic mode (the 192 kHz path; chunk-sharded at N > 1)")
    ap.add_argument("--force-exchange", action="store_true",
                    help="run the N > 1 step (graph segments + every collective) even at one rank: "
                         "an RCCL rehearsal on one GPU")
    args = ap.parse_args()

    # N ranks before anything touches the GPU: spawn them, or refuse a mismatched launch
    how, what = launch_plan(args.gpus, os.environ)
    if how == "refuse":
        print("bench.py: %s" % what, file=sys.stderr, flush=True)
        sys.exit(2)
    if how == "spawn":
        if not args.one_device:
            import torch
            have = torch.cuda.device_count()          # (counts devices without initialising them)
            if have < args.gpus:
                print("bench.py: --gpus %d but %d GPU(s) visible (--one-device --dist-backend gloo "
                      "rehearses N ranks on one)" % (args.gpus, have), file=sys.stderr, flush=True)
                sys.exit(2)
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(what, env=env))

    import numpy as np
    import torch
    import torch.distributed as dist
    from amx import capi, synth
    from amx.dist import ShardedBatch, ShardedTrack

    world = int(os.environ.get("WORLD_SIZE", "1"))
    assert world == args.gpus, (world, args.gpus)     # (launch_plan)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_dist = world > 1 or args.force_exchange
    if use_dist:
        torch.cuda.set_device(0 if args.one_device else local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group(args.dist_backend)
    fs = CONFIG_FS[args.config]
    if args.seconds is None:
        args.seconds = CONFIG_SECONDS[args.config]
    n_tr = args.tracks if args.tracks is not None else CONFIG_TRACKS[args.config]
    settings = CONFIGS[args.config]
    if args.env_warm is not None:
        settings = dict(settings, _env_warm=int(args.env_warm))
    per_track = int(args.seconds * fs)
    batch = args.config == "c4"
    if batch:
        frames = [per_track] * (n_tr * world)
        runner = ShardedBatch(fs, 2, settings, frames, rank, world, quantum=512,
                              seg_frames=args.seg_frames)
        xs = [synth_input(frames[t], fs, 1000 + t) for t in runner.tracks]
        x = np.concatenate(xs, axis=0)
    else:
        total = per_track if args.strong else per_track * world
        runner = ShardedTrack(fs, 2, settings, total, rank, world, quantum=512,
                              seg_frames=args.seg_frames, force_exchange=args.force_exchange,
                              dynamic=args.input == "dynamic")
        x = synth_input(runner.local_frames, fs, rank, args.input)
    d_in = torch.from_numpy(x).cuda()
    job = runner.job

    def barrier():
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        runner.step(d_in)
    # the step's device work is replayed from captured hipGraphs (every kernel, same
    # buffers): one graph at N = 1, the three stretches between collectives at N > 1
    graph = not args.eager
    if graph:
        runner.capture(d_in)
        runner.replay()
    run = runner.replay if graph else (lambda: runner.step(d_in))
    # soak: untimed replays for >= args.soak seconds (also sizes the default K)
    barrier()
    t0 = time.perf_counter()
    n_soak = 0
    while True:
        run()
        n_soak += 1
        if n_soak % 8 == 0 or n_soak == 1:
            if graph and hasattr(runner, "flush"):
                runner.flush()
            barrier()
            if time.perf_counter() - t0 >= args.soak:
                break
    barrier()
    soak_s = time.perf_counter() - t0
    t_est = soak_s / n_soak
    steps = args.steps if args.steps is not None else max(10, int(math.ceil(2.0 / t_est)))
    flush = getattr(runner, "flush", None) if graph else None
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    if flush is not None:
        flush()          # the pipelined N > 1 replay resolves its last step here
    barrier()
    elapsed = time.perf_counter() - t0
    if use_dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / steps
    samples_total = sum(runner.span_frames) * 2          # output channel-samples, all ranks
    samples_rank = job.info.out_frames * 2
    value = samples_total * steps / elapsed / 1e6

    # host-inclusive rate (reported beside `value`, never as it): pinned H2D of the f32
    # input, the step, D2H of the int16 output, serialised on the stream
    host_incl = None
    if world == 1:
        n_out = job.info.out_frames
        h_in = torch.from_numpy(x).pin_memory()
        h_out = torch.empty((n_out, 2), dtype=torch.int16).pin_memory()
        k_h = max(3, min(steps, 20))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(k_h):
            d_in.copy_(h_in, non_blocking=True)
            run()
            h_out.copy_(job.y[:n_out], non_blocking=True)
        torch.cuda.synchronize()
        e2e = (time.perf_counter() - t1) / k_h
        host_incl = {"value": round(samples_total / e2e / 1e6, 3), "unit": "Msamples/s",
                     "ms_per_step": round(e2e * 1e3, 4),
                     "what": "pinned H2D of the f32 input + the step + D2H of the int16 output"}
        del h_in
        # the same, double-buffered (amx.stream_io.TrackStream): H2D of track i+1, the
        # step of track i and D2H of track i-1 overlap on three streams; for f32 input
        # and for an s16 WAV input (half the H2D bytes)
        if not args.no_pipeline and not batch and fs * args.seconds <= 48000 * 600:
            from amx.stream_io import TrackStream
            host_incl["pipelined"] = {}
            for kind, s16 in (("f32", False), ("s16", True)):
                ts = TrackStream(fs, 2, settings, per_track, depth=2, input_s16=s16, quantum=512,
                                 seg_frames=args.seg_frames)
                hi = ts.pinned_input()
                hi.copy_(torch.from_numpy(synth.to_s16(x)) if s16 else torch.from_numpy(x))
                outs = [ts.pinned_output() for _ in range(2)]
                n_p = max(4, min(steps, 20))
                ts.run([hi] * 2, outs)                        # warm-up
                t1 = time.perf_counter()
                ts.run([hi] * n_p, [outs[i % 2] for i in range(n_p)])
                e2p = (time.perf_counter() - t1) / n_p
                host_incl["pipelined"][kind] = {
                    "value": round(samples_total / e2p / 1e6, 3), "ms_per_track": round(e2p * 1e3, 4),
                    "tracks": n_p, "h2d_bytes": int(hi.numel() * hi.element_size()),
                    "d2h_bytes": int(outs[0].numel() * 2)}
                del ts, hi, outs

    # per-stage device time: steps again with HIP events bracketing each stage on the
    # launch stream (kept out of the timed region above)
    n_ev = max(3, min(steps, 20))
    job.stage_events = []
    for _ in range(n_ev):
        runner.step(d_in)
    barrier()
    per_stage = {}
    for name, a, b in job.stage_events:
        per_stage[name] = per_stage.get(name, 0.0) + a.elapsed_time(b)
    per_stage = {k: v / n_ev for k, v in per_stage.items()}
    job.stage_events = None
    env_ctr = job.env_counters() if settings.get("multiband") else None
    report = job.fetch_report(raise_dynamic=False)
    frames = runner.local_frames
    mb = bool(settings.get("multiband"))
    # dominant kernel: the slowest single-kernel stage
    cand = {k: v for k, v in per_stage.items() if k in STAGE_KERNEL}
    dom = max(cand, key=cand.get)
    dom_stage_ms = cand[dom]
    dom_ms = dom_stage_ms
    dom_timing = "HIP events around the stage in an eager step (launch overhead included)"
    if dom in capi.STAGES:
        # the stage's one kernel launched back to back on the job's stream between two HIP
        # events: the per-launch host overhead of the eager step is amortised, as in the
        # captured graph (the stage is idempotent: it recomputes its outputs from the same
        # inputs)
        reps = 20
        st_ = torch.cuda.current_stream()
        L_ = capi.load()
        sid = capi.STAGES.index(dom)
        ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ea.record(st_)
        for _ in range(reps):
            capi.check(L_.amx_run_stage(job.plan.h, sid, capi.ptr(d_in), capi.ptr(job.out), capi.ptr(job.ws),
                                        job._s(st_)), "amx_run_stage")
        eb.record(st_)
        eb.synchronize()
        dom_ms = ea.elapsed_time(eb) / reps
        dom_timing = "HIP events around %d back-to-back launches of the stage's kernel on its stream" % reps
    kern = STAGE_KERNEL[dom]
    alg_bytes = CHAIN_BYTES * samples_rank                 # SURVEY §8(d) per launch
    achieved = alg_bytes / (dom_ms / 1e3) / 1e9
    model_bytes = stage_bytes(dom, frames, 2)
    traffic = load_traffic(args.config)
    dom_traffic = int(traffic[kern]["hbm_bytes"]) if traffic and kern in traffic else None
    step_traffic = None
    if traffic:
        step_traffic = int(sum(v["hbm_bytes"] * PER_STEP.get(k, 1) for k, v in traffic.items()
                               if k.startswith(PIPELINE_PREFIX)))
    f2_flops = front2_flops(frames, settings, mb)
    flops = load_flops(args.config)
    chain_flops = None
    if flops:
        f64 = sum(v["fp64_flops"] * PER_STEP.get(k, 1) for k, v in flops.items() if k.startswith(PIPELINE_PREFIX))
        f32 = sum(v["fp32_flops"] * PER_STEP.get(k, 1) for k, v in flops.items() if k.startswith(PIPELINE_PREFIX))
        chain_flops = {
            "fp64_flops_per_step": int(f64), "fp32_flops_per_step": int(f32),
            "fp64_per_sample": round(f64 / samples_rank, 1), "fp32_per_sample": round(f32 / samples_rank, 1),
            "achieved_fp64": round(f64 / (ms_per_step / 1e3) / 1e12, 3),
            "peak_fp64": FP64_PEAK_TFS, "unit": "TFLOP/s",
            "frac": round(f64 / (ms_per_step / 1e3) / 1e12 / FP64_PEAK_TFS, 4),
            "frac_fp64_plus_fp32": round((f64 / FP64_PEAK_TFS + f32 / FP32_PEAK_TFS) / (ms_per_step / 1e3) / 1e12, 4),
            "source": "profiles/flops_%s.json (rocprofv3 SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_{F64,F32} x 64 "
                      "lanes, FMA x 2; issued lanes, per launch) over the measured step time" % args.config}

    line = {
        "metric": "mastered Msamples/sec (48 kHz stereo f32) at 1/2/4/8 GPUs; % HBM roofline",
        "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (%s, seeded per rank / track)" % synth_generator(
            per_track if batch else runner.local_frames, fs),
        "config": {"workload": (WORKLOAD_STRONG.get(args.config, WORKLOAD[args.config]) if args.strong
                                else WORKLOAD[args.config]), "sample_rate": fs,
                   "settings": args.config, "seconds_per_track": args.seconds,
                   "tracks_per_gpu": len(runner.tracks) if batch else 1,
                   "seg_frames": args.seg_frames,
                   "parallelism": ("track-shard x%d" if batch else "chunk-shard x%d") % world,
                   "exchanges": ("%s collectives" % dist.get_backend()) if use_dist and not batch else None,
                   "launch": ("hipGraph replay" if (world == 1 and not args.force_exchange) or batch else
                              ("one hipGraph per step, RCCL collectives captured, two slots pipelined"
                               if args.dist_backend == "nccl" else
                               "hipGraph segments + eager (host-staged) collectives")) if graph else "eager"},
        "timed_region_s": round(elapsed, 4), "soak": {"seconds": round(soak_s, 3), "replays": n_soak},
        "roofline": {"bound": "hbm", "kernel": kern, "stage": dom, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": dom_traffic,
                     "bytes_per_launch": int(alg_bytes), "avg_launch_ms": round(dom_ms, 4),
                     "avg_launch_timing": dom_timing, "stage_event_ms": round(dom_stage_ms, 4),
                     "bytes_rule": "SURVEY §8(d): 8 B per output channel-sample (f32 read + write) "
                                   "x the %d channel-samples one launch processes" % samples_rank,
                     "kernel_model": {"bytes_per_launch": int(model_bytes),
                                      "achieved": round(model_bytes / (dom_ms / 1e3) / 1e9, 2),
                                      "frac": round(model_bytes / (dom_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                      "what": "the kernel's own minimum reads + writes (DESIGN.md §3.3)"},
                     "traffic_source": "profiles/traffic_%s.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                                       "per launch)" % args.config},
        "chain_roofline": {
            "bytes_per_step": int(CHAIN_BYTES * samples_rank),
            "achieved": round(CHAIN_BYTES * samples_rank / (ms_per_step / 1e3) / 1e9, 2),
            "frac": round(CHAIN_BYTES * samples_rank / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "frac_end_to_end": round(E2E_BYTES * samples_rank / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "step_traffic": step_traffic,
            "what": "whole step (every kernel) at SURVEY §8(d)'s 8 B/sample chain and 16 B/sample "
                    "end-to-end; step_traffic = the PMC bytes of every pipeline kernel per step"},
        "chain_flop_frac": chain_flops,
        "host_inclusive": host_incl,
        "roofline_fp64": {"bound": "fp64", "kernel": "k_front2",
                          "achieved": round(f2_flops / (per_stage["front2"] / 1e3) / 1e12, 2),
                          "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                          "frac": round(f2_flops / (per_stage["front2"] / 1e3) / 1e12 / FP64_PEAK_TFS, 4),
                          "flops_per_launch": int(f2_flops)},
        "stages_ms": {k: round(v, 4) for k, v in per_stage.items()},
        "plan": {"segments": int(job.info.n_segments), "seg_frames": int(job.info.seg_frames),
                 "scan_window_eq": int(job.info.scan_levels_eq),
                 "scan_window_xover": int(job.info.scan_levels_xover),
                 "scan_window_kw": int(job.info.scan_levels_kw)},
        "env_fixup": env_ctr,
        "limiter_fast": report.get("limiter_fast"),
        "loudnorm": report.get("stats"),
        "loudnorm_mode": report.get("modes"),
    }
    if args.input == "dynamic":
        # value counts the chain's input-rate samples; the step ends in the 192 kHz stream
        line["dynamic"] = dict(getattr(runner, "dyn_info", None) or {}, input=args.input)
        line["data"] += "; quiet programme with full-scale bursts (loudnorm dynamic mode)"
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.input == "mix":
        line.update(cpu_leg(args, runner, x, fs, settings, job, batch))
    if rank == 0 and world == 1 and args.config == "c3" and not args.no_other_configs:
        line["other_configs"] = other_configs(args)
        line["other_rates"] = other_rates(args)
        line["other_inputs"] = {"dynamic": other_inputs(args)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    # the captured graphs (RCCL nodes at N > 1) go before the process group
    runner.close()
    if use_dist:
        dist.destroy_process_group()


def cpu_leg(args, runner, x, fs, settings, job, batch):
    """cpu_baseline (the C oracle, 1 core, on a bounded sample of the workload) and
    parity_vs_oracle (the oracle over the WHOLE workload, chunk chains on a thread
    pool, compared bit for bit with the GPU output)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from concurrent.futures import ThreadPoolExecutor
    out = {}
    x16 = oracle.quantize(x)
    if batch:
        tracks = []
        off = 0
        for t in runner.tracks:
            n = runner.track_frames[t]
            tracks.append((x16[off:off + n], runner.track_bounds[t]))
            off += n
    else:
        tracks = [(x16, [(s - runner.in0, n) for s, n in runner.bounds])]
    threads = _threads()

    # 1 core on a bounded sample: whole chunks of the first track, up to ~20 s of audio
    # per... as many chunks as fit ~10-30 s of CPU (the whole 5-min track at C2/C3)
    xt0, b0 = tracks[0]
    nch = len(b0) if fs * args.seconds <= 48000 * 300 else max(1, min(len(b0), 10))
    sb = b0[:nch]
    s_end = sb[-1][0] + sb[-1][1]
    t0 = time.perf_counter()
    ref1, _ = oracle.pipeline(xt0[:s_end], fs, settings, sb)
    dt = time.perf_counter() - t0
    rp = REF_PY.get("c2" if args.config == "c2" else "c3")
    out["cpu_baseline"] = {
        "value": round(s_end * 2 / dt / 1e6, 3), "unit": "Msamples/s", "cores": 1, "kind": "port",
        "sample": "%d of %d chunks (%.0f s of audio) of the first track through the whole C oracle "
                  "pipeline (oracle/amx_oracle.c), single thread" % (nch, len(b0), s_end / fs),
        "seconds": round(dt, 3),
        "reference_python_context": {
            "value": rp[0], "unit": "Msamples/s", "cores": 1,
            "what": "the reference's own Python chain (%s), BASELINE.md, survey container -- "
                    "the C oracle above is faster than the reference itself" % rp[1]}}
    # whole workload on all cores (chunk chains on a thread pool; loudness + alimiter
    # serial per track, as in the reference) -- also the parity reference
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        refs = oracle_tracks(tracks, fs, settings, ex)
    dtp = time.perf_counter() - t0
    tot = sum(xt.shape[0] for xt, _ in tracks)
    out["cpu_baseline"]["all_cores"] = {
        "value": round(tot * 2 / dtp / 1e6, 3), "cores": threads, "seconds": round(dtp, 3),
        "what": "the whole workload: chunk chains on a thread pool, loudness + alimiter serial"}
    if nch == len(b0):
        out["cpu_baseline"]["all_cores"]["same_output_as_1_core"] = bool(np.array_equal(refs[0], ref1))
    ys = [(job.track_output(t) if batch else job.y[:job.info.out_frames]).cpu().numpy() for t in range(len(refs))]
    out["parity_vs_oracle"] = parity(ys, refs, "whole workload, bit for bit")
    return out


if __name__ == "__main__":
    main()
