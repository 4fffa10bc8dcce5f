"""Benchmark: mastered Msamples/s (48 kHz stereo f32) at N GPUs + HBM roofline.

Workload (BASELINE.json configs[1], the metric's single-GPU config): per rank a
5-minute stereo 48 kHz float32 program (synthetic, seeded), mastered with the
"Vocal Clarity" EQ preset and loudness normalisation to -14 LUFS, i.e. the whole
process_audio_with_ffmpeg_pipeline path (audio_mastering_engine.py:171-226):
chunk chain + concat, loudnorm measurement + linear gain, alimiter.  At N GPUs the
job is ONE track of N x 5 min, chunk-sharded over the ranks (weak scaling) with the
RCCL all-reduce of the loudness partials.  Input is resident in HBM before timing;
output (16-bit PCM, what the reference writes) stays in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector (spec)

VOCAL = dict(bass_boost=-1.0, mid_cut=2.0, presence_boost=2.5, treble_boost=1.0)
MB = dict(multiband=True, low_thresh=-25.0, low_ratio=6.0, mid_thresh=-20.0, mid_ratio=3.0,
          high_thresh=-15.0, high_ratio=4.0)
CONFIGS = {
    "c2": dict(VOCAL, lufs=-14.0),
    "c3": dict(VOCAL, lufs=-14.0, width=1.3, analog_character=40.0, **MB),
    "c5": dict(VOCAL, lufs=-14.0, width=1.3, analog_character=40.0, **MB),
}
# sample rate and default length per config (BASELINE.json configs; C5 = 60 min at 96 kHz)
CONFIG_FS = {"c2": 48000, "c3": 48000, "c5": 96000}
CONFIG_SECONDS = {"c2": 300.0, "c3": 300.0, "c5": 3600.0}


def stage_bytes(stage, frames, ch_in, mb):
    """Algorithmic HBM bytes of one launch: what the stage must read
    and write per frame, x frames.  int16 stereo frame = 4 B; f32 stereo = 8 B."""
    fin = 4 * ch_in
    per = {
        "front1": fin + 4,              # f32 input -> s16 chain input
        "front2": 4 + 4,                # s16 chain input -> s16 chunk output / P
        "loud1": 4,                     # K-filter GEMV + peak: reads the track once
        "loud2": 4,                     # K-filter recursion: reads the track once
        "final": 4 + 4,                 # gain + limiter: track in -> output
        "xover": 4 + 12,                # P -> 3 bands
        "rms": 12 + 24,                 # 3 bands -> 3 x f64 max attenuation m
        "env": 24 + 1.5,                # m once -> 3 x f64 checkpoint per 16 frames
        "apply": 12 + 24 + 1.5 + 4,     # bands + m + checkpoints -> output
    }
    return per.get(stage, 0) * frames


FP64_PEAK_TFS = 78.6   # MI355X fp64 vector, spec (half the 157.3 TF fp32 rate); measured 68


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


# kernels of each stage (rocprofv3 short names) for the PMC traffic lookup
STAGE_KERNELS = {
    "front1": ("k_front1s", "k_front1"), "front2": ("k_front2",), "xover": ("k_xover2",),
    "rms": ("k_rms",), "env": ("k_env0", "k_envfix"), "apply": ("k_gain_overlay",),
    "loud1": ("k_kw1", "k_peak_reduce"), "loud2": ("k_kw2", "k_hops"), "final": ("k_final",),
}


def stage_traffic(stage, config):
    """HBM bytes per launch of `stage` from the committed PMC summary
    (profiles/traffic_<config>.json, scripts/gpu_traffic.sh), or None."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                        "traffic_%s.json" % config)
    try:
        ks = json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    names = STAGE_KERNELS.get(stage, ())
    hit = [v["hbm_bytes"] for k, v in ks.items() if k in names]
    return int(sum(hit)) if hit else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--seconds", type=float, default=None, help="per GPU (default: the config's)")
    ap.add_argument("--seg-frames", type=int, default=128)
    ap.add_argument("--env-warm", type=int, default=None,
                    help="compressor envelope warm-up frames (default: the plan's, 2048)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the double-buffered host rate")
    ap.add_argument("--eager", action="store_true", help="launch every kernel from the host")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm); gloo only to rehearse N ranks on one GPU")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on cuda:0 (rehearsal with --dist-backend gloo)")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist
    from amx import synth
    from amx.dist import ShardedTrack

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(0 if args.one_device else local)
        dist.init_process_group(args.dist_backend)
    fs = CONFIG_FS[args.config]
    if args.seconds is None:
        args.seconds = CONFIG_SECONDS[args.config]
    settings = CONFIGS[args.config]
    if args.env_warm is not None:
        settings = dict(settings, _env_warm=int(args.env_warm))
    per_rank = int(args.seconds * fs)
    total = per_rank * world
    track = ShardedTrack(fs, 2, settings, total, rank, world, quantum=512,
                         seg_frames=args.seg_frames)
    x = synth.mix_like(track.local_frames, fs, 2, seed=rank)
    d_in = torch.from_numpy(x).cuda()
    job = track.job

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        track.step(d_in)
    # the step's device work is replayed from captured hipGraphs (every kernel, same
    # buffers): one graph at N = 1, the three stretches between collectives at N > 1
    graph = not args.eager
    if graph:
        track.capture(d_in)
        track.replay()
    run = track.replay if graph else (lambda: track.step(d_in))
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1000.0 / args.steps
    samples_total = sum(track.span_frames) * 2          # output channel-samples, all ranks
    value = samples_total * args.steps / elapsed / 1e6

    # host-inclusive rate (reported beside `value`, never as it): pinned H2D of the f32
    # input, the step, D2H of the int16 output, serialised on the stream
    host_incl = None
    if world == 1:
        n_out = job.info.out_frames
        h_in = torch.from_numpy(x).pin_memory()
        h_out = torch.empty((n_out, 2), dtype=torch.int16).pin_memory()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            d_in.copy_(h_in, non_blocking=True)
            run()
            h_out.copy_(job.y[:n_out], non_blocking=True)
        torch.cuda.synchronize()
        e2e = (time.perf_counter() - t1) / args.steps
        host_incl = {"value": round(samples_total / e2e / 1e6, 3), "unit": "Msamples/s",
                     "ms_per_step": round(e2e * 1e3, 4),
                     "what": "pinned H2D of the f32 input + the step + D2H of the int16 output"}
        # the same, double-buffered (amx.stream_io.TrackStream): H2D of track i+1, the
        # step of track i and D2H of track i-1 overlap on three streams; for f32 input
        # and for an s16 WAV input (half the H2D bytes)
        if not args.no_pipeline:
            from amx.stream_io import TrackStream
            host_incl["pipelined"] = {}
            del h_in
            for kind, s16 in (("f32", False), ("s16", True)):
                ts = TrackStream(fs, 2, settings, per_rank, depth=2, input_s16=s16, quantum=512,
                                 seg_frames=args.seg_frames)
                hi = ts.pinned_input()
                hi.copy_(torch.from_numpy(synth.to_s16(x)) if s16 else torch.from_numpy(x))
                outs = [ts.pinned_output() for _ in range(2)]
                n_tr = max(4, args.steps)
                ts.run([hi] * 2, outs)                        # warm-up
                t1 = time.perf_counter()
                ts.run([hi] * n_tr, [outs[i % 2] for i in range(n_tr)])
                e2p = (time.perf_counter() - t1) / n_tr
                host_incl["pipelined"][kind] = {
                    "value": round(samples_total / e2p / 1e6, 3), "ms_per_track": round(e2p * 1e3, 4),
                    "tracks": n_tr, "h2d_bytes": int(hi.numel() * hi.element_size()),
                    "d2h_bytes": int(outs[0].numel() * 2)}
                del ts, hi, outs

    # per-stage device time: the same K steps again with HIP events bracketing each
    # stage on the launch stream (kept out of the timed region above)
    job.stage_events = []
    for _ in range(args.steps):
        track.step(d_in)
    barrier()
    per_stage = {}
    for name, a, b in job.stage_events:
        per_stage[name] = per_stage.get(name, 0.0) + a.elapsed_time(b)
    per_stage = {k: v / args.steps for k, v in per_stage.items()}
    job.stage_events = None
    report = job.fetch_report()
    frames = track.local_frames
    mb = bool(settings.get("multiband"))
    candidates = {k: v for k, v in per_stage.items() if stage_bytes(k, frames, 2, mb) > 0}
    dom = max(candidates, key=candidates.get)
    dom_ms = candidates[dom]
    dom_bytes = stage_bytes(dom, frames, 2, mb)
    achieved = dom_bytes / (dom_ms / 1e3) / 1e9
    f2_flops = front2_flops(frames, settings, mb)

    line = {
        "metric": "mastered Msamples/sec (48 kHz stereo f32) at 1/2/4/8 GPUs; % HBM roofline",
        "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (amx.synth.mix_like, seeded per rank)",
        "config": {"workload": "configs[1]: 5 min stereo 48 kHz f32 per GPU, EQ 'Vocal Clarity' + "
                               "loudnorm -14 LUFS (linear) + alimiter; N GPUs = one N x 5 min track, "
                               "chunk-sharded" if args.config == "c2" else
                               ("configs[2]: C2 + multiband + width 1.3 + analog 40" if args.config == "c3"
                                else "configs[4]: 60 min stereo 96 kHz f32 per GPU, C3 settings"),
                   "sample_rate": fs,
                   "settings": args.config, "seconds_per_gpu": args.seconds,
                   "seg_frames": args.seg_frames, "parallelism": "chunk-shard x%d" % world,
                   "launch": ("hipGraph replay" if world == 1 else "hipGraph segments + eager collectives")
                             if graph else "eager"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "bytes_per_launch": int(dom_bytes), "avg_launch_ms": round(dom_ms, 4),
                     "traffic": stage_traffic(dom, args.config),
                     "traffic_source": "profiles/traffic_%s.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)"
                                       % args.config},
        "host_inclusive": host_incl,
        "roofline_fp64": {"bound": "fp64", "kernel": "front2",
                          "achieved": round(f2_flops / (per_stage["front2"] / 1e3) / 1e12, 2),
                          "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                          "frac": round(f2_flops / (per_stage["front2"] / 1e3) / 1e12 / FP64_PEAK_TFS, 4),
                          "flops_per_launch": int(f2_flops)},
        "stages_ms": {k: round(v, 4) for k, v in per_stage.items()},
        "plan": {"segments": int(job.info.n_segments), "seg_frames": int(job.info.seg_frames),
                 "scan_window_eq": int(job.info.scan_levels_eq),
                 "scan_window_xover": int(job.info.scan_levels_xover),
                 "scan_window_kw": int(job.info.scan_levels_kw)},
        "limiter_fast": report.get("limiter_fast"),
        "loudnorm": report.get("stats"),
        "loudnorm_mode": report.get("modes"),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        x16 = oracle.quantize(x)
        c = [(s - track.in0, n) for s, n in track.bounds]
        t0 = time.perf_counter()
        ref, _ = oracle.pipeline(x16, fs, settings, c)
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": round(x16.shape[0] * 2 / dt / 1e6, 3), "unit": "Msamples/s",
                                "cores": 1, "kind": "port",
                                "sample": "full workload: 1 pass of the %.0f s track through the C "
                                          "oracle (oracle/amx_oracle.c), single thread" % args.seconds,
                                "seconds": round(dt, 3)}
        # all-cores variant: the chunks are independent (:185-204), so a
        # thread pool runs the oracle's chunk chain on them at once (ctypes releases the
        # GIL); loudness, gain and the alimiter stay serial, as in the reference
        threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1,
                             len(c)))
        from concurrent.futures import ThreadPoolExecutor
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            outs = list(ex.map(lambda sn: oracle.chunk(x16[sn[0]:sn[0] + sn[1]], fs, settings), c))
        cat = np.concatenate(outs, axis=0)
        yy = cat
        if settings.get("lufs") is not None:
            mode, g = oracle.loudnorm_linear_gain(oracle.loudnorm_measure(cat, fs), float(settings["lufs"]))
            if mode == "linear":
                yy = oracle.linear_gain(cat, g)
        ref_p = oracle.alimiter(yy, fs)
        dtp = time.perf_counter() - t0
        line["cpu_baseline"]["all_cores"] = {
            "value": round(x16.shape[0] * 2 / dtp / 1e6, 3), "cores": threads, "seconds": round(dtp, 3),
            "what": "chunk chains on a thread pool, loudness + alimiter serial",
            "same_output": bool(np.array_equal(ref_p, ref))}
        y = job.y[:job.info.out_frames].cpu().numpy()
        d = np.abs(y.astype(np.int32) - ref.astype(np.int32))
        line["parity_vs_oracle"] = {"max_abs_lsb": int(d.max()), "exact_frac": float((d == 0).mean())}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
