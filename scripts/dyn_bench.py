"""Time loudnorm's dynamic mode on the GPU (MasteringJob.dynamic_track: pass 1's filter run,
the 192 kHz measurement of its output, pass 2's filter run, the alimiter at 192 kHz) for a
track that takes it, beside the C oracle's af_loudnorm on a bounded sample.

    python scripts/dyn_bench.py [--seconds 300] [--reps 3] [--cpu-seconds 20]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def signal(seconds, fs, seed):
    from amx import synth
    n = int(fs * seconds)
    x = synth.mix_like(n, fs, 2, seed=seed) * 0.12
    rng = np.random.default_rng(seed)
    for k in rng.integers(0, n - 200, max(2, int(seconds * 2))):
        x[k:k + 50] += rng.uniform(-0.9, 0.9, (50, 2))
    return np.clip(x, -1.0, 1.0).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--batch", type=int, default=0,
                    help="also time a batch of this many dynamic tracks: one after another "
                         "(dynamic_track) and side by side (finish_dynamic)")
    args = ap.parse_args()
    import torch
    from amx.engine import MasteringJob
    fs = 48000
    settings = dict(bass_boost=1.0, lufs=-14.0)
    x = signal(args.seconds, fs, 11)
    job = MasteringJob(fs, 2, settings, [x.shape[0]])
    d_in = torch.from_numpy(x).cuda()
    job.run(d_in)
    rep = job.fetch_report(raise_dynamic=False)
    assert rep["modes"][0] == "dynamic", rep
    y, info = job.dynamic_track(0, rep["stats"][0])       # warm-up (plans, buffers)
    torch.cuda.synchronize()
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        y, info = job.dynamic_track(0, rep["stats"][0])
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    gpu_s = min(times)
    out = {"what": "loudnorm dynamic mode (pass-1 filter + its 192 kHz measurement + pass-2 filter "
                   "+ alimiter at 192 kHz) after the chain, one %g s stereo 48 kHz track" % args.seconds,
           "gpu_s": round(gpu_s, 4), "reps": times, "pass1": rep["stats"][0], "info": info,
           "out_frames_192k": int(y.shape[0])}
    # CPU: the oracle's af_loudnorm (both passes + alimiter) on a bounded sample
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    n = int(fs * args.cpu_seconds)
    x16 = O.quantize(x[:n])
    t0 = time.perf_counter()
    st = O.loudnorm_measure(x16, fs)
    p1 = O.loudnorm_pass1(x16, fs, -14.0)
    y2, _ = O.loudnorm(x16, fs, -14.0, measured=st, offset=float(p1["target_offset"]))
    O.alimiter(y2, 192000)
    cpu_s = time.perf_counter() - t0
    out["cpu_oracle"] = {"seconds_of_audio": args.cpu_seconds, "s": round(cpu_s, 3),
                         "realtime_x": round(args.cpu_seconds / cpu_s, 1), "cores": 1}
    out["gpu_realtime_x"] = round(args.seconds / gpu_s, 1)
    if args.batch > 1:
        xs = [signal(args.seconds, fs, 11 + k) for k in range(args.batch)]
        bj = MasteringJob(fs, 2, settings, [v.shape[0] for v in xs])
        bj.run(torch.from_numpy(np.ascontiguousarray(np.concatenate(xs))).cuda())
        brep = bj.fetch_report(raise_dynamic=False)
        assert all(m == "dynamic" for m in brep["modes"]), brep["modes"]
        bj.finish_dynamic(brep)                                   # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for t in range(args.batch):
            bj.dynamic_track(t, brep["stats"][t])
        torch.cuda.synchronize()
        seq_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        bj.finish_dynamic(brep)
        torch.cuda.synchronize()
        par_s = time.perf_counter() - t0
        out["batch"] = {"tracks": args.batch, "one_after_another_s": round(seq_s, 4),
                        "side_by_side_s": round(par_s, 4), "speedup": round(seq_s / par_s, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
