"""General-path alimiter (:223) timing on a 5-minute 48 kHz stereo track that the
limiter engages on (settings lufs None, no EQ, so the chain output reaches full
scale).  Times amx_finalize on the device-resident chain output for several
segment lengths, next to the idle-path pass over the same frames, and checks
the full-size output against the C oracle's sequential alimiter (checker only).

    python scripts/lim_bench.py [--seconds 300] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "audio-mastering-engine_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=300.0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--segs", default="4096,8192,16384,32768")
    ap.add_argument("--warm", type=int, default=-1)
    args = ap.parse_args()
    from amx import synth
    from amx.engine import MasteringJob
    from test_gpu_parity import _bursts
    import oracle
    fs = 48000
    n = int(fs * args.seconds)
    signals = {"music+3dBFS": synth.music_like(n, fs, 2, seed=7, peak_dbfs=3.0),
               "square-bursts": _bursts(n, fs, seed=11)}
    rows = []
    for name, x in signals.items():
        d_in = torch.from_numpy(x).cuda()
        for ls in [int(v) for v in args.segs.split(",")]:
            job = MasteringJob(fs, 2, dict(lufs=None), [n], quantum=512, limiter_seg_frames=ls,
                              limiter_warm_frames=args.warm)
            y = job.run(d_in)
            rep = job.fetch_report()
            assert rep["limiter_fast"] is False
            if not rows or rows[-1]["signal"] != name:
                out = job.out[:job.info.out_frames].cpu().numpy()
                t0 = time.perf_counter()
                ref = oracle.alimiter(out, fs)
                t_cpu = time.perf_counter() - t0
            got = y.cpu().numpy()
            exact = bool(np.array_equal(got, ref))
            ev = []
            for r in range(args.reps + 1):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                job.finalize(None)
                b.record()
                torch.cuda.synchronize()
                if r:
                    ev.append(a.elapsed_time(b))
            assert np.array_equal(job.y[:job.info.out_frames].cpu().numpy(), got)
            fe = []
            for r in range(args.reps + 1):
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                job.finalize(True)
                b.record()
                torch.cuda.synchronize()
                if r:
                    fe.append(a.elapsed_time(b))
            over = int((np.abs(job.out[:job.info.out_frames].cpu().numpy().astype(np.int32)).max(1)
                        > 0.98 * 32768).sum())
            row = {"signal": name, "frames": n, "over_limit_frames": over, "seg_frames": ls,
                   "general_ms": round(float(np.median(ev)), 3),
                   "idle_pass_ms": round(float(np.median(fe)), 4),
                   "cpu_oracle_ms": round(t_cpu * 1e3, 1), "bitexact_vs_oracle": exact}
            rows.append(row)
            print(json.dumps(row), flush=True)
            del job
    return 0 if all(r["bitexact_vs_oracle"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
