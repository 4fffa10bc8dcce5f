"""Probe (measurement only): the C3 chain (bench.py's captured-graph step, one GPU) on a
5-minute stereo track at several sample rates -- 44.1 kHz runs the M > 1 192 kHz
resampler (k_up_slow), 48 / 96 kHz the unrolled one (k_up<4> / k_up<2>).

    python scripts/rate_probe.py [--rates 44100,48000,96000] [--seconds 300]
"""
import argparse
import gc
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="44100,48000,96000")
    ap.add_argument("--seconds", type=float, default=300.0)
    ap.add_argument("--config", default="c3")
    a = ap.parse_args()
    import torch
    import bench
    from amx.dist import ShardedTrack
    for fs in (int(r) for r in a.rates.split(",")):
        n = int(a.seconds * fs)
        runner = ShardedTrack(fs, 2, bench.CONFIGS[a.config], n, 0, 1, quantum=512, seg_frames=128)
        d_in = torch.from_numpy(bench.synth_input(runner.local_frames, fs, 0)).cuda()
        ms, steps = bench.time_graph(runner, d_in, 2, 0.5, 1.0)
        rep = runner.job.fetch_report()
        print(json.dumps({"fs": fs, "seconds": a.seconds, "ms_per_step": round(ms, 4), "steps": steps,
                          "Msamples_per_s": round(2 * n / ms / 1e3, 1),
                          "loudnorm_mode": rep.get("modes")}), flush=True)
        del runner, d_in
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
