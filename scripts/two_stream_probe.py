"""Probe (measurement only): does running the chunk chain as two halves on two streams
overlap the latency-bound kernels of one half with the other's compute?  C3 settings,
one 5-min track; three captured graphs: the whole chain, half A (first chunks), half B.
Times: whole, A then B on one stream, A and B on two streams.

    python scripts/two_stream_probe.py [--reps 200]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--seconds", type=float, default=300.0)
    ap.add_argument("--config", default="c3")
    a = ap.parse_args()
    import torch
    import bench
    from amx import synth
    from amx.chunking import chunk_bounds, packet_frames
    from amx.engine import MasteringJob
    fs = bench.CONFIG_FS[a.config]
    settings = bench.CONFIGS[a.config]
    n = int(fs * a.seconds)
    x = torch.from_numpy(synth.mix_like(n, fs, 2, seed=1)).cuda().contiguous()
    bounds = chunk_bounds(n, fs, packet_frames(8))
    half = len(bounds) // 2
    ch_all = [(0, s, ln) for s, ln in bounds]
    jobs = {"all": MasteringJob(fs, 2, settings, [n], chunks=ch_all),
            "A": MasteringJob(fs, 2, settings, [sum(ln for _, ln in bounds[:half])], chunks=ch_all[:half]),
            "B": MasteringJob(fs, 2, settings, [n], chunks=ch_all[half:])}
    s0, s1, s2 = torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()
    graphs = {}
    for k, j in jobs.items():
        j.run_chunks(x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            j.run_chunks(x)
        graphs[k] = g
    torch.cuda.synchronize()

    def timeit(fn):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s0)
        for _ in range(a.reps):
            fn()
        e1.record(s0)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    def whole():
        graphs["all"].replay()

    def serial():
        graphs["A"].replay()
        graphs["B"].replay()

    def overlap():
        ev = torch.cuda.Event()
        ev.record(s0)
        s1.wait_event(ev)
        s2.wait_event(ev)
        with torch.cuda.stream(s1):
            graphs["A"].replay()
        with torch.cuda.stream(s2):
            graphs["B"].replay()
        e1, e2 = torch.cuda.Event(), torch.cuda.Event()
        e1.record(s1)
        e2.record(s2)
        s0.wait_event(e1)
        s0.wait_event(e2)

    print("chain %s, %d chunks (A %d, B %d): whole %.4f ms, A then B %.4f ms, A || B %.4f ms"
          % (a.config, len(bounds), half, len(bounds) - half, timeit(whole), timeit(serial), timeit(overlap)))


if __name__ == "__main__":
    main()
