"""Diagnostics: the dynamic path's walker re-runs after eager steps and graph replays
(MasteringJob.capture(dynamic=True)), C3 settings on the bench's dynamic input."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from amx.dist import ShardedTrack
    fs, n = 48000, int(float(sys.argv[1]) * 48000) if len(sys.argv) > 1 else 48000 * 60
    tr = ShardedTrack(fs, 2, bench.CONFIGS["c3"], n, 0, 1, quantum=512, dynamic=True)
    d_in = torch.from_numpy(bench.synth_input(tr.local_frames, fs, 0, "dynamic")).cuda()
    y = tr.step(d_in)
    torch.cuda.synchronize()
    print("eager", tr.dyn_info.get("pass2_parallel"), flush=True)
    ref = y.cpu().numpy()
    tr.capture(d_in)
    for k in range(4):
        t0 = time.perf_counter()
        y = tr.replay()
        torch.cuda.synchronize()
        same = bool((y.cpu().numpy() == ref).all())
        print("replay", k, round((time.perf_counter() - t0) * 1e3, 2), "ms", tr.dyn_info.get("pass2_parallel"),
              "same as eager", same, flush=True)


if __name__ == "__main__":
    main()
