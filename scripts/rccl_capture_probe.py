"""Probe: can RCCL collectives (torch.distributed nccl backend) be captured into a
hipGraph (torch.cuda.CUDAGraph) on this image?  World 1 (one GPU), and the time per
replay of a graph holding the N > 1 step's exchange pattern against the same
collectives launched eagerly.

    python scripts/rccl_capture_probe.py
"""
import os
import time

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    dev = torch.device("cuda")
    a = torch.randn(1 << 20, device=dev)
    e = torch.zeros(1000, dtype=torch.float64, device=dev)
    eall = torch.zeros(1000, dtype=torch.float64, device=dev)
    h = torch.ones(30000, dtype=torch.float64, device=dev)
    x = torch.zeros(12, dtype=torch.float64, device=dev)
    xall = torch.zeros(12, dtype=torch.float64, device=dev)

    def body():
        a.mul_(1.0000001)
        dist.all_gather_into_tensor(eall, e)
        a.add_(1e-9)
        dist.all_gather_into_tensor(xall, x)
        a.mul_(0.9999999)
        dist.all_reduce(h)
        h.mul_(0.5)

    for _ in range(3):
        body()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        body()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / 200 * 1e6
    print("eager us/step", round(eager, 1), flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            body()
    except Exception as ex:  # noqa
        print("CAPTURE FAILED:", type(ex).__name__, str(ex)[:500], flush=True)
        dist.destroy_process_group()
        return
    print("captured", flush=True)
    h.fill_(2.0)
    g.replay()
    torch.cuda.synchronize()
    print("after replay h[0] =", float(h[0]), "(expect 1.0 at world 1)", flush=True)
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
    torch.cuda.synchronize()
    print("graph us/step", round((time.perf_counter() - t0) / 200 * 1e6, 1), flush=True)
    # the host read pattern of ShardedTrack.replay
    hc = torch.zeros(1, dtype=torch.int32).pin_memory()
    ev = torch.cuda.Event()
    w = torch.zeros(1, dtype=torch.int32, device=dev)
    t0 = time.perf_counter()
    for _ in range(200):
        g.replay()
        hc.copy_(w, non_blocking=True)
        ev.record()
        ev.synchronize()
    print("graph + host read us/step", round((time.perf_counter() - t0) / 200 * 1e6, 1), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
