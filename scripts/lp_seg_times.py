"""Per-segment times of k_lp_seg (measurement build libamx_lptime: each segment's
workgroup writes s_memrealtime (100 MHz) at its start and end into its record's free
slots 8 / 9), on the C3 dynamic-mode bench input.  Prints the slowest segments and the
distribution; the record layout follows amx_plan.cpp ln_layout (scripts/dyn_graph_probe.py)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

from bench import CONFIGS, synth_input  # noqa: E402
from amx.engine import MasteringJob  # noqa: E402
from dyn_graph_probe import layout, REC  # noqa: E402


def main():
    fs = 48000
    n = 300 * fs
    x = synth_input(n, fs, 0, "dynamic")
    job = MasteringJob(fs, 2, CONFIGS["c3"], [n], quantum=512)
    d_in = torch.from_numpy(x).cuda()
    job.capture(d_in, dynamic=True)
    for _ in range(3):
        job.replay()
    torch.cuda.synchronize()
    n192, job2, ws2, summ = job._dyn_sides[0]
    geo, regs = layout(n192)
    off = dict((r[0], r[1]) for r in regs)
    w = ws2.cpu().numpy()
    rec = w[off["recG"]:off["recG"] + geo["K"] * REC * 8].view(np.float64).reshape(geo["K"], REC)
    t0, t1 = rec[:, 8], rec[:, 9]
    ok = (t1 > t0) & (t0 > 0)
    dt = (t1 - t0)[ok] * 10e-3                       # 100 MHz ticks -> us
    ks = np.nonzero(ok)[0]
    base = t0[ok].min()
    print("segments %d (K %d, Fs %d), kernel span %.1f us" % (ok.sum(), geo["K"], geo["Fs"], (t1[ok].max() - base) * 10e-3))
    print("segment time us: median %.1f p90 %.1f p99 %.1f max %.1f" % tuple(np.percentile(dt, [50, 90, 99, 100])))
    t2, t3, t4 = rec[:, 10][ok], rec[:, 11][ok], rec[:, 12][ok]
    warm = (t2 - t0[ok]) * 10e-3
    snap = (t3 - t2) * 10e-3
    body = (t4 - t3) * 10e-3
    tail = (t1[ok] - t4) * 10e-3
    for name, v in (("warm-up frames", warm), ("snapshot + arrive at the start", snap),
                    ("the segment's frames", body), ("end: refill, snapshot, arrive", tail)):
        print("  %-32s median %6.1f p90 %6.1f max %6.1f us" % ((name,) + tuple(np.percentile(v, [50, 90, 100]))))
    order = np.argsort(-dt)[:15]
    for i in order:
        print("  k %4d  start %7.1f  dt %7.1f us  warm %6.1f snap %6.1f body %6.1f tail %6.1f" % (
            ks[i], (t0[ok][i] - base) * 10e-3, dt[i], warm[i], snap[i], body[i], tail[i]))


if __name__ == "__main__":
    main()
