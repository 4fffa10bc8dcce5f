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
    tf = rec[:, 10:16][ok]
    order = np.argsort(-dt)[:15]
    for i in order:
        prev = t0[ok][i]
        fr = []
        for q in range(6):
            if tf[i, q] > 0:
                fr.append((tf[i, q] - prev) * 10e-3)
                prev = tf[i, q]
        print("  k %4d  dt %7.1f us  frames (warm-up 2, then the segment's):" % (ks[i], dt[i]),
              " ".join("%6.1f" % v for v in fr), " tail %6.1f" % ((t1[ok][i] - prev) * 10e-3))


if __name__ == "__main__":
    main()
