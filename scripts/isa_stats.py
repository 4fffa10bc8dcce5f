"""Per-kernel resource usage and instruction mix of a libamx translation unit.

    python scripts/isa_stats.py amx_chain.hip [kernel-substring ...]

Compiles the .hip for gfx950 to assembly (device only) and prints, per kernel,
VGPRs / SGPR spills / LDS bytes from the .s metadata and the most frequent
opcodes, so register-pressure regressions are visible without a GPU.
"""
import collections
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "audio-mastering-engine_amd", "csrc")


def main():
    src = sys.argv[1]
    want = sys.argv[2:]
    out = "/tmp/_isa_%s.s" % os.path.basename(src)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                           "-ffp-contract=off", "--cuda-device-only", "-S", os.path.join(CSRC, src),
                           "-o", out])
    s = open(out).read()
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n", s, re.M):
        name = m.group(1)
        if want and not any(w in name for w in want):
            continue
        end = s.index(".Lfunc_end", m.end())
        body = s[m.end():end]
        meta = s[end:end + 4000]
        ops = collections.Counter()
        for line in body.split("\n"):
            line = line.strip()
            if not line or line.startswith((".", ";")) or line.endswith(":"):
                continue
            ops[line.split()[0]] += 1
        vg = re.search(r"; NumVgprs: (\d+)", meta)
        sp = re.search(r"; ScratchSize: (\d+)", meta)
        occ = re.search(r"; Occupancy: (\d+)", meta)
        print("%s\n  vgpr=%s scratch=%s occ=%s insts=%d" % (
            name[:90], vg and vg.group(1), sp and sp.group(1), occ and occ.group(1), sum(ops.values())))
        print("  " + ", ".join("%s:%d" % kv for kv in ops.most_common(14)))


if __name__ == "__main__":
    main()
