"""Measurement build with per-segment timestamps in k_lp_seg (scripts/lp_seg_times.py):
a patched copy of the sources (build/lptime_src) -> lib_var/libamx_lptime.so."""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "audio-mastering-engine_amd"))
from amx import build  # noqa: E402

OLD = """        if (k < kh) continue;
        const int ak = lp_seg_start(a, k), bk = k + 1 < a.K ? lp_seg_start(a, k + 1) : NF;"""
NEW = """        if (k < kh) continue;
        const uint64_t tq0 = __builtin_amdgcn_s_memrealtime();
        uint64_t tf[7] = {0, 0, 0, 0, 0, 0, 0};
        const int ak = lp_seg_start(a, k), bk = k + 1 < a.K ? lp_seg_start(a, k + 1) : NF;"""
OLD3 = """                if (phi == ak) {
                    lp_snapshot(a, W, a.recG + (int64_t)k * LP_REC);
                    if (k > kh) lp_arrive(a, W, k);
                }
                lp_call(a, W, phi >= ak ? (a.bm ? 1 : 2) : 0);
            }"""
NEW3 = """                if (phi == ak) {
                    lp_snapshot(a, W, a.recG + (int64_t)k * LP_REC);
                    if (k > kh) lp_arrive(a, W, k);
                }
                lp_call(a, W, phi >= ak ? (a.bm ? 1 : 2) : 0);
                __syncthreads();
                if (phi - w < 7) tf[phi - w] = __builtin_amdgcn_s_memrealtime();
            }"""
OLD2 = """            lp_snapshot(a, W, a.recE + (int64_t)k * LP_REC);
            lp_arrive(a, W, k + 1);
        }
    }
}"""
NEW2 = """            lp_snapshot(a, W, a.recE + (int64_t)k * LP_REC);
            lp_arrive(a, W, k + 1);
        }
        __syncthreads();
        const uint64_t tq1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            a.recG[(int64_t)k * LP_REC + 8] = (double)tq0;
            a.recG[(int64_t)k * LP_REC + 9] = (double)tq1;
            for (int q = 0; q < 6; q++) a.recG[(int64_t)k * LP_REC + 10 + q] = (double)tf[q];
        }
    }
}"""


def main():
    src_dir = os.path.join(build.PKG, "..", "build", "lptime_src")
    shutil.rmtree(src_dir, ignore_errors=True)
    shutil.copytree(build.CSRC, src_dir)
    p = os.path.join(src_dir, "amx_loudnorm.hip")
    s = open(p).read()
    for o, nw in ((OLD, NEW), (OLD3, NEW3), (OLD2, NEW2)):
        assert s.count(o) == 1, o[:60]
        s = s.replace(o, nw)
    open(p, "w").write(s)
    out = os.path.join(build.PKG, "lib_var", "libamx_lptime.so")
    flags = [f for f in build.FLAGS if f != "-shared"] + ['-DAMX_SRC_HASH="variant-lptime"']
    objs = []
    for src in build.SOURCES:
        o = os.path.join(src_dir, src + ".o")
        subprocess.check_call(["/opt/rocm/bin/hipcc"] + flags + ["-c", os.path.join(src_dir, src), "-o", o])
        objs.append(o)
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + build.FLAGS + objs + ["-o", out])
    print(out)


if __name__ == "__main__":
    main()
