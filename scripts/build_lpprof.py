"""Measurement build of libamx with per-frame counters in k_lp_seg (device printf per
frame: detect calls, groups scanned, skip votes, serial steps, envelope calls / slots,
limiter mode before / after).  The counters are patched into a copy of the sources
(build/lpprof_src); the product sources are untouched.

    python scripts/build_lpprof.py    ->  audio-mastering-engine_amd/lib_var/libamx_lpprof.so
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "audio-mastering-engine_amd"))
from amx import build  # noqa: E402

PATCHES = [
    ("""    double d0, off;
};""", """    double d0, off;
    unsigned p_det, p_grp, p_vote, p_envc, p_env, p_ser;
};"""),
    ("""    const int lane = threadIdx.x;
    int slot0 = W.f.lbi + smp + LP_ATT;""", """    const int lane = threadIdx.x;
    W.p_det++;
    int slot0 = W.f.lbi + smp + LP_ATT;"""),
    ("""                lp_vote(W, may, mask);
                mask_base = nb00;""", """                lp_vote(W, may, mask);
                W.p_vote++;
                mask_base = nb00;"""),
    ("""        const int nb0 = nb00 + LP_NT * p;
        if (nb0 >= count) break;
        {""", """        const int nb0 = nb00 + LP_NT * p;
        if (nb0 >= count) break;
        W.p_grp++;
        {"""),
    ("""        for (int k = L0; k <= last; k++) {
            const int nn = nb0 + k;""", """        for (int k = L0; k <= last; k++) {
            W.p_ser++;
            const int nn = nb0 + k;"""),
    ("""__device__ __forceinline__ void lp_env(const LpArgs &a, LpWave &W, int e0, int k, F env) {
""", """__device__ __forceinline__ void lp_env(const LpArgs &a, LpWave &W, int e0, int k, F env) {
    W.p_envc++;
    W.p_env += k > 0 ? k : 0;
"""),
    ("""            for (int phi = w; phi < bk; phi++) {
                W.f = lp_frame(a, phi);
                lp_refill(a, W, phi);
                if (phi == ak) {
                    lp_snapshot(a, W, a.recG + (int64_t)k * LP_REC);
                    if (k > kh) lp_arrive(a, W, k);
                }
                lp_call(a, W, phi >= ak ? (a.bm ? 1 : 2) : 0);
            }""", """            for (int phi = w; phi < bk; phi++) {
                W.p_det = W.p_grp = W.p_vote = W.p_envc = W.p_env = W.p_ser = 0;
                const int mode0 = W.mode;
                W.f = lp_frame(a, phi);
                lp_refill(a, W, phi);
                if (phi == ak) {
                    lp_snapshot(a, W, a.recG + (int64_t)k * LP_REC);
                    if (k > kh) lp_arrive(a, W, k);
                }
                lp_call(a, W, phi >= ak ? (a.bm ? 1 : 2) : 0);
                if (threadIdx.x == 0)
                    printf("LPPROF k %d phi %d fin %d det %u grp %u vote %u ser %u envc %u env %u mode %d %d\\n", k, phi,
                           W.f.fin, W.p_det, W.p_grp, W.p_vote, W.p_ser, W.p_envc, W.p_env, mode0, W.mode);
            }"""),
]


def main():
    src_dir = os.path.join(build.PKG, "..", "build", "lpprof_src")
    shutil.rmtree(src_dir, ignore_errors=True)
    shutil.copytree(build.CSRC, src_dir)
    p = os.path.join(src_dir, "amx_loudnorm.hip")
    s = open(p).read()
    for old, new in PATCHES:
        assert s.count(old) == 1, old[:60]
        s = s.replace(old, new)
    open(p, "w").write(s)
    out = os.path.join(build.PKG, "lib_var", "libamx_lpprof.so")
    flags = [f for f in build.FLAGS if f != "-shared"] + ['-DAMX_SRC_HASH="variant-lpprof"']
    objs = []
    for src in build.SOURCES:
        o = os.path.join(src_dir, src + ".o")
        subprocess.check_call(["/opt/rocm/bin/hipcc"] + flags + ["-c", os.path.join(src_dir, src), "-o", o])
        objs.append(o)
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + build.FLAGS + objs + ["-o", out])
    print(out)


if __name__ == "__main__":
    main()
