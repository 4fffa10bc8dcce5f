"""Build a measurement variant of libamx.so with extra -D flags into
audio-mastering-engine_amd/lib_var/libamx_<name>.so (selected at run time with
AMX_LIB=<path>; capi.load checks provenance only for the in-tree library).

    python scripts/build_var.py go2 -DAMX_GO_ILP=2
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "audio-mastering-engine_amd"))
from amx import build  # noqa: E402


def main():
    from concurrent.futures import ThreadPoolExecutor
    name, defs = sys.argv[1], sys.argv[2:]
    out = os.path.join(build.PKG, "lib_var", "libamx_%s.so" % name)
    odir = os.path.join(build.PKG, "..", "build", "var_%s" % name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    os.makedirs(odir, exist_ok=True)
    cflags = [f for f in build.FLAGS if f != "-shared"] + defs + ['-DAMX_SRC_HASH="variant-%s"' % name]

    def one(src):
        o = os.path.join(odir, src + ".o")
        r = subprocess.run(["/opt/rocm/bin/hipcc"] + cflags + ["-c", os.path.join(build.CSRC, src), "-o", o],
                           capture_output=True, text=True)
        if r.returncode:
            sys.exit("\n".join(l for l in (r.stdout + r.stderr).splitlines() if "error" in l))
        return o
    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, build.SOURCES))
    r = subprocess.run(["/opt/rocm/bin/hipcc"] + build.FLAGS + objs + ["-o", out], capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stdout + r.stderr)
    print(out)


if __name__ == "__main__":
    main()
