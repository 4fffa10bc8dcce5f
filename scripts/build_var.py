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
    name, defs = sys.argv[1], sys.argv[2:]
    out = os.path.join(build.PKG, "lib_var", "libamx_%s.so" % name)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = (["/opt/rocm/bin/hipcc"] + build.FLAGS + defs + ['-DAMX_SRC_HASH="variant-%s"' % name] +
           [os.path.join(build.CSRC, s) for s in build.SOURCES] + ["-o", out])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit("\n".join(l for l in (r.stdout + r.stderr).splitlines() if "error" in l))
    print(out)


if __name__ == "__main__":
    main()
