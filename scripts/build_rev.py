"""Build libamx from the sources of a git revision into lib_var/libamx_<name>.so (A/B
measurements against an earlier tree on the same GPU box; AMX_LIB selects it).

    python scripts/build_rev.py HEAD base
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.join(HERE, "..")
sys.path.insert(0, os.path.join(ROOT, "audio-mastering-engine_amd"))
from amx import build  # noqa: E402


def main():
    rev, name = sys.argv[1], sys.argv[2]
    src_dir = os.path.join(ROOT, "build", "rev_%s" % name)
    shutil.rmtree(src_dir, ignore_errors=True)
    os.makedirs(src_dir)
    rel = os.path.relpath(build.CSRC, ROOT)
    files = subprocess.check_output(["git", "-C", ROOT, "ls-tree", "--name-only", rev, rel + "/"], text=True).split()
    for f in files:
        data = subprocess.check_output(["git", "-C", ROOT, "show", "%s:%s" % (rev, f)])
        with open(os.path.join(src_dir, os.path.basename(f)), "wb") as fh:
            fh.write(data)
    out = os.path.join(build.PKG, "lib_var", "libamx_%s.so" % name)
    flags = [f for f in build.FLAGS if f != "-shared"] + ['-DAMX_SRC_HASH="variant-%s"' % name]
    objs = []
    for src in build.SOURCES:
        o = os.path.join(src_dir, src + ".o")
        subprocess.check_call(["/opt/rocm/bin/hipcc"] + flags + ["-c", os.path.join(src_dir, src), "-o", o])
        objs.append(o)
    subprocess.check_call(["/opt/rocm/bin/hipcc"] + build.FLAGS + objs + ["-o", out])
    print(out)


if __name__ == "__main__":
    main()
