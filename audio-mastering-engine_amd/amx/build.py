"""In-tree build of libamx.so with hipcc for gfx950 (no JIT cache, no pip install).

The .so lands in audio-mastering-engine_amd/lib/ so it travels with the repo
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).

Provenance: the SHA-256 of every source the library is compiled from
(source_hash) is stamped into it (-DAMX_SRC_HASH, read back by amx_build_id).
capi.load() recomputes the hash from the tree it runs in and refuses a library
built from other sources, so a GPU run always executes the committed kernels.
"""
import hashlib
import os
import subprocess

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "lib", "libamx.so")
HEADER = os.path.join(PKG, "..", "include", "amx.h")
SOURCES = ["amx_chain.hip", "amx_scan.hip", "amx_dyn.hip", "amx_loud.hip", "amx_loud192.hip", "amx_final.hip", "amx_io.hip",
           "amx_loudnorm.hip",
           "amx_plan.cpp", "amx_flac.cpp"]
HEADERS = ["amx_internal.hpp", "amx_dev.hpp"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-fvisibility=hidden", "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


def source_files():
    return [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [HEADER]


def source_hash():
    """SHA-256 over the compile inputs (names + contents, in a fixed order) and the flags."""
    h = hashlib.sha256()
    for p in source_files():
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()


def built_hash(path=OUT):
    """the stamp of an existing library (None: missing / unstamped), read from the file:
    loading it here would start a HIP runtime before torch's"""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        data = f.read()
    i = data.find(b"AMX_SRC_HASH=")
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + 13:j].decode(errors="replace")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    if any(os.path.getmtime(p) > t for p in source_files()):
        return True
    return built_hash() != source_hash()


def _obj_key(src):
    """cache key of one object: the source, the shared headers and the flags"""
    h = hashlib.sha256()
    for p in [src] + [os.path.join(CSRC, f) for f in HEADERS] + [HEADER]:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:24]


def build(force=False, verbose=False):
    """Compile every source to an object (in parallel, objects cached by content under
    build/amx_obj/), then link libamx.so.  Only amx_plan.cpp carries the stamp, so a
    change to one kernel file recompiles that file and the stamp's object."""
    if not force and not needs_build():
        return OUT
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    obj_dir = os.path.join(PKG, "..", "build", "amx_obj")
    os.makedirs(obj_dir, exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cflags = [f for f in FLAGS if f != "-shared"]
    stamp = source_hash()

    def compile_one(s):
        src = os.path.join(CSRC, s)
        extra = ['-DAMX_SRC_HASH="%s"' % stamp] if s == "amx_plan.cpp" else []
        key = _obj_key(src) + ("-" + stamp[:16] if extra else "")
        obj = os.path.join(obj_dir, "%s.%s.o" % (s, key))
        if force or not os.path.exists(obj):
            r = subprocess.run([hipcc] + cflags + extra + ["-c", src, "-o", obj + ".tmp"],
                               capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError("hipcc failed on %s:\n%s%s" % (s, r.stdout, r.stderr))
            if verbose and (r.stdout or r.stderr):
                print(r.stdout + r.stderr)
            os.replace(obj + ".tmp", obj)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1), 16))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    r = subprocess.run([hipcc] + FLAGS + objs + ["-o", OUT + ".tmp"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc link failed:\n" + r.stdout + r.stderr)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
