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


def build(force=False, verbose=False):
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = ([hipcc] + FLAGS + ['-DAMX_SRC_HASH="%s"' % source_hash()] +
           [os.path.join(CSRC, s) for s in SOURCES] + ["-o", OUT + ".tmp"])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + r.stdout + r.stderr)
    if verbose and (r.stdout or r.stderr):
        print(r.stdout + r.stderr)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
