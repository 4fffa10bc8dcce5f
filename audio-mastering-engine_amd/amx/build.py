"""In-tree build of libamx.so with hipcc for gfx950 (no JIT cache, no pip install).

The .so lands in audio-mastering-engine_amd/lib/ so it travels with the repo
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
import os
import subprocess

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "lib", "libamx.so")
SOURCES = ["amx_chain.hip", "amx_scan.hip", "amx_dyn.hip", "amx_loud.hip", "amx_loud192.hip", "amx_final.hip", "amx_io.hip",
           "amx_loudnorm.hip",
           "amx_plan.cpp"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-fvisibility=hidden", "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = SOURCES + ["amx_internal.hpp", "amx_dev.hpp"]
    hdr = os.path.join(PKG, "..", "include", "amx.h")
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in deps) or os.path.getmtime(hdr) > t


def build(force=False, verbose=False):
    if not force and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc] + FLAGS + [os.path.join(CSRC, s) for s in SOURCES] + ["-o", OUT + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed:\n" + r.stdout + r.stderr)
    if verbose and (r.stdout or r.stderr):
        print(r.stdout + r.stderr)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
