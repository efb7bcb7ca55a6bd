"""Build the in-tree HIP library `chemeleon_amd/lib/libchemeleon_hip.so` for gfx950.

    python -m chemeleon_amd.build          # or: python chemeleon_amd/build.py

hipcc cross-compiles without a GPU, so this runs in the CPU container too.
The .so stays in-tree (git-ignored, shipped to the GPU box with the snapshot).
"""

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libchemeleon_hip.so")
# (A/B builds only: extra -D flags and another output path, e.g. CHM_BUILD_DEFS="-DCHM_X=1"
# CHM_BUILD_LIB=abl/x/libchemeleon_hip.so, loaded with CHM_LIB; the product build sets neither)
DEFS = os.environ.get("CHM_BUILD_DEFS", "").split()
if os.environ.get("CHM_BUILD_LIB"):
    LIB = os.path.abspath(os.environ["CHM_BUILD_LIB"])
    LIBDIR = os.path.dirname(LIB)
SOURCES = ["kernels.hip", "gemm_bf16x3.hip", "split16.hip", "edge16.hip", "node_gemm.hip", "knn.hip", "runtime.hip", "host_noise.cpp"]
ARCH = os.environ.get("CHM_OFFLOAD_ARCH", "gfx950")


def hipcc():
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), "hipcc"):
        if os.path.isfile(c) or c == "hipcc":
            return c


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "chemeleon_hip.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    from concurrent.futures import ThreadPoolExecutor

    def compile_one(src):
        obj = os.path.join(LIBDIR, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", os.path.join(CSRC, src),
               "-o", obj, "-Wno-unused-result"] + DEFS
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "4"))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
