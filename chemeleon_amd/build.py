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


# The torch-op layer (csrc/torch_ops.cpp: TORCH_LIBRARY(chemeleon) over the C ABI), built against this
# torch's headers and libraries next to libchemeleon_hip.so (which it links, rpath $ORIGIN).
OPS_SRC = os.path.join(CSRC, "torch_ops.cpp")
OPS_LIB = os.path.join(os.path.dirname(LIB), "libchemeleon_torch_ops.so")


def build_torch_ops(force: bool = False, verbose: bool = True) -> str:
    if not force and os.path.exists(OPS_LIB) and os.path.getmtime(OPS_LIB) >= max(
            os.path.getmtime(OPS_SRC), os.path.getmtime(LIB)):
        return OPS_LIB
    import torch
    import torch.utils.cpp_extension as ce
    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    tmp = OPS_LIB + ".tmp"
    cmd = ([hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
            f"-D_GLIBCXX_USE_CXX11_ABI={abi}"] + [f"-I{p}" for p in ce.include_paths()] +
           [OPS_SRC, "-o", tmp, f"-L{tlib}", "-ltorch", "-ltorch_cpu", "-lc10", "-lc10_hip", "-ltorch_hip",
            f"-L{os.path.dirname(LIB)}", "-lchemeleon_hip", "-Wl,-rpath,$ORIGIN"])
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, OPS_LIB)
    return OPS_LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_torch_ops(force="--force" in sys.argv)
