"""Build ``librecoup_amd.so`` in-tree with hipcc for gfx950 (no JIT cache, no pip install).

    python -m recoup_amd.build [--force]
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "librecoup_amd.so")
ARCH = os.environ.get("RCP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
            "-fvisibility=hidden"]
SOURCES = ["rcp_kernels.hip", "rcp_rle.hip", "rcp_shard.hip", "rcp_host.cpp", "rcp_shard.cpp", "rcp_stage.cpp", "rcp_bam.cpp"]
DEPS = ["rcp_internal.h", "rcp_device.h", "rcp_divrn.h", "rcp_rng.h", "rcp_stage.h", "rcp_pack.h", "rcp_splitvector.h", "rcp_rle.h", os.path.join("..", "..", "include", "recoup_amd.h")]


def _newer(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build(force=False, verbose=True):
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    deps = [os.path.join(CSRC, d) for d in DEPS]
    objs = []
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(objdir, src + ".o")
        objs.append(o)
        if force or _newer(o, [s] + deps):
            cmd = [HIPCC] + CXXFLAGS + ["-c", s, "-o", o]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.check_call(cmd)
    if force or _newer(OUT, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fvisibility=hidden", "-o", OUT] + objs + ["-lz",
                                                                                                   "-pthread"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
