"""Build libspe.so (gfx950 HIP kernels + C ABI), libshdtopo.so (C host shim) and
the C demo in-tree with hipcc / gcc.  Used by __graft_entry__.build(); the
CMake build (CMakeLists.txt) produces the same artefacts for a Shadow build."""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
HOST = os.path.join(HERE, "host")
LIB_SPE = os.path.join(HERE, "libspe.so")
LIB_TOPO = os.path.join(HERE, "libshdtopo.so")
DEMO = os.path.join(HERE, "shd_topology_demo")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_FLAGS = ["-O3", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "-fPIC",
             "-std=c++17", "-Wall", "-Wno-unused-function"]


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def build_spe(force: bool = False) -> str:
    srcs = [os.path.join(CSRC, f) for f in ("spe.hip", "spe_graph_prep.cpp", "spe_multi.cpp", "spe_internal.h")]
    srcs.append(os.path.join(ROOT, "include", "spe.h"))
    # spe.hip #includes its kernels and host code from csrc/spe/*.inc
    srcs += sorted(glob.glob(os.path.join(CSRC, "spe", "*.inc")))
    if force or _stale(LIB_SPE, srcs):
        _run([HIPCC, *HIP_FLAGS, "-shared", "-o", LIB_SPE,
              os.path.join(CSRC, "spe.hip"), os.path.join(CSRC, "spe_graph_prep.cpp"),
              os.path.join(CSRC, "spe_multi.cpp"), "-ldl", "-lpthread"])
    return LIB_SPE


def build_topo(force: bool = False) -> str:
    src = os.path.join(HOST, "shd_topology_spe.c")
    hdrs = [os.path.join(ROOT, "include", "shd_topology_spe.h"), os.path.join(ROOT, "include", "spe.h")]
    if not os.path.exists(src):
        return ""
    if force or _stale(LIB_TOPO, [src, LIB_SPE] + hdrs):
        _run(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-std=c11", "-D_GNU_SOURCE", "-Wall", "-shared",
              "-o", LIB_TOPO, src, "-I", os.path.join(ROOT, "include"), "-I", "/usr/include/libxml2",
              "-L", HERE, "-lspe", "-Wl,-rpath,$ORIGIN", "-lxml2", "-lpthread", "-lm"])
    return LIB_TOPO


SINGLE = os.path.join(HERE, "shd_topology_single_calls")


def build_demo(force: bool = False) -> str:
    """examples/shd_topology_demo.c: a Shadow-worker-shaped C user of libshdtopo;
    examples/shd_topology_single_calls.c: per-packet single calls timed in C (bench.py's shim lines)."""
    hdr = os.path.join(ROOT, "include", "shd_topology_spe.h")
    for src, out in ((os.path.join(ROOT, "examples", "shd_topology_demo.c"), DEMO),
                     (os.path.join(ROOT, "examples", "shd_topology_single_calls.c"), SINGLE)):
        if force or _stale(out, [src, LIB_TOPO, hdr]):
            _run(["gcc", "-O2", "-std=c11", "-D_GNU_SOURCE", "-Wall", "-o", out, src, "-I", os.path.join(ROOT, "include"),
                  "-L", HERE, "-lshdtopo", "-lspe", "-Wl,-rpath,$ORIGIN", "-lpthread"])
    return DEMO


LEXREPRO_SRC = os.path.join(ROOT, "tests", "native", "lexrepro.hip")
LEXREPRO = os.path.join(ROOT, "tests", "native", "liblexrepro.so")


def build_lexrepro(force: bool = False) -> str:
    """Test-only: the gfx950 compare reproducer tests/test_gpu_lexrepro.py runs
    (not part of the product; built beforehand so no GPU run compiles)."""
    if force or _stale(LEXREPRO, [LEXREPRO_SRC]):
        _run([HIPCC, *HIP_FLAGS, "-shared", "-o", LEXREPRO, LEXREPRO_SRC])
    return LEXREPRO


def build_all(force: bool = False) -> None:
    build_spe(force)
    build_topo(force)
    build_demo(force)
    build_lexrepro(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
