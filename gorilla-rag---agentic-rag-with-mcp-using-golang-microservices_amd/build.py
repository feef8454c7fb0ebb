"""Builds lib/libvsearch.so in-tree with hipcc for gfx950.

The .so is git-ignored but travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "lib", "libvsearch.so")
SVC_LIB = os.path.join(HERE, "lib", "libvsearch_service.so")
SVC_SOURCES = ["service/json.cpp", "service/vector_service.cpp", "service/batcher.cpp",
               "service/loadgen.cpp", "service/http.cpp"]
SVC_HEADERS = ["service/json.h", "service/batcher.h", "service/http.h"]
# the vector-service process (PORT, VS_DEVICES, ...; csrc/service/server_main.cpp)
SERVER = os.path.join(HERE, "lib", "vsearch_server")
ROOT = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("VS_OFFLOAD_ARCH", "gfx950")

SOURCES = {
    "vs_kernels.o": (["vs_kernels.hip"], ["--offload-arch=" + ARCH, "-O3"]),
    "vs_engine.o": (["vs_engine.cpp"], ["-O2", "-Wall"]),
    "vs_api.o": (["vs_api.cpp"], ["-O2", "-Wall"]),
}
HEADERS = ["vs_common.h", "vs_kernels.h", "vs_dev.h"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else -1.0


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    hdr_t = max([_mtime(os.path.join(CSRC, h)) for h in HEADERS] +
                [_mtime(os.path.join(ROOT, "include", "vsearch.h"))])
    objs = []
    for obj, (srcs, flags) in SOURCES.items():
        out = os.path.join(BUILD, obj)
        src = os.path.join(CSRC, srcs[0])
        objs.append(out)
        if not force and _mtime(out) > max(_mtime(src), hdr_t):
            continue
        cmd = [HIPCC, "-std=c++17", "-fPIC", *flags, "-c", src, "-o", out]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    if force or _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB, *objs,
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib",
               "-Wl,-soname,libvsearch.so"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    # host-only service layer (the rag/vector-service handler mirror) over the C-ABI
    svc_srcs = [os.path.join(CSRC, x) for x in SVC_SOURCES]
    svc_hdrs = [os.path.join(CSRC, x) for x in SVC_HEADERS] + [
        os.path.join(ROOT, "include", "vsearch_service.h")]
    if force or _mtime(SVC_LIB) < max(_mtime(x) for x in svc_srcs + svc_hdrs + [LIB]):
        cmd = [os.environ.get("CXX", "g++"), "-std=c++17", "-O2", "-fPIC", "-Wall", "-shared",
               "-o", SVC_LIB, *svc_srcs, "-L" + os.path.dirname(LIB), "-lvsearch",
               "-pthread", "-Wl,-rpath,$ORIGIN", "-Wl,-soname,libvsearch_service.so"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    main_src = os.path.join(CSRC, "service", "server_main.cpp")
    if force or _mtime(SERVER) < max(_mtime(main_src), _mtime(SVC_LIB)):
        cmd = [os.environ.get("CXX", "g++"), "-std=c++17", "-O2", "-Wall", "-o", SERVER, main_src,
               "-L" + os.path.dirname(LIB), "-lvsearch_service", "-lvsearch", "-pthread",
               "-Wl,-rpath,$ORIGIN"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
