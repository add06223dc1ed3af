"""Builds the engine's shared library in-tree with hipcc for gfx950.

Output: roaringbitmap_amd/lib/libroaring_mi355x.so (git-ignored, travels with the
repo snapshot to the GPU box).  Objects are rebuilt only when a source is newer.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libroaring_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["kernels.hip", "pairwise.hip", "wide.hip", "pq.hip", "synth.hip", "bsi.hip", "runopt.hip", "ornot.hip", "rangemut.hip", "addoffset.hip", "decode.hip", "engine.cpp", "format.cpp"]
HEADERS = ["device.hpp", "kernels.hpp", "format.hpp", "wave.hpp", "vb.hpp"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-Wno-unused-result"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def build(verbose=False, jobs=8):
    os.makedirs(OBJDIR, exist_ok=True)
    inc = os.path.join(os.path.dirname(HERE), "include", "roaring_mi355x.h")
    dep_time = max([_mtime(os.path.join(CSRC, h)) for h in HEADERS] + [_mtime(inc), _mtime(__file__)])
    procs, objs = [], []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        op = os.path.join(OBJDIR, src + ".o")
        objs.append(op)
        if _mtime(op) >= max(_mtime(sp), dep_time):
            continue
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        cmd = [HIPCC] + FLAGS + lang + ["-c", sp, "-o", op]
        if verbose:
            print(" ".join(cmd))
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
        while len([p for _, p in procs if p.poll() is None]) >= jobs:
            procs[0][1].wait()
    failed = []
    for src, p in procs:
        out = p.communicate()[0].decode()
        if p.returncode != 0:
            failed.append((src, out))
        elif verbose and out.strip():
            print(out)
    if failed:
        msg = "\n".join(f"--- {s}\n{o}" for s, o in failed)
        raise RuntimeError(f"hipcc failed:\n{msg}")
    if _mtime(LIB) < max(_mtime(o) for o in objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs + ["-lpthread"]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
