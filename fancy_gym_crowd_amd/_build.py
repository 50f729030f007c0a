"""Build libfgx.so (HIP, gfx950) in-tree with hipcc.  Used by __graft_entry__.build().

Translation units are compiled in parallel (the episode kernels of each env kind live in their
own TU) and linked into one shared library.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INC = os.path.join(HERE, "..", "include")
LIB = os.path.join(HERE, "libfgx.so")
OBJDIR = os.path.join(HERE, "csrc", "build")
SOURCES = ["fgx_ep_simple_gen.hip", "fgx_ep_hole_gen.hip", "fgx_ep_via_gen.hip", "fgx_ep_simple.hip",
           "fgx_ep_hole.hip", "fgx_ep_via.hip", "fgx_api.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         # numerics: every expression rounds like the numpy reference; fmas only where written
         "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-Wno-unused-result"]


def _deps():
    return (glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.hip")) +
            [os.path.join(INC, "fgx.h"), os.path.abspath(__file__)])


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _hipcc():
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _compile(src, verbose):
    obj = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
    if not _stale(obj, _deps()):
        return obj
    cmd = [_hipcc(), *FLAGS, "-I", INC, "-c", os.path.join(CSRC, src), "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)
    return obj


def build(force=False, verbose=True):
    if not force and not _stale(LIB, _deps()):
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    if force:
        for f in glob.glob(os.path.join(OBJDIR, "*.o")):
            os.remove(f)
    with cf.ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), SOURCES))
    cmd = [_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
