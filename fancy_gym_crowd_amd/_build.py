"""Build libfgx.so (HIP, gfx950) in-tree with hipcc.  Used by __graft_entry__.build().

Translation units are compiled in parallel (the episode kernels of each env kind live in their
own TU) and linked into one shared library.

Build provenance: the library carries ``fgx_build_id()``, a hash of the sources it was compiled
from (csrc/*.h, csrc/*.hip, include/fgx.h and the compiler flags).  ``build()`` recompiles
whenever that hash differs from the one recorded for the existing library, and ``_lib.load()``
refuses a library whose id does not match the sources next to it.
"""
import concurrent.futures as cf
import glob
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INC = os.path.join(HERE, "..", "include")
LIB = os.path.join(HERE, "libfgx.so")
STAMP = LIB + ".buildid"
OBJDIR = os.path.join(HERE, "csrc", "build")
# (the longest units first: the pool starts them before the short ones)
SOURCES = ["fgx_ep_hole_gen.hip", "fgx_ep_hole.hip", "fgx_ep_simple_gen.hip", "fgx_ep_simple.hip",
           "fgx_ep_via_gen.hip", "fgx_ep_via.hip", "fgx_ep_jl.hip", "fgx_ep_hp.hip"] + \
          [f"fgx_ep_nl{n}.hip" for n in (1, 3, 4, 6, 7, 8)] + ["fgx_api.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         # numerics: every expression rounds like the numpy reference; fmas only where written
         "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "-Wno-unused-result"]


def source_files():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.hip"))) + \
        [os.path.join(INC, "fgx.h")]


def source_hash():
    """16 hex digits of sha256 over the source files (name + bytes) and the compiler flags."""
    h = hashlib.sha256(" ".join(FLAGS + sorted(sum(UNIT_FLAGS.values(), []))).encode())
    for f in source_files():
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def built_id():
    """Build id recorded for the existing library (None if missing)."""
    if not (os.path.exists(LIB) and os.path.exists(STAMP)):
        return None
    with open(STAMP) as f:
        return f.read().strip()


def _hipcc():
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


# per-unit extra flags: k_episode_jl's one-joint lanes gain nothing from SLP-pairing consecutive
# samples (the table entries of two rows need SGPR shuffles first): plain f32 fmas.  Its epilogue
# calls ocml's sincos (FGX_OCML_SINCOS, csrc/fgx_trig.h; bit-identical to the inlined restatement):
# 1-2% faster for jl (profiles/r03_ab_s4.jsonl), where the inlined form's registers cost more than
# the large-argument path it skips.  Device code is not linked across units, so each unit keeps its own.
UNIT_FLAGS = {"fgx_ep_jl.hip": ["-fno-slp-vectorize", "-DFGX_OCML_SINCOS"]}


def _deps(path, seen=None):
    """path and the local headers it includes, transitively (#include "..." under csrc / include)."""
    seen = set() if seen is None else seen
    if path in seen:
        return seen
    seen.add(path)
    with open(path) as f:
        for line in f:
            m = re.match(r'\s*#\s*include\s+"([^"]+)"', line)
            if m:
                for d in (os.path.dirname(path), CSRC, INC):
                    cand = os.path.normpath(os.path.join(d, m.group(1)))
                    if os.path.exists(cand):
                        _deps(cand, seen)
                        break
    return seen


_TOOLCHAIN = None


def toolchain_id():
    """`hipcc --version` (compiler and ROCm release): part of every object's cache key, so a
    toolchain change recompiles."""
    global _TOOLCHAIN
    if _TOOLCHAIN is None:
        try:
            _TOOLCHAIN = subprocess.run([_hipcc(), "--version"], capture_output=True, text=True).stdout
        except OSError:
            _TOOLCHAIN = "unknown"
    return _TOOLCHAIN


def _unit_key(src, bid):
    """Object cache key of one translation unit: toolchain, flags, its include closure and
    (fgx_api.hip only, the unit that embeds it) the library build id."""
    h = hashlib.sha256(toolchain_id().encode() + b"\0" + " ".join(FLAGS + UNIT_FLAGS.get(src, [])).encode())
    if src == "fgx_api.hip":
        h.update(bid.encode())
    for f in sorted(_deps(os.path.join(CSRC, src))):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _compile(src, bid, verbose, force=False):
    obj = os.path.join(OBJDIR, os.path.splitext(src)[0] + ".o")
    key = _unit_key(src, bid)
    if not force and os.path.exists(obj) and os.path.exists(obj + ".key") and open(obj + ".key").read().strip() == key:
        return obj   # unchanged unit: reuse its object
    defs = [f'-DFGX_BUILD_ID="{bid}"'] if src == "fgx_api.hip" else []
    cmd = [_hipcc(), *FLAGS, *UNIT_FLAGS.get(src, []), *defs, "-I", INC, "-c", os.path.join(CSRC, src), "-o",
           obj + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)
    with open(obj + ".key", "w") as f:
        f.write(key)
    return obj


def build_variant(out, defines=(), verbose=False):
    """A diagnostics build of the same sources with extra -D flags (e.g. FGX_STAMPS) into `out`
    (loaded with FGX_LIB; its build id is not checked).  Never the in-tree library."""
    objdir = os.path.join(OBJDIR, "variant_" + "_".join(d.split("=")[0] for d in defines))
    os.makedirs(objdir, exist_ok=True)
    bid = source_hash() + "+" + ",".join(defines)

    def one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        key = _unit_key(src, bid) + ",".join(defines)
        if os.path.exists(obj) and os.path.exists(obj + ".key") and open(obj + ".key").read().strip() == key:
            return obj
        cmd = [_hipcc(), *FLAGS, *UNIT_FLAGS.get(src, []), *[f"-D{d}" for d in defines], f'-DFGX_BUILD_ID="{bid}"',
               "-I", INC, "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        with open(obj + ".key", "w") as f:
            f.write(key)
        return obj
    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 8)) as ex:
        objs = list(ex.map(one, SOURCES))
    subprocess.run([_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out], check=True)
    return out


def build(force=False, verbose=True):
    bid = source_hash()
    if not force and built_id() == bid:
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, bid, verbose, force), SOURCES))   # force: no cached objects
    cmd = [_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    with open(STAMP, "w") as f:
        f.write(bid + "\n")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
