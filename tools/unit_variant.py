"""A diagnostics library that differs from the in-tree build in ONE translation unit.

    python tools/unit_variant.py OUT.so UNIT.hip [DEFINE ...]

Compiles UNIT (e.g. fgx_ep_hp.hip) with the -D flags given and links it with the in-tree build's
objects of every other unit (fancy_gym_crowd_amd/csrc/build, made by _build.build()), so an A/B of
one kernel family costs one unit's compile instead of the whole library's.  Load the result with
FGX_LIB (its build id is not checked); never the in-tree library.
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from fancy_gym_crowd_amd import _build  # noqa: E402


def main():
    out, unit, defines = sys.argv[1], sys.argv[2], sys.argv[3:]
    for s in _build.SOURCES:   # the other units' objects must be those of the current sources
        o = os.path.join(_build.OBJDIR, os.path.splitext(s)[0] + ".o")
        if s != unit and s != "fgx_api.hip" and open(o + ".key").read().strip() != _build._unit_key(s, ""):
            sys.exit(f"{s}: stale object, run __graft_entry__.build() first")
    vdir = os.path.join(_build.OBJDIR, "unit_variant")
    os.makedirs(vdir, exist_ok=True)
    tag = "_".join(d.split("=")[0] for d in defines) or "plain"
    obj = os.path.join(vdir, os.path.splitext(unit)[0] + "." + tag + ".o")
    bid = _build.source_hash() + "+" + unit + ":" + ",".join(defines)
    defs = [f'-DFGX_BUILD_ID="{bid}"'] if unit == "fgx_api.hip" else []
    cmd = [_build._hipcc(), *_build.FLAGS, *_build.UNIT_FLAGS.get(unit, []), *[f"-D{d}" for d in defines], *defs,
           "-I", _build.INC, "-c", os.path.join(_build.CSRC, unit), "-o", obj]
    subprocess.run(cmd, check=True)
    objs = [obj if s == unit else os.path.join(_build.OBJDIR, os.path.splitext(s)[0] + ".o") for s in _build.SOURCES]
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    subprocess.run([_build._hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out], check=True)
    print(out)


if __name__ == "__main__":
    main()
