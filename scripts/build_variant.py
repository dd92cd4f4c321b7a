#!/usr/bin/env python3
"""A/B builds: the library with extra compile flags, linked as lib/libhgnn_<name>.so (load it
with HGNN_LIB=libhgnn_<name>.so).  Objects of sources the flags do not touch are shared with the
default build's.

  python scripts/build_variant.py NAME -DHGNN_FOO=1 [...] [--only linear_xs]"""
import json
import os
import pathlib
import subprocess
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
from truth_recommendation_gnn_amd import build as B  # noqa: E402


def main():
    name, rest = sys.argv[1], sys.argv[2:]
    only = None
    if "--only" in rest:
        i = rest.index("--only")
        only = set(rest[i + 1].split(","))
        rest = rest[:i] + rest[i + 2:]
    B.build(verbose=False)
    objdir = B.PKG.parent / "build" / "obj"
    vdir = B.PKG.parent / "build" / f"obj_{name}"
    vdir.mkdir(parents=True, exist_ok=True)
    objs = []
    for src in B._sources():
        if only is not None and src.stem not in only:
            objs.append(objdir / (src.stem + ".o"))
            continue
        obj = vdir / (src.stem + ".o")
        r = subprocess.run([B.HIPCC, *B.FLAGS, *B.FILE_FLAGS.get(src.stem, []), *rest, "-c", str(src), "-o", str(obj)],
                           capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr)
        objs.append(obj)
    out = B.LIBDIR / f"libhgnn_{name}.so"
    r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out),
                        *map(str, objs)], capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(r.stderr)
    # the stamp _native checks before it loads this library through HGNN_LIB: the digest of the
    # current sources with these flags, and the flags themselves
    only_l = sorted(only) if only else None
    B.stamp_path(out).write_text(B._digest(tuple(rest), only_l) + "\n" +
                                 json.dumps({"extra": rest, "only": only_l}) + "\n")
    print(f"built {out}")


if __name__ == "__main__":
    main()
