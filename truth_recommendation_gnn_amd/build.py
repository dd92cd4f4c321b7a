"""Build the in-tree C-ABI library ``lib/libhgnn.so`` from ``csrc/*.hip`` for gfx950.

``python -m truth_recommendation_gnn_amd.build`` (or ``__graft_entry__.build()``).  hipcc
cross-compiles here without a GPU; the built ``.so`` stays in-tree (git-ignored, not
gpurun-ignored) so it travels to the GPU box with the snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import pathlib
import subprocess
import sys

PKG = pathlib.Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
LIB = LIBDIR / "libhgnn.so"
INCLUDE = PKG.parent / "include"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
         "-Wno-unused-result", f"-I{INCLUDE}"]
# per-source extra flags: the split-once K3 kernels are vector-issue-bound beside their MFMAs,
# where SLP-packed v_pk_add_f32 costs more than two scalar adds (MI355X_MICROARCH.md; A/B at the
# cfg4 shapes: 9M-row backward 3.65 -> 3.62 ms at K = 256, 3.88 -> 3.83 ms at K = 128)
FILE_FLAGS = {"linear_xs": ["-fno-slp-vectorize"]}


def _sources():
    return sorted(CSRC.glob("*.hip"))


def _digest(extra=(), only=None) -> str:
    """Hash of the sources and the flags they are built with.  ``extra`` / ``only``: the added
    flags of an A/B variant build (scripts/build_variant.py) and the sources they apply to."""
    h = hashlib.sha256()
    for p in _sources() + sorted(CSRC.glob("*.h")) + [INCLUDE / "hgnn.h"]:
        h.update(p.name.encode())
        h.update(p.read_bytes())
    # flags without the absolute include path: the same tree built elsewhere (the GPU box's copy)
    # must hash the same, or the shipped library would be rebuilt there
    h.update(" ".join(f for f in FLAGS if not f.startswith("-I")).encode())
    h.update(repr(sorted(FILE_FLAGS.items())).encode())
    if extra:
        h.update(repr((list(extra), sorted(only) if only else None)).encode())
    return h.hexdigest()[:16]


def stamp_path(lib: pathlib.Path) -> pathlib.Path:
    return lib.with_name(lib.name[:-len(".so")] + ".digest")


def check_library(lib: pathlib.Path) -> None:
    """Refuse a library not built from the sources in this tree: its stamp (written by
    ``build()`` or scripts/build_variant.py beside it) must hold the digest of the current
    sources and of the flags it records."""
    st = stamp_path(lib)
    if not st.exists():
        raise RuntimeError(f"{lib.name}: no build stamp {st.name}; rebuild with "
                           "`python -m truth_recommendation_gnn_amd.build`")
    lines = st.read_text().splitlines()
    extra, only = (), None
    if len(lines) > 1 and lines[1].strip():
        rec = json.loads(lines[1])
        extra, only = tuple(rec["extra"]), rec.get("only")
    want = _digest(extra, only)
    if not lines or lines[0].strip() != want:
        raise RuntimeError(f"{lib.name} was built from other sources (stamp "
                           f"{lines[0].strip() if lines else '?'}, tree {want}); rebuild it")


def build(force: bool = False, verbose: bool = True) -> pathlib.Path:
    """Compile every ``csrc/*.hip`` to an object and link ``lib/libhgnn.so``.

    Skips the work when the sources' digest matches the one recorded beside the library.
    """
    LIBDIR.mkdir(exist_ok=True)
    stamp = stamp_path(LIB)
    dig = _digest()
    if not force and LIB.exists() and stamp.exists() and stamp.read_text().strip() == dig:
        return LIB
    objdir = PKG.parent / "build" / "obj"
    objdir.mkdir(parents=True, exist_ok=True)

    def compile_one(src: pathlib.Path) -> pathlib.Path:
        obj = objdir / (src.stem + ".o")
        cmd = [HIPCC, *FLAGS, *FILE_FLAGS.get(src.stem, []), "-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stdout}\n{r.stderr}")
        if verbose and r.stderr.strip():
            sys.stderr.write(r.stderr)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, _sources()))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    stamp.write_text(dig + "\n")
    if verbose:
        print(f"built {LIB} ({LIB.stat().st_size // 1024} KiB)")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
