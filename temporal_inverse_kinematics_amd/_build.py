"""Build libtik.so in-tree with hipcc for gfx950 (no JIT cache, no torch extension).

    python -m temporal_inverse_kinematics_amd._build [--debug]

The shared library lands next to this file (git-ignored, but it travels to
the GPU box with the gpurun snapshot).
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
REPO = os.path.dirname(PKG)
LIB = os.path.join(PKG, "libtik.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def source_digest() -> str:
    """sha256 over the library's sources (csrc/*.hip, *.cpp, *.h and
    include/tik.h, by file name and content): names the tree a measurement
    was taken on. The PMC summaries under profiles/ carry it, and bench.py
    takes counter fields only from a summary of the tree it benchmarks."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(_sources() + glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(REPO, "include", "tik.h")]
    for f in files:
        h.update(os.path.relpath(f, REPO).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def _needs_rebuild(objs_srcs, lib):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = _sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(REPO, "include", "tik.h"),
                                                                 os.path.abspath(__file__)]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, debug: bool = False, verbose: bool = False, out: str = None, flags=None) -> str:
    """Build libtik.so in-tree (or a diagnostic variant: `out` = another path,
    `flags` = extra hipcc flags such as -DTIK_XTUNE; loaded with TIK_LIB=out)."""
    srcs = _sources()
    lib = out or LIB
    objdir = os.path.join(PKG, "build") if out is None else out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    if not force and out is None and not _needs_rebuild(srcs, LIB):
        return LIB
    opt = ["-O0", "-g"] if debug else ["-O3"]
    # diagnostic builds: e.g. TIK_HIPCC_FLAGS="-DTIK_XTRACE" (xgemm phase stamps), "-DTIK_XTUNE"
    opt += os.environ.get("TIK_HIPCC_FLAGS", "").split() + list(flags or [])
    common = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-result",
              f"-I{os.path.join(REPO, 'include')}", *opt]

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = common + ["-c", src, "-o", obj]
        if src.endswith(".cpp"):
            cmd = common + ["-x", "hip", "-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{r.stdout}\n{r.stderr}")
        if verbose and (r.stderr or r.stdout):
            print(r.stdout + r.stderr)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = lib + ".tmp"
    r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    # python -m temporal_inverse_kinematics_amd._build [--debug] [--out PATH -DFLAG ...]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    fl = [a for a in sys.argv[1:] if a.startswith("-D")]
    print(build(force=True, debug="--debug" in sys.argv, verbose=True, out=out, flags=fl))
