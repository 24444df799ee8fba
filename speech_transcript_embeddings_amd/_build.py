"""Build libste.so (all HIP kernels + the C ABI of include/ste.h) for gfx950, in-tree.

hipcc cross-compiles without a GPU, so this runs in the CPU container and the
resulting .so travels to the GPU box with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
INCLUDE = PKG.parent / "include"
OBJ = PKG / "_obj"
LIB = PKG / "libste.so"
# -DSTE_AB: the A/B build (libste_ab.so, objects in _obj_ab) whose switches read STE_* environment
# variables (csrc/common.h STE_AB_ENV); the shipped libste.so reads none.  Select it at run time with
# STE_LIB=.../libste_ab.so (_lib.py).
OBJ_AB = PKG / "_obj_ab"
LIB_AB = PKG / "libste_ab.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# No packed-fp32 VALU code (v_pk_add/mul/fma_f32): on the MI355X, with another stream's MFMA
# GEMM running on the same CUs, the LayerNorm backward-pair kernel's SLP-packed f32 ops returned
# wrong values in lanes 48-63 of single registers (profiles/det_ln.py: 12/39 and 39/39
# repetitions differed from the first; 0/39 with packed fp32 disabled, 0/39 without the
# concurrent GEMM).  Beside MFMAs they are also no faster than two single-issue ops
# (MI355X_MICROARCH.md, filler prices).  The host compilation warns that it ignores the
# device feature.
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
         "-munsafe-fp-atomics", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
         f"-I{INCLUDE}", f"-I{CSRC}"]


def _headers_mtime() -> float:
    hs = list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h")) + [Path(__file__)]
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _compile(src: Path, hdr_mtime: float, verbose: bool, ab: bool = False) -> Path:
    obj = (OBJ_AB if ab else OBJ) / (src.stem + ".o")
    if obj.exists() and obj.stat().st_mtime >= max(src.stat().st_mtime, hdr_mtime):
        return obj
    # STE_BUILD_DEFINES="-DNAME=V ...": extra macros for one-off experiment builds (A/B only)
    extra = os.environ.get("STE_BUILD_DEFINES", "").split() if ab else []
    cmd = [HIPCC, *FLAGS, *(["-DSTE_AB"] if ab else []), *extra, "-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int = 8, ab: bool = False) -> Path:
    obj_dir, lib = (OBJ_AB, LIB_AB) if ab else (OBJ, LIB)
    obj_dir.mkdir(exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))
    hm = _headers_mtime()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hm, verbose, ab), srcs))
    newest = max(o.stat().st_mtime for o in objs)
    if not lib.exists() or lib.stat().st_mtime < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs)]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return lib


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, ab="--ab" in sys.argv))
