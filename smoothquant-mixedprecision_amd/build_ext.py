"""Build libsqmp_w4a4.so (gfx950) in-tree with hipcc.

    python smoothquant-mixedprecision_amd/build_ext.py [--force]

Objects go to csrc/_obj/ (rebuilt when a source or header is newer), the shared
library to smoothquant/libsqmp_w4a4.so, next to the ctypes loader that opens it.
No torch C++ ABI is involved: the library exports the plain C functions declared in
include/sqmp_w4a4.h.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(CSRC, "_obj")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(HERE, "smoothquant", "libsqmp_w4a4.so")
ARCH = os.environ.get("SQMP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE,
          "-Wno-unused-result"]
# SQMP_DIAG=1: also instantiate the timing-diagnostic kernel variants (wrong results by
# design; never in the product build), into libsqmp_w4a4_diag.so (loaded by SQMP_DIAG_LIB=1)
if os.environ.get("SQMP_DIAG") == "1":
    CFLAGS.append("-DSQMP_DIAG_BUILD")
    OBJ = os.path.join(CSRC, "_obj_diag")
    LIB = os.path.join(HERE, "smoothquant", "libsqmp_w4a4_diag.so")


# per-source extra flags: the FP8 GEMM's fold stays scalar v_fma_f32 (SLP-packed v_pk_fma_f32
# beside MFMAs costs more issue cycles than the two FMAs it replaces, MI355X_MICROARCH.md)
FILE_FLAGS = {"sqmp_gemm_f8.hip": ["-fno-slp-vectorize"]}


def _headers():
    return glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o"))
    newest = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _headers()])
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= newest:
        return obj
    cmd = [HIPCC, *CFLAGS, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    jobs = min(len(srcs), int(os.environ.get("MAX_JOBS", "8")), 16)
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    newest_obj = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < newest_obj:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
