"""Build libpathfeas.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libpathfeas.so")
SOURCES = ["pathfeas.hip", "pf_eval.hip", "pf_keccak.hip", "u256.h", "u256_cols.h",
           os.path.join("..", "..", "include", "pathfeas.h"),
           os.path.join("..", "..", "include", "pf_bytecode.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -structurizecfg-skip-uniform-regions: the interpreter loop's dispatch is wave-uniform (the
# kernels keep every per-lane condition a select, pf_eval.hip / u256.h lane_mask), so the
# structurizer may leave its regions as plain scalar branches instead of flag-driven flow
# blocks (fewer SALU and branches per bytecode instruction)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-value",
         "-mllvm", "-structurizecfg-skip-uniform-regions=true"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(os.path.join(CSRC, s)) > t for s in SOURCES)


LOWER_OUT = os.path.join(HERE, "libpflower.so")
LOWER_SOURCES = ["pf_lower.cpp", "pf_seed.cpp", "pf_terms.cpp", "pf_recheck.cpp", "pf_pool.h", os.path.join("..", "..", "include", "pf_lower.h"),
                 os.path.join("..", "..", "include", "pf_bytecode.h")]


def build_lower(force: bool = False, verbose: bool = False) -> str:
    """libpflower.so: the host-only native lowering (g++, no HIP runtime)."""
    if not force and os.path.exists(LOWER_OUT) and all(
            os.path.getmtime(os.path.join(CSRC, s)) <= os.path.getmtime(LOWER_OUT) for s in LOWER_SOURCES):
        return LOWER_OUT
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", LOWER_OUT + ".tmp",
           os.path.join(CSRC, "pf_lower.cpp"), os.path.join(CSRC, "pf_seed.cpp"),
           os.path.join(CSRC, "pf_terms.cpp"), os.path.join(CSRC, "pf_recheck.cpp")]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(LOWER_OUT + ".tmp", LOWER_OUT)
    return LOWER_OUT


def build_library(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", os.path.join(CSRC, "pathfeas.hip")]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True, cwd=CSRC)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build_lower(force="--force" in sys.argv, verbose=True))
    print(build_library(force="--force" in sys.argv, verbose=True))
