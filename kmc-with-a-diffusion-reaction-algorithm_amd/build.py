"""Build libkmc.so (HIP, gfx950) in-tree: lib/libkmc.so next to this file.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the
development container; the built library travels to the GPU box with the
repository snapshot.  Flags: -ffp-contract=off is load-bearing (no FMA
contraction: results must match the sequential oracle bit for bit).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libkmc.so")
RUN = os.path.join(LIB_DIR, "kmc_run")
STAMP = os.path.join(LIB_DIR, ".build_stamp")  # content hash of the inputs of the current build
SOURCES = ["kmc_engine.hip", "kmc_io.cpp"]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",
    "-fno-fast-math",
    "-fPIC",
    "-shared",
    "-Wall",
    "-Wno-unused-function",
]


def _inputs():
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    files.append(os.path.join(os.path.dirname(HERE), "include", "kmc.h"))
    return files


def source_hash() -> str:
    """sha256 over every source file and the compiler flags: a build is reused only if it was made from exactly these inputs
    (modification times are not trusted: a checkout or a copy resets them)."""
    h = hashlib.sha256()
    for f in sorted(_inputs()):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS + os.environ.get("KMC_EXTRA_FLAGS", "").split()).encode())
    return h.hexdigest()


def stale() -> bool:
    if not (os.path.exists(LIB) and os.path.exists(RUN) and os.path.exists(STAMP)):
        return True
    with open(STAMP) as f:
        return f.read().strip() != source_hash()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not stale():
        return LIB
    _build_lib(verbose)
    _build_driver(verbose)
    with open(STAMP, "w") as f:
        f.write(source_hash() + "\n")
    return LIB


def _build_driver(verbose: bool) -> None:
    """kmc_run: the drop-in executable (host C++, links libkmc.so)."""
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-o", RUN, os.path.join(CSRC, "kmc_run.cpp"),
           "-L" + LIB_DIR, "-lkmc", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("g++ failed building kmc_run")


def _build_lib(verbose: bool) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    extra = os.environ.get("KMC_EXTRA_FLAGS", "").split()  # diagnostic builds only (e.g. -DKMC_STAMPS)
    cmd = [HIPCC, *FLAGS, *extra, "-o", tmp, *[os.path.join(CSRC, s) for s in SOURCES]]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("hipcc failed building libkmc.so")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
