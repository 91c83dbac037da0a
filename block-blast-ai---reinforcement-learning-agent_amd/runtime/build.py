"""Build libbbvec.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

from .lib import HOST_LIB_PATH, LIB_PATH, PKG_DIR, REPO_DIR

CSRC = os.path.join(PKG_DIR, "csrc")
SOURCES = ["bb_env.hip", "bb_ppo.hip", "bb_nn.hip", "bb_loss.hip", "bb_conv.hip", "bb_conv32.hip", "bb_optim.hip", "bb_capi.cpp", "bb_tables.cpp"]
HEADERS = ["bb_device.h", "bb_solver.h", "bb_env_internal.h", "bb_seed.h"]
ARCH = os.environ.get("BB_OFFLOAD_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",  # reward / GAE arithmetic must not be fused into FMAs
    "-fPIC",
    "-shared",
    "-Wno-unused-result",
    # LLVM's max-ILP machine scheduler: +0.8% on the rollout kernel (8.85e9 vs 8.78e9 env-steps/s, 3 interleaved
    # repeats, profiles/r02/ab/schedab_*), the PPO update step unchanged; max-memory-clause was -1.8%
    "-mllvm", "-amdgpu-sched-strategy=max-ilp",
    # a higher loop-unroll threshold: +0.6% on the rollout kernel (8.90e9 vs 8.85e9, 3 interleaved repeats,
    # profiles/r02/ab/flagab2_*), the update step 1.863 vs 1.868 ms (unrupd_*)
    "-mllvm", "-unroll-threshold=600",
]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if cand and (os.path.isabs(cand) and os.path.exists(cand) or not os.path.isabs(cand)):
            return cand
    return "hipcc"


MARKER = b"bbvec-build-id:"  # csrc/bb_capi.cpp / bb_host.cpp kBuildIdMarker
HEADER = os.path.join(REPO_DIR, "include", "bbvec.h")


def _source_id(files, flags) -> str:
    """First 16 hex digits of SHA-256 over the flags and every input file's name and bytes: the id a
    library built from exactly these sources carries (bb_build_id)."""
    h = hashlib.sha256()
    h.update("\0".join(flags).encode())
    for f in files:
        h.update(b"\0" + os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def source_id() -> str:
    """The build id of libbbvec.so for the sources in this tree."""
    return _source_id([os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [HEADER], HIPCC_FLAGS)


def host_source_id() -> str:
    """The build id of libbbvec_host.so for the sources in this tree."""
    return _source_id([os.path.join(CSRC, s) for s in HOST_SOURCES + HOST_HEADERS] + [HEADER], HOST_FLAGS)


def built_id(path: str):
    """The build id embedded in a built library (read from its bytes; the library is not loaded), or None."""
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    k = data.find(MARKER)
    return data[k + len(MARKER):k + len(MARKER) + 16].decode("ascii", "replace") if k >= 0 else None


def build_lib(force: bool = False, verbose: bool = True) -> str:
    """Build libbbvec.so unless the one in the tree already carries the id of these sources."""
    sid = source_id()
    if not force and built_id(LIB_PATH) == sid:
        return LIB_PATH
    tmp = LIB_PATH + ".tmp"
    cmd = [_hipcc(), *HIPCC_FLAGS, f'-DBB_BUILD_ID="{sid}"', f"-I{os.path.join(REPO_DIR, 'include')}",
           *[os.path.join(CSRC, s) for s in SOURCES], "-o", tmp]
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


# the host backend of the env entry points (csrc/bb_host.cpp): plain C++, OpenMP over envs
HOST_SOURCES = ["bb_host.cpp"]
HOST_HEADERS = ["bb_seed.h"]
HOST_FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-fopenmp", "-Wall", "-Wextra"]


def build_host_lib(force: bool = False, verbose: bool = True) -> str:
    sid = host_source_id()
    if not force and built_id(HOST_LIB_PATH) == sid:
        return HOST_LIB_PATH
    tmp = HOST_LIB_PATH + ".tmp"
    cmd = [os.environ.get("CXX", "g++"), *HOST_FLAGS, f'-DBB_BUILD_ID="{sid}"', f"-I{os.path.join(REPO_DIR, 'include')}",
           *[os.path.join(CSRC, s) for s in HOST_SOURCES], "-o", tmp]
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, HOST_LIB_PATH)
    return HOST_LIB_PATH


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv)
    build_host_lib(force="--force" in sys.argv)
