"""Build the C oracle (oracle/bb_oracle.c) into oracle/_build/libbboracle.so.

TEST INFRASTRUCTURE ONLY: called by __graft_entry__.build() next to the
product build; the product never loads the result.  The .so is git-ignored
but travels to the GPU box with the tree (gpurun ships built libraries).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "bb_oracle.c")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libbboracle.so")
CFLAGS = ["-O2", "-std=gnu11", "-fopenmp", "-ffp-contract=off", "-fPIC", "-shared", "-Wall", "-Wextra",
          "-Wno-unused-parameter"]


def build_oracle(force: bool = False, verbose: bool = True) -> str:
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [os.environ.get("CC", "gcc"), *CFLAGS, SRC, "-o", tmp]
    if verbose:
        print("[build oracle]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build_oracle(force="--force" in sys.argv)
