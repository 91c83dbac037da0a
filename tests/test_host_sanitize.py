"""The host backend (csrc/bb_host.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer
(no compute-sanitizer exists for the device, so the C++ twin of the env kernels is
sanitized on the host).  tests/native/host_sanitize.cpp drives every env entry point of include/bbvec.h
and compares each output with the C oracle (oracle/bb_oracle.c, compiled into the same binary as the
checker); any sanitizer report aborts it."""
import os
import shutil
import subprocess

import pytest

from runtime.build import CSRC, HOST_SOURCES
from runtime.lib import REPO_DIR

SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1",
       "-fopenmp", "-ffp-contract=off"]


@pytest.fixture(scope="module")
def sanitized_driver(tmp_path_factory):
    if not shutil.which("g++") or not shutil.which("gcc"):
        pytest.skip("no host compiler")
    out = tmp_path_factory.mktemp("san")
    inc = f"-I{os.path.join(REPO_DIR, 'include')}"
    oracle_o = str(out / "bb_oracle.o")
    subprocess.run(["gcc", *SAN, "-std=gnu11", "-c", os.path.join(REPO_DIR, "oracle", "bb_oracle.c"), "-o",
                    oracle_o], check=True)
    exe = str(out / "host_sanitize")
    subprocess.run(["g++", *SAN, "-std=c++17", inc, os.path.join(REPO_DIR, "tests", "native", "host_sanitize.cpp"),
                    *[os.path.join(CSRC, s) for s in HOST_SOURCES], oracle_o, "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("n,steps,threads", [(517, 160, "4"), (64, 400, "1")])
def test_host_backend_under_asan_ubsan(sanitized_driver, n, steps, threads):
    env = dict(os.environ, OMP_NUM_THREADS=threads,
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sanitized_driver, str(n), str(steps)], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "bit-exact" in r.stdout
