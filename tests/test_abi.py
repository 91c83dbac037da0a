"""The C-ABI library loads (no GPU needed) and exports every symbol that
include/bbvec.h declares; host-only entry points are exact."""
import os
import re

import numpy as np
import pytest

from runtime import lib as L

HEADER = os.path.join(os.path.dirname(os.path.dirname(__file__)), "include", "bbvec.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bb_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert set(declared_symbols()) == set(L.SIGNATURES)


def test_library_exports_every_symbol(lib):
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.bb_abi_version() == L.ABI_VERSION == 8


def test_build_id_is_these_sources(lib):
    """bb_build_id ties the binary to HEAD's sources: the id is the hash of csrc/, include/bbvec.h and the
    flags, the .so carries it where build.py reads it without loading, and load() refuses a mismatch."""
    from runtime import build as B

    sid = B.source_id()
    assert len(sid) == 16 and lib.bb_build_id().decode() == sid == B.built_id(L.LIB_PATH)
    assert L.build_id() == sid
    host = B.build_host_lib(verbose=False)
    assert B.built_id(host) == B.host_source_id() == L.build_id(host=True)


def test_stale_library_is_refused(lib, tmp_path, monkeypatch):
    """A library whose id differs from the sources beside it is refused by name, not loaded silently."""
    from runtime import build as B

    monkeypatch.setattr(B, "source_id", lambda: "0" * 16)
    monkeypatch.setattr(L, "_lib", None)
    with pytest.raises(L.BBNativeError, match="built from other sources"):
        L.load()


def test_struct_sizes(lib):
    assert L.INFO_BYTES == 56


@pytest.mark.parametrize("seed", [0, 1, 42, 43, 2 ** 32 - 1, 2 ** 32, 2 ** 40 + 7, 2 ** 63, 2 ** 64 - 1])
def test_pcg64_seeding_matches_numpy(lib, seed):
    w = L.pcg64_seed(seed)
    st = np.random.PCG64(seed).state["state"]
    assert (w[0] << 64 | w[1]) == st["state"]
    assert (w[2] << 64 | w[3]) == st["inc"]


def test_seed42_golden_state(lib):
    import json
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_seed42.json")))
    w = L.pcg64_seed(42)
    assert str(w[0] << 64 | w[1]) == g["numpy_pcg64_seed42"]["state"]
    assert str(w[2] << 64 | w[3]) == g["numpy_pcg64_seed42"]["inc"]


def test_create_without_gpu_fails_loudly(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import ctypes as C
    h = C.c_void_p()
    rc = lib.bb_create(4, 0, C.byref(L.reward_cfg(dict(
        line_clear_base=1.0, block_placed=0.01, game_over_penalty=-1.0, hole_penalty=-0.05, center_bonus=0.02,
        combo_multiplier_bonus=0.5, survival_bonus=0.001))), 1, C.byref(h))
    assert rc != 0 and "no HIP device" in L.last_error()
