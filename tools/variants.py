#!/usr/bin/env python3
"""Diagnostics (not product): tuning builds of libbbvec.so, recorded here so
every A/B number in DESIGN.md can be rebuilt from the repo.

    python tools/variants.py build NAME [NAME ...]   -> tools/variants/libbbvec_NAME.so
    python tools/variants.py list

Load one with BBVEC_LIB=tools/variants/libbbvec_NAME.so (runtime/lib.py).
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd", "csrc")
OUT = os.path.join(REPO, "tools", "variants")
sys.path.insert(0, os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"))
from runtime.build import HIPCC_FLAGS, SOURCES  # noqa: E402  the shipped source list and flags

VARIANTS = {
    # name: extra -D flags on top of the shipped build (runtime/build.py).  Only knobs the source still has;
    # the round-3 compile-time variants measured slower were removed (tools/patches/r03_compile_variants.diff
    # restores them), so their A/B arms cannot be rebuilt from this tree.
    "main": [],
    # round 6: LLVM machine-scheduler strategy and unroll threshold re-measured on the current kernels (shipped:
    # max-ilp, 600; round 2 measured them on the round-2 rollout kernel)
    "siilp": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    "simaxocc": ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc"],
    "sminreg": ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"],
    "u300": ["-mllvm", "-unroll-threshold=300"],
    "u1200": ["-mllvm", "-unroll-threshold=1200"],
    "o2": ["-O2"],
    "trk": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
    "nocl": ["-mllvm", "-misched-cluster=0"],
    # BatchNorm finalisation: one wave per channel (round 4) instead of one workgroup
    "fin4": ["-DBB_BN_FIN_CPB=4"],
    # round 6: BatchNorm apply passes' loads per thread in flight (shipped 1, the round-5 form)
    "bau1": ["-DBB_BN_APPLY_UNROLL=1"],
    # BatchNorm NHWC reductions re-measured on the round-6 step: blocks (shipped 512), backward rows in flight
    # (shipped 2)
    "rb256": ["-DBB_BN_RBLOCKS=256"],
    "rb1024": ["-DBB_BN_RBLOCKS=1024"],
    "ub4": ["-DBB_BN_UNROLL_BWD=4"],
    "bau2": ["-DBB_BN_APPLY_UNROLL=2"],
    "bau4": ["-DBB_BN_APPLY_UNROLL=4"],
    "bau8": ["-DBB_BN_APPLY_UNROLL=8"],
    # chunks per thread of the NHWC apply grids (shipped 8): more, smaller workgroups
    "bpt4": ["-DBB_BN_APPLY_PT=4"],
    "bpt16": ["-DBB_BN_APPLY_PT=16"],
    "bpt16u1": ["-DBB_BN_APPLY_PT=16", "-DBB_BN_APPLY_UNROLL=1"],
    "bpt16u4": ["-DBB_BN_APPLY_PT=16", "-DBB_BN_APPLY_UNROLL=4"],
    "bpt32": ["-DBB_BN_APPLY_PT=32"],
    "bpt2": ["-DBB_BN_APPLY_PT=2"],
    "bpt2u1": ["-DBB_BN_APPLY_PT=2", "-DBB_BN_APPLY_UNROLL=1"],
    "bpt1u1": ["-DBB_BN_APPLY_PT=1", "-DBB_BN_APPLY_UNROLL=1"],
    # the gradient-norm pass: four 2,048-element chunks per workgroup (measured slower)
    "an4": ["-DBB_ADAM_NORM_CPB=4"],
    # round 6: the last-arriver hand-offs' arrive add relaxed (the round-5 form) instead of acq_rel
    "hrx": ["-DBB_HANDOFF_ORDER=__ATOMIC_RELAXED"],
    # round 5: search waves' pass schedule -- 0: gen_hands_multi's packed passes (round 4); quota per attempt
    # in a round's first pass (shipped 4) and later passes (shipped 64)
    "mq0": ["-DBB_SEARCH_QUOTA=0"],
    "q2": ["-DBB_QUOTA_FIRST=2"],
    "q8": ["-DBB_QUOTA_FIRST=8"],
    "qn16": ["-DBB_QUOTA_NEXT=16"],
    "sq1": ["-DBB_STEP_QUOTA=1"],
    # bb_rollout (rollout_async_kernel): search waves per workgroup, their priority, in-lane quick-test slots
    "asw3": ["-DBB_ASYNC_SW=3"],
    "asw5": ["-DBB_ASYNC_SW=5"],
    "asw6": ["-DBB_ASYNC_SW=6"],
    "asp2": ["-DBB_ASYNC_SPRIO=2"],
    "aslot0": ["-DBB_ASYNC_SLOTS=0"],
    "aslot2": ["-DBB_ASYNC_SLOTS=2"],
    "asl4": ["-DBB_ASYNC_SLEEP=4"],
    # the one in-lane slot starts from the fewest-anchor piece (quick_least_bf)
    "aqp0": ["-DBB_ASYNC_QPICK=0"],
    # diagnostics: every search call run a second time, results dropped (search waves' share of the SQ counts)
    "adup": ["-DBB_ASYNC_DIAG_DUPSEARCH=1"],
    "adupdiag": ["-DBB_ASYNC_DIAG_DUPSEARCH=1", "-DBB_ASYNC_DIAG=1"],
    # conv_fwd_kernel's stage loop rolled (address arithmetic per read) instead of unrolled
    "cfu0": ["-DBB_CONV_FWD_UNROLL=0"],
    # bb_step (step_fused_kernel): copy c's slot from the anchor-count rank c instead of hand slot c
    "sqp1": ["-DBB_STEP_QPICK=1"],
    "aphx": ["-DBB_ASYNC_PHILOX_EARLY=1"],
    # search waves: the exact phase's line-only second order above BB_SLOW_LINE_MIN tasks
    "alo0": ["-DBB_ASYNC_LINEONLY=1", "-DBB_SLOW_LINE_MIN=0"],
    "alo128": ["-DBB_ASYNC_LINEONLY=1", "-DBB_SLOW_LINE_MIN=128"],
    "alo512": ["-DBB_ASYNC_LINEONLY=1"],
    "aloff": ["-DBB_ASYNC_LINEONLY=0"],
    # fp32 board convolutions (csrc/bb_conv32.hip): input channels per weight stage, LDS ring slots
    "c32s64": ["-DBB_CONV32_SCI=64"],
    "c32r3": ["-DBB_CONV32_RING=3"],
    "l32bm64": ["-DBB_LINEAR32_BM=64", "-DBB_LINEAR32_WPE=1"],
    "l32wpe1": ["-DBB_LINEAR32_WPE=1"],
    "asw8": ["-DBB_ASYNC_SW=8"],
    # per-wave counters of rollout_async_kernel (tools/diag_async.py)
    "adiag": ["-DBB_ASYNC_DIAG=1"],
    "adiag2": ["-DBB_ASYNC_DIAG=2"],
    # LDS row stride of the piece table (shipped: 8 bytes of padding, 72-byte rows)
    "rp0": ["-DBB_ROW_PAD=0"],
    "rp16": ["-DBB_ROW_PAD=16"],
    "rp40": ["-DBB_ROW_PAD=40"],
    # gen_hands_multi: attempt batch sized for 1..4 passes of 64 slots (shipped 3)
    "mp2": ["-DBB_MULTI_PASSES=2"],
    "mp4": ["-DBB_MULTI_PASSES=4"],
    # exact phase: line-only second order above this many tasks (bb_step's single step; shipped 512)
    "slm256": ["-DBB_SLOW_LINE_MIN=256"],
    "slm1024": ["-DBB_SLOW_LINE_MIN=1024"],
    # board convolutions (csrc/bb_conv.hip): forward weight stages (input channels, ring slots);
    # NOT a correct convolution: cdiag1 = no output stores, cdiag2 = one tap of nine
    "cf64r3": ["-DBB_CONV_FWD_SCI=64", "-DBB_CONV_FWD_RING=3"],
    "cf32r3": ["-DBB_CONV_FWD_SCI=32", "-DBB_CONV_FWD_RING=3"],
    "cf32r4": ["-DBB_CONV_FWD_SCI=32", "-DBB_CONV_FWD_RING=4"],
    "cfb1": ["-DBB_CONV_FWD_BOARDS=1"],
    "cm32": ["-DBB_CONV_MFMA16=0"],
    "cw16": ["-DBB_CONV_WG16=1"],
    "cst0": ["-DBB_CONV_STORE_LDS=0"],
    "cdiag1": ["-DBB_CONV_DIAG=1"],
    "cdiag2": ["-DBB_CONV_DIAG=2"],
    # NHWC BatchNorm reductions: rows in flight per thread (shipped: backward 2, forward 8), reduction blocks
    "bnu4": ["-DBB_BN_UNROLL_BWD=4"],
    "bnf16": ["-DBB_BN_UNROLL_FWD=16"],
    "bnr1024": ["-DBB_BN_RBLOCKS=1024"],
    "bnr256": ["-DBB_BN_RBLOCKS=256"],
    # NHWC BatchNorm elementwise passes: 16-byte chunks per thread (shipped 8)
    "bnpt2": ["-DBB_BN_APPLY_PT=2"],
    "bnpt4": ["-DBB_BN_APPLY_PT=4"],
    "bnpt16": ["-DBB_BN_APPLY_PT=16"],
    # LLVM AMDGPU scheduler strategies (shipped: max-ilp, runtime/build.py) and -O2
    "sdef": ["-mllvm", "-amdgpu-sched-strategy=default"],
    "smem": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    "o2": ["-O2"],
    "ut300": ["-mllvm", "-unroll-threshold=300"],
    "ut1200": ["-mllvm", "-unroll-threshold=1200"],
    # bb_linear_bgrad shapes (shipped BB_BGRAD_CFG 0, 128-row chunks) and dropout grid caps / loads in flight
    # (shipped 128 blocks, 4): tools/bench_linear_tail.py, profiles/r05/lt/
    "bg1": ["-DBB_BGRAD_CFG=1"],
    "bg2": ["-DBB_BGRAD_CFG=2"],
    "bg3": ["-DBB_BGRAD_CFG=3"],
    "bgc32": ["-DBB_BGRAD_CHUNK=32"],
    "bgc64": ["-DBB_BGRAD_CHUNK=64"],
    "drop64": ["-DBB_DROP_BLOCKS=64"],
    "drop256": ["-DBB_DROP_BLOCKS=256"],
    "drop512": ["-DBB_DROP_BLOCKS=512"],
    "dropu1": ["-DBB_DROP_UNROLL=1"],
    # the input layer (conv 4 -> 64): forward workgroups at most (shipped 256: two boards per wave at 2,048
    # boards), weight-gradient partial chunks (shipped 128); tools/bench_conv_in.py, profiles/r05/ci/
    "if128": ["-DBB_IN_FWD_BLOCKS=128"],
    "if512": ["-DBB_IN_FWD_BLOCKS=512"],
    "iw32": ["-DBB_IN_WG_CHUNKS=32"],
    "iw64": ["-DBB_IN_WG_CHUNKS=64"],
    "iw256": ["-DBB_IN_WG_CHUNKS=256"],
}


def build(name: str) -> str:
    flags = VARIANTS[name]
    os.makedirs(OUT, exist_ok=True)
    out = os.path.join(OUT, f"libbbvec_{name}.so")
    base = [f for f in HIPCC_FLAGS if not f.startswith("--offload-arch")]  # the shipped flags (runtime/build.py)
    for opt in ("-amdgpu-sched-strategy", "-unroll-threshold"):  # a variant of a shipped -mllvm option replaces it
        if any(f.startswith(opt) for f in flags):
            i = next(k for k in range(len(base)) if base[k].startswith(opt))
            del base[i - 1:i + 1]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", *base, *flags, f"-I{os.path.join(REPO, 'include')}",
           *[os.path.join(CSRC, s) for s in SOURCES], "-o", out]
    subprocess.run(cmd, check=True)
    return out


def main():
    if len(sys.argv) < 2 or sys.argv[1] == "list":
        for k, v in VARIANTS.items():
            print(f"{k:12s} {' '.join(v)}")
        return
    names = sys.argv[2:]
    with ThreadPoolExecutor(max_workers=4) as ex:
        for out in ex.map(build, names):
            print(out)


if __name__ == "__main__":
    main()
