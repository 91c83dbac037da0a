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
    # name: extra -D flags on top of the shipped build (runtime/build.py)
    "main": [],
    # bb_rollout with search waves (rollout_async_kernel) vs in-step wave searches (rollout_kernel)
    "sync": ["-DBB_ASYNC=0"],
    "asw8": ["-DBB_ASYNC_SW=8"],
    "asp0": ["-DBB_ASYNC_SPRIO=0"],
    "asp2": ["-DBB_ASYNC_SPRIO=2"],
    "asl4": ["-DBB_ASYNC_SLEEP=4"],
    "asp3": ["-DBB_ASYNC_SPRIO=3"],
    "a2sw8": ["-DBB_ASYNC_SPRIO=2", "-DBB_ASYNC_SW=8"],
    "a2sl0": ["-DBB_ASYNC_SPRIO=2", "-DBB_ASYNC_SLEEP=0"],
    "a3sw8": ["-DBB_ASYNC_SPRIO=3", "-DBB_ASYNC_SW=8"],
    "apool": ["-DBB_ASYNC_POOL=1"],
    "apool0": ["-DBB_ASYNC_POOL=0"],
    "alate": ["-DBB_ASYNC_LATEPOLL=1"],
    "ae64": ["-DBB_ASYNC_ENVS=64"],
    "aptop": ["-DBB_ASYNC_PTOP=1"],
    # search waves hand back each env when its round decides it (shipped; "aearly0" is the call-end hand-back)
    "aearly": ["-DBB_ASYNC_EARLY=1"],
    "aearly0": ["-DBB_ASYNC_EARLY=0"],
    "astep": ["-DBB_ASYNC_STEP=1"],
    "astep32": ["-DBB_ASYNC_STEP=1", "-DBB_ASYNC_ENVS=32"],
    "alo": ["-DBB_ASYNC_LINEONLY=1"],
    "alo256": ["-DBB_ASYNC_LINEONLY=1", "-DBB_SLOW_LINE_MIN=256"],
    "alo128": ["-DBB_ASYNC_LINEONLY=1", "-DBB_SLOW_LINE_MIN=128"],
    "asexit0": ["-DBB_SLOW_EXIT=0"],
    "adearly": ["-DBB_ASYNC_DEARLY=1"],
    "aptde": ["-DBB_ASYNC_PTOP=1", "-DBB_ASYNC_DEARLY=1"],
    "ae32": ["-DBB_ASYNC_ENVS=32"],
    "ae64sw2": ["-DBB_ASYNC_SW=2"],
    "ae64sw3": ["-DBB_ASYNC_SW=3"],
    "ae64f0": ["-DBB_ASYNC_FAIR=0"],
    "ae64sp2": ["-DBB_ASYNC_SPRIO=2"],
    "ae64s1d": ["-DBB_ASYNC_SLOTS64=1"],
    "ae64s3": ["-DBB_ASYNC_SLOTS64=3"],
    "ae64sw8": ["-DBB_ASYNC_ENVS=64", "-DBB_ASYNC_SW=8"],
    "ae64sw6": ["-DBB_ASYNC_ENVS=64", "-DBB_ASYNC_SW=6"],
    "ae64s1": ["-DBB_ASYNC_ENVS=64", "-DBB_ASYNC_SLOTS64=1"],
    "alatediag": ["-DBB_ASYNC_LATEPOLL=1", "-DBB_ASYNC_DIAG=1"],
    "apsw8": ["-DBB_ASYNC_SW=8"],
    "apsw2": ["-DBB_ASYNC_SW=2"],
    "apsw6": ["-DBB_ASYNC_SW=6"],
    "afair0": ["-DBB_ASYNC_FAIR=0"],
    "aslot2": ["-DBB_ASYNC_SLOTS=2"],
    "apool3": ["-DBB_ASYNC_POOL=1", "-DBB_ASYNC_SPRIO=3"],
    "adiag": ["-DBB_ASYNC_DIAG=1"],
    "adiagp": ["-DBB_ASYNC_DIAG=1", "-DBB_ASYNC_POOL=1"],
    "adiag2": ["-DBB_ASYNC_DIAG=1", "-DBB_ASYNC_SPRIO=2"],
    # env waves: an env moves only while it is < W steps ahead of its wave's slowest env (output-row window)
    "aw4": ["-DBB_ASYNC_WINDOW=4"],
    "aw8": ["-DBB_ASYNC_WINDOW=8"],
    "aw12": ["-DBB_ASYNC_WINDOW=12"],
    "aw16": ["-DBB_ASYNC_WINDOW=16"],
    "aw24": ["-DBB_ASYNC_WINDOW=24"],
    # env waves: output rows [lo, lo + R) staged in LDS and written out as whole lines (BB_ASYNC_RING)
    "ar8": ["-DBB_ASYNC_RING=8"],
    "ar12": ["-DBB_ASYNC_RING=12"],
    "ar16": ["-DBB_ASYNC_RING=16"],
    "adiagr16": ["-DBB_ASYNC_DIAG=1", "-DBB_ASYNC_RING=16"],
    # LDS bank spread of the per-lane table reads: PieceRow 64 -> 80 bytes, JumpRow 32 -> 48 bytes
    "rp16": ["-DBB_ROW_PAD=16"],
    "jp16": ["-DBB_JUMP_PAD=16"],
    "rjp16": ["-DBB_ROW_PAD=16", "-DBB_JUMP_PAD=16"],
    "rp8": ["-DBB_ROW_PAD=8"],
    "rp24": ["-DBB_ROW_PAD=24"],
    "rp40": ["-DBB_ROW_PAD=40"],
    # rollout kernel workgroup shape (waves per workgroup; SIMD partners share LDS progress words at 512)
    "rblk64": ["-DBB_ROLL_BLOCK=64"],
    "rblk256": ["-DBB_ROLL_BLOCK=256"],
    # 64 envs per wave, one wave per SIMD (256-thread workgroups, no partner priority), in-lane slots 0|1
    "e64": ["-DBB_ROLL_ENVS=64", "-DBB_ROLL_BLOCK=256", "-DBB_ROLL_FAIR=0", "-DBB_ROLL_SLOTS=2"],
    "e64s1": ["-DBB_ROLL_ENVS=64", "-DBB_ROLL_BLOCK=256", "-DBB_ROLL_FAIR=0", "-DBB_ROLL_SLOTS=1"],
    # rollout: branchy apply_move; policy Philox at the top of every step
    "brmove": ["-DBB_ROLL_BFMOVE=0"],
    "ptop": ["-DBB_ROLL_PHILOX_TOP=1"],
    # rollout: attempt 1 drawn before the move, quick slot in every lane (no branch)
    "dearly": ["-DBB_ROLL_DRAW_EARLY=1"],
    # gen_hands_multi passes: slot owner by scalar reads of the attempt offsets instead of LDS markers
    "ownrl": ["-DBB_PASS_OWNER_RL=1"],
    # rollout: copy 1 exec-masked off through the move and the finalize (board + drawn ids by permlane32_swap);
    # shipped (r03), "halfoff" is the round-2 form with both copies doing the move and the finalize
    "halfidle": ["-DBB_ROLL_HALF_IDLE=1"],
    "halfoff": ["-DBB_ROLL_HALF_IDLE=0"],
    # bb_step (single-step instantiation): eager seeded-reset state / unconditional column stores
    "seager": ["-DBB_STEP_LAZY_RESET=0"],
    "sallst": ["-DBB_STEP_COND_STORE=0"],
    "scond1": ["-DBB_STEP_COND_STORE=1"],
    "seager_allst": ["-DBB_STEP_LAZY_RESET=0", "-DBB_STEP_COND_STORE=0"],
    "brquick": ["-DBB_ROLL_BFQUICK=0"],
    "brpass": ["-DBB_PASS_BF=0"],
    # rollout SIMD-partner priority: 0 none, 1 alternate per step, 2 the wave behind takes it (shipped)
    "fair0": ["-DBB_ROLL_FAIR=0"],
    "fair1": ["-DBB_ROLL_FAIR=1"],
    # round-1 escalate variants (their flags were not recorded)
    "esc0": ["-DBB_ESC_MULTI=0", "-DBB_ESC_GROUP=8"],
    "escg8": ["-DBB_ESC_GROUP=8"],
    "escg16": ["-DBB_ESC_GROUP=16"],
    "escg32": ["-DBB_ESC_GROUP=32"],  # == the shipped default, kept as a named A/B arm
    "escj": ["-DBB_ESC_LDS_JUMP=1"],
    "escjb128": ["-DBB_ESC_LDS_JUMP=1", "-DBB_ESC_BLOCK=128"],
    "escb128": ["-DBB_ESC_BLOCK=128"],
    # gen_hands_multi: attempt batch sized for 1..4 passes of 64 slots (shipped 3)
    "mp1": ["-DBB_MULTI_PASSES=1"],
    "mp2": ["-DBB_MULTI_PASSES=2"],
    "mp4": ["-DBB_MULTI_PASSES=4"],
    "mp6": ["-DBB_MULTI_PASSES=6"],
    # pass leaf tests without the line clear (pair_quick_nc): measured -1.3%, not shipped
    "passnc": ["-DBB_PASS_NC=1"],
    # board convolutions (csrc/bb_conv.hip): forward weight stages (input channels, ring slots);
    # NOT a correct convolution: 1 = no output stores, 2 = one tap of nine
    "cf64r2": ["-DBB_CONV_FWD_SCI=64", "-DBB_CONV_FWD_RING=2"],
    "cf64r3": ["-DBB_CONV_FWD_SCI=64", "-DBB_CONV_FWD_RING=3"],
    "cf32r3": ["-DBB_CONV_FWD_SCI=32", "-DBB_CONV_FWD_RING=3"],
    "cf32r2": ["-DBB_CONV_FWD_SCI=32", "-DBB_CONV_FWD_RING=2"],
    "cfb1": ["-DBB_CONV_FWD_BOARDS=1"],
    "cfb1s32": ["-DBB_CONV_FWD_BOARDS=1", "-DBB_CONV_FWD_SCI=32", "-DBB_CONV_FWD_RING=3"],
    "cm32": ["-DBB_CONV_MFMA16=0"],
    # LLVM AMDGPU scheduler strategies (whole library; the rollout kernel is the one that cares); shipped:
    # max-ilp (runtime/build.py), so "silp" == "main" and "sdef" is the LLVM default measured against it
    "sdef": ["-mllvm", "-amdgpu-sched-strategy=default"],
    "silp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
    "smem": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
    # on top of the shipped max-ilp: GCN register-pressure trackers in the scheduler; -O2
    "strk": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
    "o2": ["-O2"],
    # "unr600" (-mllvm -unroll-threshold=600) was measured here and is now shipped (runtime/build.py)
    "inl": ["-mllvm", "-inline-threshold=1000"],
    # NHWC BatchNorm reductions: rows in flight per thread (shipped: backward 2, forward 8)
    "bnu8": ["-DBB_BN_UNROLL_BWD=8"],
    "bnu4": ["-DBB_BN_UNROLL_BWD=4"],  # the round-2 default before bnab
    "bnu2": ["-DBB_BN_UNROLL_BWD=2"],
    "bnf16": ["-DBB_BN_UNROLL_FWD=16"],
    "cw16": ["-DBB_CONV_WG16=1"],
    "cst0": ["-DBB_CONV_STORE_LDS=0"],
    "cdiag1": ["-DBB_CONV_DIAG=1"],
    # BatchNorm NHWC reduction blocks (shipped 512)
    "bnr1024": ["-DBB_BN_RBLOCKS=1024"],
    "bnr2048": ["-DBB_BN_RBLOCKS=2048"],
    "cdiag2": ["-DBB_CONV_DIAG=2"],
    # bb_step (T = 1) workgroup-cooperative hand search (tools/patches/step_coop.diff, measured slower and
    # not shipped; apply the patch to rebuild these): off, own-search rounds first, attempts per wave and round
    "coop0": ["-DBB_STEP_COOP=0"],
    "coopr2": ["-DBB_STEP_COOP_ROUNDS=2"],
    "coopkw8": ["-DBB_STEP_COOP_KW=8"],
    "coopkw16": ["-DBB_STEP_COOP_KW=16"],
    # exact phase (slow_phase_wave): no early exit; both orders' leaves in full
    "sexit0": ["-DBB_SLOW_EXIT=0"],
    "sline0": ["-DBB_SLOW_LINE_ONLY=0"],
    "slm256": ["-DBB_SLOW_LINE_MIN=256"],
    "slm512": ["-DBB_SLOW_LINE_MIN=512"],
    "slm1024": ["-DBB_SLOW_LINE_MIN=1024"],
    # hand searches balanced over the workgroup's 8 waves (BB_WG_BALANCE, measured slower, shipped 0):
    # 1 = bb_step only; 2 = bb_rollout's steps too
    "wgb1": ["-DBB_WG_BALANCE=1"],
    "wgb2": ["-DBB_WG_BALANCE=2"],
    # bb_step's single-step instantiation with 16 / 8 envs per wave (4 / 8 copies, as many quick-test slots;
    # 4,096 / 8,192 waves at 65,536 envs: more waves than resident slots, so the dispatcher balances them)
    "st16": ["-DBB_STEP_ENVS=16"],
    "st8": ["-DBB_STEP_ENVS=8"],
    # ... and with 256 / 128-thread workgroups (BB_STEP_ROLL_BLOCK; 3 resident waves per SIMD at <= 168 VGPRs)
    "st32b256": ["-DBB_STEP_ROLL_BLOCK=256"],
    "st16b256": ["-DBB_STEP_ENVS=16", "-DBB_STEP_ROLL_BLOCK=256"],
    "st8b256": ["-DBB_STEP_ENVS=8", "-DBB_STEP_ROLL_BLOCK=256"],
    "st16b128": ["-DBB_STEP_ENVS=16", "-DBB_STEP_ROLL_BLOCK=128"],
    # timing diagnostics of the rollout phases (tools/diag_rollout.py, BB_DEBUG_MODE=16)
    "diag3": ["-DBB_ROLL_DIAG=3", "-DBB_ASYNC=0"],
    # NOT reference semantics (instruction-count attribution only): 1 = in-lane quick test, no wave
    # search (an unaccepted draw is kept); 2 = first draw kept, no test at all
    "diag1": ["-DBB_ROLL_DIAG=1", "-DBB_ASYNC=0"],
    "diag2": ["-DBB_ROLL_DIAG=2", "-DBB_ASYNC=0"],
}


def build(name: str) -> str:
    flags = VARIANTS[name]
    os.makedirs(OUT, exist_ok=True)
    out = os.path.join(OUT, f"libbbvec_{name}.so")
    base = [f for f in HIPCC_FLAGS if not f.startswith("--offload-arch")]  # the shipped flags (runtime/build.py)
    if any(f.startswith("-amdgpu-sched-strategy") for f in flags):  # a scheduler variant replaces the shipped one
        i = base.index("-mllvm")
        del base[i:i + 2]
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
