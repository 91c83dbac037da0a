"""Device-resident batch of Block Blast envs: one libbbvec handle + its buffers.

This is the torch-facing layer under the Gym surface.  All tensors live on the
handle's GPU; every call launches on torch's current stream of that device and
never synchronises (except the explicit host copies ``state()`` /
``set_state()``).

``device="cpu"`` selects the host backend (libbbvec_host.so, the same C-ABI on
CPU tensors, csrc/bb_host.cpp) explicitly; without it a missing HIP device is
an error, never a silent switch to the CPU.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np
import torch

from . import lib as L

DEFAULT_REWARDS = {  # block_blast_env.py:63-71
    "line_clear_base": 1.0,
    "block_placed": 0.01,
    "game_over_penalty": -1.0,
    "hole_penalty": -0.05,
    "center_bonus": 0.02,
    "combo_multiplier_bonus": 0.5,
    "survival_bonus": 0.001,
}

INFO_DTYPE = np.dtype(
    [
        ("score", "<i8"), ("score_gained", "<i8"), ("term_board", "<u8"),
        ("moves", "<i4"), ("lines", "<i4"), ("max_combo", "<i4"), ("blocks", "<i4"),
        ("term_hand", "<u4"), ("holes", "u1"), ("filled", "u1"), ("flags", "u1"),
        ("last_blocks", "u1"), ("last_lines", "u1"), ("last_cm", "u1"), ("pad", "u1", (2,)),
    ],
    align=True,
)
assert INFO_DTYPE.itemsize == L.INFO_BYTES


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    if device.type == "cpu":
        return None
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def resolve_device(device=None) -> torch.device:
    if device is not None and torch.device(device).type == "cpu":  # the host backend, asked for by name
        return torch.device("cpu")
    if not torch.cuda.is_available():
        raise L.BBNativeError("no GPU visible to torch: the Block Blast env runs only on the HIP device")
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device)
    if d.type != "cuda":
        raise L.BBNativeError(f"Block Blast env needs a cuda (HIP) device, got {d}")
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


def seeds_to_arrays(seeds: Sequence[Optional[int]]):
    """Per-env seeds (int or None) -> (seed u64, has_seed u8, raw u64[N,4])."""
    n = len(seeds)
    s = np.zeros(n, dtype=np.uint64)
    has = np.zeros(n, dtype=np.uint8)
    raw = np.zeros((n, 4), dtype=np.uint64)
    need_entropy = []
    for i, sd in enumerate(seeds):
        if sd is None:
            need_entropy.append(i)
            continue
        sd = int(sd)
        if sd < 0:
            raise ValueError("expected non-negative integer seed (numpy SeedSequence semantics)")
        if sd < 2 ** 64:
            s[i] = sd
            has[i] = 1
        else:  # does not fit the C-ABI's uint64: let numpy's SeedSequence do it
            st = np.random.PCG64(sd).state["state"]
            raw[i] = [st["state"] >> 64, st["state"] & (2 ** 64 - 1), st["inc"] >> 64, st["inc"] & (2 ** 64 - 1)]
            has[i] = 2
    if need_entropy:  # seed_value None: fresh OS entropy, stream continues across resets
        ent = np.random.default_rng().integers(0, 2 ** 63, size=(len(need_entropy), 4), dtype=np.int64)
        raw[need_entropy] = ent.astype(np.uint64)
    return s, has, raw


class DeviceEnvBatch:
    """``num_envs`` Block Blast games stepped in lockstep by ``bb_step``."""

    def __init__(
        self,
        num_envs: int,
        seeds: Optional[Sequence[Optional[int]]] = None,
        reward_config: Optional[dict] = None,
        autoreset: bool = True,
        device=None,
        env_offset: int = 0,
    ):
        self.device = resolve_device(device)
        self.lib = L.load_host() if self.device.type == "cpu" else L.load()
        self.num_envs = int(num_envs)
        self.env_offset = int(env_offset)
        rw = dict(DEFAULT_REWARDS)
        if reward_config:
            rw.update(reward_config)
        self.reward_config = rw
        h = C.c_void_p()
        L.check(
            self.lib.bb_create(self.num_envs, self.device.index or 0, C.byref(L.reward_cfg(rw)), int(bool(autoreset)),
                               C.byref(h)),
            "bb_create", lib=self.lib,
        )
        self.handle = h
        dev = self.device
        n = self.num_envs
        self.reward = torch.zeros(n, dtype=torch.float32, device=dev)
        self.terminated = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.reward_f64 = torch.zeros(n, dtype=torch.float64, device=dev)
        self.lines = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.info = torch.zeros(n * L.INFO_BYTES, dtype=torch.uint8, device=dev)
        self._out = L.StepOut()
        self.seed(seeds if seeds is not None else [None] * n)

    # ------------------------------------------------------------------ seeding
    def seed(self, seeds: Sequence[Optional[int]]) -> None:
        if len(seeds) != self.num_envs:
            raise ValueError("one seed (or None) per env expected")
        s, has, raw = seeds_to_arrays(seeds)
        L.check(
            self.lib.bb_seed(self.handle, s.ctypes.data_as(C.c_void_p), has.ctypes.data_as(C.c_void_p),
                             raw.ctypes.data_as(C.c_void_p)),
            "bb_seed", self.handle, self.lib,
        )

    # --------------------------------------------------------------- hot path
    def reset(self, env_mask: Optional[torch.Tensor] = None) -> None:
        L.check(self.lib.bb_reset(self.handle, _ptr(env_mask), _stream(self.device)), "bb_reset", self.handle, self.lib)

    def step(
        self,
        actions: torch.Tensor,
        want_info: bool = False,
        want_f64: bool = False,
        want_lines: bool = False,
        next_action: Optional[torch.Tensor] = None,
        policy_seed: int = 0xB10C,
        policy_step: int = 0,
        mask_out: Optional[torch.Tensor] = None,
        final_score: Optional[torch.Tensor] = None,
        final_moves: Optional[torch.Tensor] = None,
    ) -> None:
        """actions: int32 [N] on this device.  Outputs land in self.reward /
        self.terminated (+ reward_f64 / lines / info when requested).
        final_score (int64 [N]) / final_moves (int32 [N]) receive the score and
        moves of the envs that terminated (info['final_score'] / info['moves'])
        and are left untouched elsewhere."""
        assert actions.dtype == torch.int32 and actions.device == self.device and actions.numel() == self.num_envs
        for t, dt in ((final_score, torch.int64), (final_moves, torch.int32)):
            assert t is None or (t.dtype == dt and t.device == self.device and t.is_contiguous() and t.numel() == self.num_envs)
        o = self._out
        o.reward = self.reward.data_ptr()
        o.terminated = self.terminated.data_ptr()
        o.reward_f64 = self.reward_f64.data_ptr() if want_f64 else None
        o.mask = mask_out.data_ptr() if mask_out is not None else None
        o.lines = self.lines.data_ptr() if want_lines else None
        o.info = self.info.data_ptr() if want_info else None
        o.next_action = next_action.data_ptr() if next_action is not None else None
        o.policy_seed = policy_seed
        o.policy_step = policy_step
        o.env_offset = self.env_offset
        o.final_score = final_score.data_ptr() if final_score is not None else None
        o.final_moves = final_moves.data_ptr() if final_moves is not None else None
        L.check(self.lib.bb_step(self.handle, _ptr(actions), C.byref(o), _stream(self.device)), "bb_step",
                self.handle, self.lib)

    def rollout(
        self,
        steps: int,
        actions: torch.Tensor,
        reward: torch.Tensor,
        terminated: torch.Tensor,
        lines: Optional[torch.Tensor] = None,
        actions_out: Optional[torch.Tensor] = None,
        mask_out: Optional[torch.Tensor] = None,
        next_action: Optional[torch.Tensor] = None,
        policy_seed: int = 0xB10C,
        policy_step0: int = 0,
    ) -> None:
        """``steps`` fused steps under the synthetic random policy (bb_rollout).
        actions: int32 [N], the action of the first step; reward f32 / terminated
        u8 / lines u8 / actions_out i32 are [steps, N], mask_out i64 [steps, N, 3].
        Equals ``steps`` chained ``step(..., next_action=, policy_step=policy_step0+t+1)``."""
        n = self.num_envs
        assert actions.dtype == torch.int32 and actions.device == self.device and actions.numel() == n
        assert reward.dtype == torch.float32 and reward.numel() >= steps * n
        assert terminated.dtype == torch.uint8 and terminated.numel() >= steps * n
        for t, dt, per in ((lines, torch.uint8, 1), (actions_out, torch.int32, 1), (mask_out, torch.int64, 3),
                           (next_action, torch.int32, 0)):
            if t is not None:
                assert t.dtype == dt and t.device == self.device and t.numel() >= (steps * n * per if per else n)
        o = L.RolloutOut(reward=reward.data_ptr(), terminated=terminated.data_ptr(),
                         lines=lines.data_ptr() if lines is not None else None,
                         actions=actions_out.data_ptr() if actions_out is not None else None,
                         mask=mask_out.data_ptr() if mask_out is not None else None,
                         next_action=next_action.data_ptr() if next_action is not None else None,
                         policy_seed=policy_seed, policy_step0=policy_step0, env_offset=self.env_offset)
        L.check(self.lib.bb_rollout(self.handle, int(steps), _ptr(actions), C.byref(o), _stream(self.device)),
                "bb_rollout", self.handle, self.lib)

    def sync(self) -> None:
        """Wait for this handle's launches on the current stream and raise BBNativeError if a kernel reported
        a device-side failure (bb_sync; e.g. a rollout wave that hit its iteration cap)."""
        L.check(self.lib.bb_sync(self.handle, _stream(self.device)), "bb_sync", self.handle, self.lib)

    def obs(self, x=None, mask_i8=None, mask_f32=None, mask_bits=None) -> None:
        L.check(
            self.lib.bb_obs(self.handle, _ptr(x), _ptr(mask_i8), _ptr(mask_f32), _ptr(mask_bits),
                            _stream(self.device)),
            "bb_obs", self.handle, self.lib,
        )

    def snapshot(self, board=None, hand=None, mask_bits=None) -> None:
        L.check(
            self.lib.bb_snapshot(self.handle, _ptr(board), _ptr(hand), _ptr(mask_bits), _stream(self.device)),
            "bb_snapshot", self.handle, self.lib,
        )

    def random_actions(self, mask_bits: torch.Tensor, out: torch.Tensor, seed: int = 0xB10C, step: int = 0):
        L.check(
            self.lib.bb_random_actions(_ptr(mask_bits), self.num_envs, seed, step, self.env_offset, _ptr(out),
                                       _stream(self.device)),
            "bb_random_actions", None, self.lib,
        )

    # ------------------------------------------------------------ host copies
    def state(self) -> dict:
        n = self.num_envs
        out = {
            "board": np.zeros(n, np.uint64), "hand": np.zeros(n, np.uint32), "score": np.zeros(n, np.int64),
            "combo": np.zeros(n, np.int32), "max_combo": np.zeros(n, np.int32), "moves": np.zeros(n, np.int32),
            "lines": np.zeros(n, np.int32), "blocks": np.zeros(n, np.int32), "prev_holes": np.zeros(n, np.uint8),
            "prev_center": np.zeros(n, np.uint8), "rng": np.zeros((n, 3), np.uint64),
        }
        v = L.StateView(**{k: a.ctypes.data for k, a in out.items()})
        L.check(self.lib.bb_get_state(self.handle, C.byref(v)), "bb_get_state", self.handle, self.lib)
        return out

    def set_state(self, **arrays) -> None:
        dt = {"board": np.uint64, "hand": np.uint32, "score": np.int64, "combo": np.int32, "max_combo": np.int32,
              "moves": np.int32, "lines": np.int32, "blocks": np.int32, "prev_holes": np.uint8,
              "prev_center": np.uint8, "rng": np.uint64}
        keep = {}
        kw = {}
        for k, a in arrays.items():
            arr = np.ascontiguousarray(a, dtype=dt[k])
            keep[k] = arr
            kw[k] = arr.ctypes.data
        v = L.StateView(**kw)
        L.check(self.lib.bb_set_state(self.handle, C.byref(v)), "bb_set_state", self.handle, self.lib)

    def info_host(self) -> np.ndarray:
        return self.info.cpu().numpy().view(INFO_DTYPE)

    def close(self) -> None:
        if getattr(self, "handle", None):
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self.lib.bb_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
