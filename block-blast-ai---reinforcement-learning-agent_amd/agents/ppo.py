"""Masked PPO on the MI355X: rollout buffers in HBM, fused HIP rollout kernels,
PyTorch-ROCm CNN update, RCCL gradient all-reduce for data parallelism.

Drop-in for the reference ``src/agents/ppo.py`` (PPOConfig 26-67,
RolloutBuffer 70-218, PPOAgent 221-449): same class names, constructor
arguments, method names, return types and checkpoint format.  What changes is
where the work runs:

* ``RolloutBuffer`` keeps the reference's float32 layout but lives on the
  device; GAE is the ``bb_gae`` kernel (numpy float32 op order, bit-exact).
* ``PackedRolloutBuffer`` stores ~60 B per env-step instead of ~1.8 KiB (board
  bits, hand word, mask bits, ...) and expands minibatches with ``bb_gather_obs``.
* action sampling / log-prob / masked entropy on the rollout path is the fused
  ``bb_masked_sample`` kernel (Philox uniforms instead of torch.multinomial).
* the update is the reference loss (network.py:210-262, ppo.py:362-401); under
  torch.distributed every optimizer step all-reduces ONE flat gradient buffer
  (the parameters' .grad are views into it) and advantage moments are global.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, Callable, Dict, Iterator, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from models.network import BlockBlastNetwork, masked_entropy
from runtime import kernels as K
from runtime import lib as L

from .base import BaseAgent

_EPS32 = float(torch.finfo(torch.float32).eps)  # Categorical clamp_probs
FUSED_ADAM = os.environ.get("BB_FUSED_ADAM", "1") != "0"  # clip_grad_norm_ + Adam on bb_adam_clip_step (GPU)
DP_OVERLAP_MODES = ("graph-segments", "graph-split", "capture")  # PPOAgent.dp_overlap


@dataclass
class PPOConfig:
    """ppo.py:26-67."""
    learning_rate: float = 3e-4
    gamma: float = 0.99
    gae_lambda: float = 0.95
    clip_epsilon: float = 0.2
    entropy_coef: float = 0.01
    value_coef: float = 0.5
    max_grad_norm: float = 0.5
    num_epochs: int = 10
    batch_size: int = 64
    conv_channels: Tuple[int, ...] = (64, 128, 128)
    fc_hidden: Tuple[int, ...] = (512, 256)

    def to_dict(self) -> Dict[str, Any]:
        return {
            "learning_rate": self.learning_rate, "gamma": self.gamma, "gae_lambda": self.gae_lambda,
            "clip_epsilon": self.clip_epsilon, "entropy_coef": self.entropy_coef, "value_coef": self.value_coef,
            "max_grad_norm": self.max_grad_norm, "num_epochs": self.num_epochs, "batch_size": self.batch_size,
            "conv_channels": self.conv_channels, "fc_hidden": self.fc_hidden,
        }

    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "PPOConfig":
        return cls(**{k: v for k, v in data.items() if k in cls.__dataclass_fields__})


# bench.py's dp_update leg only: a rank's local agent timed without the collective (None: the process group's)
_WORLD_OVERRIDE: Optional[int] = None


def _world() -> int:
    if _WORLD_OVERRIDE is not None:
        return _WORLD_OVERRIDE
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _as_tensor(x, device, dtype) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype, non_blocking=True)
    return torch.as_tensor(np.asarray(x), dtype=dtype).to(device, non_blocking=True)


def _global_moments(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Mean / population std (np.std, ddof 0) over every rank's samples."""
    if _world() == 1:
        return x.mean(), x.std(unbiased=False)
    s = torch.stack([x.double().sum(), (x.double() ** 2).sum(), torch.tensor(float(x.numel()), device=x.device,
                                                                               dtype=torch.float64)])
    dist.all_reduce(s)
    mean = s[0] / s[2]
    var = (s[1] / s[2] - mean * mean).clamp(min=0.0)
    return mean.float(), var.sqrt().float()


class RolloutBuffer:
    """ppo.py:70-218 with device storage (float32 layout of the reference)."""

    def __init__(self, buffer_size: int, num_envs: int, board_size: int = 8, num_pieces: int = 3,
                 action_space_size: int = 192, device: torch.device = torch.device("cpu")):
        self.buffer_size = buffer_size
        self.num_envs = num_envs
        self.device = torch.device(device)
        d, T, N = self.device, buffer_size, num_envs
        z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=d)  # noqa: E731
        self.boards = z(T, N, board_size, board_size)
        self.pieces = z(T, N, num_pieces, board_size, board_size)
        self.action_masks = z(T, N, action_space_size)
        self.actions = z(T, N, dt=torch.int64)
        self.log_probs = z(T, N)
        self.rewards = z(T, N)
        self.dones = z(T, N)
        self.values = z(T, N)
        self.advantages = z(T, N)
        self.returns = z(T, N)
        self.ptr = 0
        self.full = False
        # minibatch order per epoch: None = numpy's global permutation, as the reference (ppo.py:199);
        # or a callable total -> index array (tests inject the same order on both sides)
        self.permutation: Optional[Callable[[int], Any]] = None

    def add(self, board, pieces, action_mask, action, log_prob, reward, done, value) -> None:
        d, t = self.device, self.ptr
        self.boards[t] = _as_tensor(board, d, torch.float32)
        self.pieces[t] = _as_tensor(pieces, d, torch.float32)
        self.action_masks[t] = _as_tensor(action_mask, d, torch.float32)
        self.actions[t] = _as_tensor(action, d, torch.int64)
        self.log_probs[t] = _as_tensor(log_prob, d, torch.float32)
        self.rewards[t] = _as_tensor(reward, d, torch.float32)
        self.dones[t] = _as_tensor(done, d, torch.float32)
        self.values[t] = _as_tensor(value, d, torch.float32)
        self.ptr += 1
        if self.ptr >= self.buffer_size:
            self.full = True

    def _gpu(self) -> torch.device:
        return self.device if self.device.type == "cuda" else torch.device("cuda", 0)

    def compute_returns_and_advantages(self, last_values, gamma: float, gae_lambda: float) -> None:
        """ppo.py:141-169 as the bb_gae kernel."""
        g = self._gpu()
        adv, ret = K.gae(self.rewards.to(g), self.values.to(g), self.dones.to(g),
                         _as_tensor(last_values, g, torch.float32), gamma, gae_lambda)
        self.advantages = adv.to(self.device)
        self.returns = ret.to(self.device)

    def normalized_advantages(self) -> torch.Tensor:
        """ppo.py:196 over the flattened advantages (moments over every rank)."""
        adv = self.advantages.reshape(-1)
        mean, std = _global_moments(adv)
        return (adv - mean) / (std + 1e-8)

    def get_samples(self, batch_size: int) -> Iterator[Tuple[torch.Tensor, ...]]:
        """ppo.py:171-213: flatten, normalise advantages (ppo.py:196), random
        minibatches from numpy's global permutation (ppo.py:199)."""
        total = self.buffer_size * self.num_envs
        boards = self.boards.reshape(total, *self.boards.shape[2:])
        pieces = self.pieces.reshape(total, *self.pieces.shape[2:])
        masks = self.action_masks.reshape(total, -1)
        actions = self.actions.reshape(total)
        log_probs = self.log_probs.reshape(total)
        returns = self.returns.reshape(total)
        adv = self.normalized_advantages()
        perm = np.random.permutation(total) if self.permutation is None else self.permutation(total)
        idx = torch.as_tensor(np.asarray(perm) if not torch.is_tensor(perm) else perm,
                              dtype=torch.int64).to(self.device)
        for start in range(0, total, batch_size):
            b = idx[start:start + batch_size]
            yield (boards[b], pieces[b], masks[b], actions[b], log_probs[b], adv[b], returns[b])

    def reset(self) -> None:
        self.ptr = 0
        self.full = False


class PackedRolloutBuffer:
    """Device rollout storage in the env's packed format (~60 B / env-step):
    board bits, hand word, mask bits, action, log-prob, reward, done, value.
    Minibatch observations are expanded on the fly by ``bb_gather_obs``."""

    def __init__(self, buffer_size: int, num_envs: int, device: torch.device):
        self.buffer_size, self.num_envs = buffer_size, num_envs
        self.device = torch.device(device)
        T, N, d = buffer_size, num_envs, self.device
        self.board = torch.zeros((T, N), dtype=torch.int64, device=d)
        self.hand = torch.zeros((T, N), dtype=torch.int32, device=d)
        self.mask_bits = torch.zeros((T, N, 3), dtype=torch.int64, device=d)
        self.actions = torch.zeros((T, N), dtype=torch.int64, device=d)
        self.log_probs = torch.zeros((T, N), dtype=torch.float32, device=d)
        self.rewards = torch.zeros((T, N), dtype=torch.float32, device=d)
        self.dones = torch.zeros((T, N), dtype=torch.float32, device=d)
        self.values = torch.zeros((T, N), dtype=torch.float32, device=d)
        self.advantages = torch.zeros((T, N), dtype=torch.float32, device=d)
        self.returns = torch.zeros((T, N), dtype=torch.float32, device=d)
        self.ptr = 0
        self.full = False
        # minibatch order per epoch: None = torch.randperm on the device (no host round trip);
        # "numpy" = np.random.permutation like the reference (ppo.py:199); or a callable total -> indices
        self.permutation: Optional[Any] = None

    def reset(self) -> None:
        self.ptr = 0
        self.full = False

    def normalized_advantages(self) -> torch.Tensor:
        """ppo.py:196 over the flattened advantages (moments over every rank)."""
        adv = self.advantages.reshape(-1)
        mean, std = _global_moments(adv)
        return (adv - mean) / (std + 1e-8)

    def _permutation(self, total: int, generator: Optional[torch.Generator]) -> torch.Tensor:
        if self.permutation is None:
            return torch.randperm(total, device=self.device, generator=generator)
        perm = np.random.permutation(total) if self.permutation == "numpy" else self.permutation(total)
        if not torch.is_tensor(perm):
            perm = torch.from_numpy(np.ascontiguousarray(perm, dtype=np.int64))
        return perm.to(self.device, torch.int64)

    def advance(self) -> None:
        self.ptr += 1
        self.full = self.ptr >= self.buffer_size

    def compute_returns_and_advantages(self, last_values: torch.Tensor, gamma: float, gae_lambda: float) -> None:
        K.gae(self.rewards, self.values, self.dones, last_values.float(), gamma, gae_lambda,
              adv=self.advantages, ret=self.returns)

    def get_minibatches(self, batch_size: int, generator: Optional[torch.Generator] = None, out=None):
        """Yields (x (B,4,8,8), mask f32 (B,192), actions, old log-probs,
        normalised advantages, returns) in a random order.  ``out(B)`` may
        return 6 tensors to gather into (a captured optimizer step's inputs,
        PPOAgent.minibatch_inputs), or None."""
        total = self.buffer_size * self.num_envs
        adv = self.normalized_advantages()
        perm = self._permutation(total, generator)
        board, hand, mb = self.board.reshape(total), self.hand.reshape(total), self.mask_bits.reshape(total, 3)
        actions, logp, ret = self.actions.reshape(total), self.log_probs.reshape(total), self.returns.reshape(total)
        for start in range(0, total, batch_size):
            b = perm[start:start + batch_size]
            dst = out(b.numel()) if out is not None else None
            if dst is not None:  # straight into the step's input buffers: no copies before the replay
                K.gather_obs(board, hand, mb, b, out_x=dst[0], out_mask=dst[1])
                for src, o in zip((actions, logp, adv, ret), dst[2:]):
                    torch.index_select(src, 0, b, out=o)
                yield tuple(dst)
                continue
            x, mf = K.gather_obs(board, hand, mb, b)
            yield x, mf, actions[b], logp[b], adv[b], ret[b]


def categorical_log_prob(probs: torch.Tensor, action: torch.Tensor) -> torch.Tensor:
    """Categorical(probs).log_prob(action) without the validation sync:
    log(clamp(p / sum p, eps, 1 - eps))[action] (torch clamp_probs)."""
    p = probs / probs.sum(dim=-1, keepdim=True)
    return torch.log(p.clamp(min=_EPS32, max=1.0 - _EPS32)).gather(-1, action.unsqueeze(-1)).squeeze(-1)


def ppo_loss_torch(logits, values, masks, actions, old_log_probs, advantages, returns, cfg: "PPOConfig"):
    """ppo.py:362-392 on torch ops: the CPU path and the parity reference of
    the fused bb_ppo_loss kernels.  Returns (loss, 6 detached statistics)."""
    masked = logits + torch.where(masks.bool(), torch.zeros_like(logits), torch.full_like(logits, float("-inf")))
    probs = F.softmax(masked, dim=-1)
    new_log_probs = categorical_log_prob(probs, actions)
    entropy = masked_entropy(probs, masks)
    ratio = torch.exp(new_log_probs - old_log_probs)
    surr1 = ratio * advantages
    surr2 = torch.clamp(ratio, 1 - cfg.clip_epsilon, 1 + cfg.clip_epsilon) * advantages
    policy_loss = -torch.min(surr1, surr2).mean()
    value_loss = F.mse_loss(values, returns)
    entropy_loss = -entropy.mean()
    loss = policy_loss + cfg.value_coef * value_loss + cfg.entropy_coef * entropy_loss
    with torch.no_grad():
        approx_kl = ((ratio - 1) - torch.log(ratio)).mean()
        clip_fraction = ((ratio - 1).abs() > cfg.clip_epsilon).float().mean()
        stats = torch.stack([policy_loss, value_loss, entropy.mean(), loss, approx_kl, clip_fraction]).detach()
    return loss, stats


class PPOAgent(BaseAgent):
    """ppo.py:221-449."""

    def __init__(self, config: Optional[PPOConfig] = None, device: Optional[torch.device] = None,
                 sample_seed: Optional[int] = None):
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        super().__init__(torch.device(device))
        self.config = config or PPOConfig()
        self.network = BlockBlastNetwork(conv_channels=self.config.conv_channels,
                                         fc_hidden=self.config.fc_hidden).to(self.device)
        # On the GPU: capturable (the step count lives on the device, so the
        # whole optimizer step can be replayed from a HIP graph, see
        # train_minibatch) and fused (one multi-tensor kernel; the capturable
        # foreach path divides every tensor by a 0-dim bias correction in a
        # separate strided kernel, 86 launches per step)
        on_gpu = self.device.type == "cuda"
        # conv-stack activations NHWC on the GPU (set_channels_last): no NCHW<->NHWC
        # transposes around MIOpen's implicit-GEMM convolutions
        self.channels_last = False
        if on_gpu:
            self.network.to(memory_format=torch.channels_last)
            self.channels_last = True
        self.optimizer = torch.optim.Adam(self.network.parameters(), lr=self.config.learning_rate, eps=1e-5,
                                          capturable=on_gpu, fused=True if on_gpu else None)
        self.scheduler = None
        # Philox key for rollout sampling (derived from torch's seeded RNG)
        self.sample_seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if sample_seed is None else int(sample_seed)
        self.sample_step = 0
        self._flat_grad = None
        # data parallelism (world > 1), dp_overlap (DP_OVERLAP_MODES):
        #  "graph-segments" (default): backward in two segments cut at the conv stack's output, each its own HIP
        #    graph: heads + FC backward (graph A1, ~85% of the gradient floats), then the all-reduce of that
        #    bucket is issued and runs on RCCL's stream while the conv-stack backward (graph A2, ~85% of the
        #    backward FLOPs) replays; then the conv bucket's all-reduce; then average + clip + Adam (graph B);
        #  "graph-split": one forward + backward graph, one all-reduce of the whole buffer after it (exposed);
        #  "capture": the bucketed collectives issued by post-accumulate-grad hooks (buckets of about
        #    dp_bucket_floats, from the end of the buffer) captured inside one graph per step (nccl = RCCL only)
        # Eager steps (no graphs) use the same segments in "graph-segments" mode and the hooks otherwise.
        self.dp_bucket_floats = 1 << 21
        self.dp_overlap = "graph-segments"
        self._seg = None  # (conv-stack output, its detached leaf) of the last segmented forward
        self._loss_seed: Optional[torch.Tensor] = None  # _backward_loss
        self._dp_hooks = None
        self._dp_hooks_on = True  # off while a graph without collectives is captured
        self._dp_works: List[Any] = []
        # bumped whenever parameter storage, layout or precision changes: captured graphs of the
        # optimizer step (here) and of the rollout (training.trainer.DeviceRollout) are then stale
        self.graph_epoch = 0
        self._autocast_dtype: Optional[torch.dtype] = None  # e.g. torch.bfloat16 for the CNN
        # one optimizer step per minibatch replayed from HIP graphs (CUDA device): one graph on one
        # rank; with data parallelism forward + backward, then the RCCL all-reduce, then clip + Adam
        self.use_graphs = self.device.type == "cuda"
        self._graphs = {}
        self.fused_loss = True  # the minibatch loss on bb_ppo_loss_* (GPU tensors only)
        # bb_adam_clip_step scratch per parameter-size set; never dropped, since captured optimizer
        # steps hold the workspace's address
        self._adam_ws: Dict[Tuple[int, ...], torch.Tensor] = {}
        self._adam_tables: Dict[Tuple[int, ...], Any] = {}  # key -> (params, gradient addresses) last stepped
        # update(): keep every minibatch's 6 statistics (device tensors) in minibatch_stats (parity tests)
        self.record_minibatch_stats = False
        self.minibatch_stats: List[torch.Tensor] = []
        # update(): called as f(index, stats) after every optimizer step (logging, parity tests)
        self.minibatch_callback: Optional[Callable[[int, torch.Tensor], None]] = None

    @property
    def autocast_dtype(self) -> Optional[torch.dtype]:
        return self._autocast_dtype

    @autocast_dtype.setter
    def autocast_dtype(self, dt: Optional[torch.dtype]) -> None:
        if dt != self._autocast_dtype:
            self.graph_epoch += 1
        self._autocast_dtype = dt

    # ------------------------------------------------------------ helpers
    def set_channels_last(self, on: bool = True) -> None:
        """Keep the conv stack's activations NHWC (torch.channels_last): MIOpen's
        implicit-GEMM convolutions are NHWC kernels, so NCHW tensors are
        transposed around every convolution; the BatchNorm kernels take both."""
        self.channels_last = bool(on)
        self.network.to(memory_format=torch.channels_last if on else torch.contiguous_format)
        self._graphs = {}
        self.graph_epoch += 1
        self._flat_grad = None  # gradient views must follow the parameters' strides
        self._remove_dp_hooks()

    def _raw(self, x: torch.Tensor, keep_dtype: bool = False):
        """(logits, value) of the network; under autocast cast to f32 unless keep_dtype (the fused loss reads
        the bf16 outputs as they are: bb_ppo_loss_forward_bf16)."""
        bf16_in = self.autocast_dtype == torch.bfloat16 and K.CONV_IN  # the input layer reads either layout
        if self.channels_last and x.is_cuda and not bf16_in:
            x = x.contiguous(memory_format=torch.channels_last)
        if self.autocast_dtype is not None and x.is_cuda:
            with torch.autocast("cuda", dtype=self.autocast_dtype, cache_enabled=False):
                logits, value = self.network.raw(x)
            return (logits, value) if keep_dtype else (logits.float(), value.float())
        return self.network.raw(x)

    def _obs_to_device(self, obs: Dict[str, Any]):
        board = _as_tensor(obs["board"], self.device, torch.float32)
        pieces = _as_tensor(obs["pieces"], self.device, torch.float32)
        return BlockBlastNetwork.stack_input(board, pieces)

    def _sample(self, logits: torch.Tensor, mask: torch.Tensor, deterministic: bool, env_offset: int = 0,
                want_entropy: bool = False):
        if not logits.is_cuda:
            raise RuntimeError("PPOAgent rollout sampling runs on the HIP device (no CPU fallback)")
        mb = K.pack_mask(mask)
        step = self.sample_step
        self.sample_step += 1
        return K.masked_sample(logits, mb, seed=self.sample_seed, step=step, env_offset=env_offset,
                               deterministic=deterministic, want_entropy=want_entropy)

    # ------------------------------------------------- reference interface
    def select_action(self, observation: Dict[str, np.ndarray], deterministic: bool = False):
        """ppo.py:261-289."""
        with torch.no_grad():
            x = self._obs_to_device({k: np.asarray(v)[None] for k, v in observation.items()})
            mask = _as_tensor(np.asarray(observation["action_mask"])[None], self.device, torch.float32)
            logits, value = self._raw(x)
            a, lp, ent = self._sample(logits, mask, deterministic, want_entropy=True)
            return int(a.item()), {"log_prob": float(lp.item()), "entropy": float(ent.item()),
                                   "value": float(value.item())}

    def select_actions(self, observations: Dict[str, np.ndarray], deterministic: bool = False):
        """ppo.py:291-319 (numpy in, numpy out)."""
        with torch.no_grad():
            x = self._obs_to_device(observations)
            mask = _as_tensor(observations["action_mask"], self.device, torch.float32)
            logits, value = self._raw(x)
            a, lp, _ = self._sample(logits, mask, deterministic)
            return a.cpu().numpy(), lp.cpu().numpy(), value.cpu().numpy()

    def get_values(self, observations: Dict[str, np.ndarray]) -> np.ndarray:
        """ppo.py:321-328."""
        with torch.no_grad():
            return self._raw(self._obs_to_device(observations))[1].cpu().numpy()

    # ------------------------------------------------------ device fast path
    def act_device(self, x: torch.Tensor, mask_bits: torch.Tensor, env_offset: int = 0,
                   deterministic: bool = False, step_base: Optional[torch.Tensor] = None, step_add: int = 0):
        """Rollout step on device tensors: (action int64, log-prob, value).
        With ``step_base`` (graph capture) the sampling step is
        ``step_base[0] + step_add`` read on the device, and ``sample_step`` is
        left to the caller (who advances both between replays)."""
        with torch.no_grad():
            logits, value = self._raw(x)
            if step_base is not None:
                a, lp, _ = K.masked_sample(logits, mask_bits, seed=self.sample_seed, step=step_add,
                                           env_offset=env_offset, deterministic=deterministic, want_entropy=False,
                                           step_base=step_base)
                return a, lp, value
            step = self.sample_step
            self.sample_step += 1
            a, lp, _ = K.masked_sample(logits, mask_bits, seed=self.sample_seed, step=step, env_offset=env_offset,
                                       deterministic=deterministic, want_entropy=False)
            return a, lp, value

    def values_device(self, x: torch.Tensor) -> torch.Tensor:
        with torch.no_grad():
            return self._raw(x)[1]

    # ------------------------------------------------------------- update
    def _grad_buffer(self) -> torch.Tensor:
        """Flat fp32 gradient buffer for data-parallel runs; every parameter's
        .grad is a view into it (same strides as the parameter, 256-byte
        aligned so the accumulating adds stay vectorised), so the all-reduce
        covers the whole model (5,290,113 floats plus alignment padding) in a
        few contiguous buckets (_dp_buckets)."""
        if self._flat_grad is None:
            params = [p for p in self.network.parameters() if p.requires_grad]
            offs, n = [], 0
            for p in params:
                offs.append(n)
                n += -(-p.numel() // 64) * 64
            self._flat_grad = torch.zeros(n, dtype=torch.float32, device=self.device)
            for p, off in zip(params, offs):
                p.grad = torch.as_strided(self._flat_grad, p.size(), p.stride(), off)
            self._flat_layout = [(p, off, -(-p.numel() // 64) * 64) for p, off in zip(params, offs)]
            self._remove_dp_hooks()  # the buckets are ranges of this buffer
        return self._flat_grad

    def _remove_dp_hooks(self) -> None:
        if self._dp_hooks is not None:
            for h in self._dp_hooks[0]:
                h.remove()
        self._dp_hooks = None

    def _dp_buckets(self):
        """Post-accumulate-grad hooks that all-reduce the flat gradient buffer in contiguous buckets.  Backward
        produces the gradients roughly in reverse parameter order, so the buckets are taken from the end of the
        buffer; a bucket's all-reduce is issued (async_op) once all of its parameters have accumulated, and
        ``_dp_finish`` waits for them (a bucket that never completed is issued there)."""
        flat = self._grad_buffer()
        if self._dp_hooks is not None:
            return self._dp_hooks
        layout = self._flat_layout
        buckets, cur, size = [], [], 0
        for p, off, n in reversed(layout):
            cur.append((p, off, n))
            size += n
            if size >= self.dp_bucket_floats:
                buckets.append(cur)
                cur, size = [], 0
        if cur:
            buckets.append(cur)
        state = []  # per bucket: [lo, hi, remaining, total, launched]
        owner = {}
        for b, items in enumerate(buckets):
            lo = min(off for _, off, _ in items)
            hi = max(off + n for _, off, n in items)
            state.append([lo, hi, len(items), len(items), False])
            for p, _, _ in items:
                owner[p] = b

        def make_hook(b):
            def hook(_p):
                if not self._dp_hooks_on:
                    return
                st = state[b]
                st[2] -= 1
                if st[2] == 0 and not st[4]:
                    st[4] = True
                    self._dp_works.append(dist.all_reduce(flat[st[0]:st[1]], async_op=True))
            return hook

        handles = [p.register_post_accumulate_grad_hook(make_hook(owner[p])) for p, _, _ in layout]
        self._dp_hooks = (handles, state)
        return self._dp_hooks

    def _dp_arm(self) -> None:
        """Before a backward pass: every bucket waits for all of its gradients again."""
        for st in self._dp_buckets()[1]:
            st[2], st[4] = st[3], False
        self._dp_works = []

    def _dp_finish(self, world: int) -> None:
        """After backward: issue the buckets whose hooks did not all fire, wait for every bucket's all-reduce
        (the current stream waits on RCCL's; the host does not block), then average."""
        flat = self._flat_grad
        for st in self._dp_hooks[1]:
            if not st[4]:
                st[4] = True
                self._dp_works.append(dist.all_reduce(flat[st[0]:st[1]], async_op=True))
        for w in self._dp_works:
            w.wait()
        self._dp_works = []
        flat.div_(world)

    def _segmented(self) -> bool:
        """The data-parallel step runs backward in two segments (dp_overlap "graph-segments")."""
        return _world() > 1 and self.dp_overlap == "graph-segments" and torch.is_grad_enabled()

    def _dp_split_offset(self) -> int:
        """Flat-buffer offset where the conv stack's gradients end (they come first: parameter order)."""
        conv = {id(p) for p in self.network.conv_encoder.parameters()}
        lay = self._flat_layout
        split = min(off for p, off, _ in lay if id(p) not in conv)
        if any(off >= split for p, off, _ in lay if id(p) in conv):
            raise RuntimeError("conv-stack gradients are not a prefix of the flat buffer")
        return split

    def _minibatch_loss(self, x, masks, actions, old_log_probs, advantages, returns):
        """(loss, stats) of one minibatch.  In the segmented data-parallel mode the forward is cut at the conv
        stack's output (self._seg): that loss must go through _optimizer_step, whose backward runs both
        segments; a bare loss.backward() would stop at the cut."""
        cfg = self.config
        keep = self.fused_loss and x.is_cuda
        if self._segmented():
            self.network.grad_split = []
            try:
                logits, values = self._raw(x, keep)
            finally:
                cut, self.network.grad_split = self.network.grad_split, None
            self._seg = cut[0] if len(cut) == 1 else None
        else:
            logits, values = self._raw(x, keep)
        if self.fused_loss and logits.is_cuda:  # bb_ppo_loss_fused (bb_ppo_loss_forward / _backward otherwise)
            seed = self._seed(logits.device) if torch.is_grad_enabled() and logits.requires_grad else None
            return K.PPOLossFunction.apply(logits, values, masks, actions, old_log_probs, advantages, returns,
                                           cfg.clip_epsilon, cfg.value_coef, cfg.entropy_coef, seed)
        return ppo_loss_torch(logits, values, masks, actions, old_log_probs, advantages, returns, cfg)

    def _seed(self, device: torch.device) -> torch.Tensor:
        """The persistent 1.0 every minibatch loss is backpropagated with (f32, made by the first eager step,
        before any capture).  The fused loss receives it up front (bb_ppo_loss_fused: forward and backward in one
        launch) and hands its gradients over when autograd passes this very tensor back."""
        seed = self._loss_seed
        if seed is None or seed.device != torch.device(device):
            seed = self._loss_seed = torch.ones((), dtype=torch.float32, device=device)
        return seed

    def _backward_loss(self, loss: torch.Tensor) -> None:
        """loss.backward() seeded with the persistent 1.0 (loss.backward() fills a fresh one: one more kernel in
        every graph replay)."""
        seed = self._seed(loss.device)
        if seed.dtype != loss.dtype:
            seed = seed.to(loss.dtype)
        loss.backward(seed)

    def _backward_segments(self, loss: torch.Tensor, world: int) -> None:
        """Segmented data-parallel backward: heads + FC, their bucket's all-reduce issued (async), the conv
        stack's backward while it runs, the conv bucket's all-reduce, then average."""
        flat = self._grad_buffer()
        split = self._dp_split_offset()
        h, hd = self._seg
        self._seg = None
        flat.zero_()
        self._backward_loss(loss)
        w_fc = dist.all_reduce(flat[split:], async_op=True)
        with K.deferred_wgrad(self.device):  # joined before the conv bucket's all-reduce
            h.backward(hd.grad)
        w_conv = dist.all_reduce(flat[:split], async_op=True)
        w_fc.wait()
        w_conv.wait()
        flat.div_(world)

    def _optimizer_step(self, loss: torch.Tensor) -> None:
        world = _world()
        if world > 1 and self._seg is not None:
            self._remove_dp_hooks()
            self._backward_segments(loss, world)
        elif world > 1:  # all-reduce (average) of the flat gradient buffer, bucketed and overlapped with backward
            flat = self._grad_buffer()
            flat.zero_()
            self._dp_arm()
            self._backward_loss(loss)
            self._dp_finish(world)
        else:  # autograd hands its gradient tensors over: no zero fill, no accumulating adds
            self._flat_grad = None
            self._remove_dp_hooks()
            for p in self.network.parameters():
                p.grad = None
            # conv weight gradients beside the rest of the backward (opt-in), or their partial-sum reductions
            # carried by the next BatchNorm backward's launch (every .grad is None here, so autograd keeps the
            # returned tensors and nothing reads them before the block closes)
            with K.deferred_wgrad(self.device), K.wgrad_piggyback(self.device, params=list(self.network.parameters())):
                self._backward_loss(loss)
        self._clip_and_step()

    def _fused_clip_adam(self) -> bool:
        """clip_grad_norm_(max_grad_norm) + Adam.step() (ppo.py:400-401) on
        bb_adam_clip_step: three launches instead of torch's ~8 (per-tensor norms,
        scalar ops, a multi-tensor scale, two multi-tensor Adam launches).  Same
        state tensors as torch's fused Adam (exp_avg, exp_avg_sq, device step),
        so save / load are unchanged.  False (nothing done) where it does not
        apply: then the torch path runs."""
        opt = self.optimizer
        if not (FUSED_ADAM and self.device.type == "cuda" and type(opt) is torch.optim.Adam
                and len(opt.param_groups) == 1):
            return False
        grp = opt.param_groups[0]
        if (grp["weight_decay"] != 0 or grp["amsgrad"] or grp["maximize"] or torch.is_tensor(grp["lr"])
                or grp.get("differentiable")):
            return False
        params = [p for p in grp["params"] if p.grad is not None]  # clip and Adam both skip the others
        if not params or len(params) > K.OPT_MAX_TENSORS:
            return False
        for p in params:
            g = p.grad
            dense = p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))
            if not (p.is_cuda and p.dtype == g.dtype == torch.float32 and dense and g.stride() == p.stride()
                    and not g.is_sparse):
                return False
            st = opt.state[p]
            if len(st) == 0:  # torch's _init_group for fused / capturable Adam: the step count on the device
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if not (st["step"].is_cuda and st["step"].dtype == torch.float32
                    and st["exp_avg"].stride() == p.stride() and st["exp_avg_sq"].stride() == p.stride()):
                return False
        key = tuple(p.numel() for p in params)
        ws = self._adam_ws.get(key)
        if ws is None:
            ws = self._adam_ws[key] = K.adam_clip_workspace(list(key), self.device)
        # for the guard's report: the parameters and gradient addresses this table (and any graph it is captured
        # into) reads
        self._adam_tables[key] = (params, tuple(p.grad.data_ptr() for p in params))
        b1, b2 = grp["betas"]
        K.adam_clip_step(params, [p.grad for p in params], [opt.state[p]["exp_avg"] for p in params],
                         [opt.state[p]["exp_avg_sq"] for p in params], [opt.state[p]["step"] for p in params],
                         grp["lr"], b1, b2, grp["eps"], self.config.max_grad_norm, ws)
        return True

    def check_optimizer_guard(self) -> None:
        """Raise when the fused clip + Adam flagged a non-finite or huge gradient-norm operand since the last
        check (bb_adam_clip_step's guard word, csrc/bb_optim.hip adam_finalize_kernel), naming the parameter."""
        if not self._adam_ws:
            return
        pname = {id(p): n for n, p in self.network.named_parameters()}
        for key, ws in self._adam_ws.items():
            params, ptrs = self._adam_tables.get(key, ((), ()))
            names = [pname.get(id(p), "?") for p in params] if params else None
            try:
                K.adam_guard_check(ws, key, names)
            except L.BBNativeError as exc:  # what the table read against what .grad holds now
                info = []
                for p, ptr, n in zip(params, ptrs, names or []):
                    g = p.grad
                    cur = g.data_ptr() if g is not None else 0
                    fin = bool(torch.isfinite(g).all()) if g is not None else None
                    nrm = float(g.detach().double().norm()) if g is not None and fin else None
                    if cur != ptr or not fin or (nrm is not None and nrm > 1e6):
                        info.append(f"{n}: table grad 0x{ptr:x}, .grad 0x{cur:x}, finite {fin}, norm {nrm}")
                # (the clip rescaled every .grad in place since the flagged read: a finite norm here says little)
                raise L.BBNativeError(f"{exc}; {'; '.join(info) if info else 'every .grad is the table one'}")

    def _clip_and_step(self) -> None:
        """clip_grad_norm_(max_grad_norm) + Adam.step() (ppo.py:397-401)."""
        if not self._fused_clip_adam():
            nn.utils.clip_grad_norm_(self.network.parameters(), self.config.max_grad_norm)
            self.optimizer.step()

    def train_minibatch(self, x, masks, actions, old_log_probs, advantages, returns) -> torch.Tensor:
        """One PPO optimizer step on a minibatch (ppo.py:362-401): loss, backward,
        gradient all-reduce, clip, Adam.  Returns the 6 loss statistics on the
        device.  On a single CUDA device the step is captured once per minibatch
        shape into a HIP graph and replayed: a step is ~440 kernels, and issued
        one by one from Python they left the GPU idle a third of the time.
        Data parallel: two graphs around the eager RCCL all-reduce of the flat
        gradient buffer -- (zero fill, forward, loss, backward into the buffer)
        and (average, clip, Adam) -- so the ranks keep graph replay."""
        if not (self.use_graphs and x.is_cuda):
            loss, stats = self._minibatch_loss(x, masks, actions, old_log_probs, advantages, returns)
            self._optimizer_step(loss)
            return stats
        inputs = (x, masks, actions, old_log_probs, advantages, returns)
        key = (tuple(t.shape for t in inputs), self.autocast_dtype, self.network.training)
        ent = self._graphs.get(key)
        if ent is None:
            ent = self._graphs[key] = self._capture_step(inputs)
        graphs, static_in, static_stats, flat = ent
        for dst, src in zip(static_in, inputs):
            if dst.data_ptr() != src.data_ptr():  # minibatch_inputs() buffers are the inputs already
                dst.copy_(src)
        graphs[0].replay()
        if len(graphs) == 3:  # segments: heads + FC backward, its all-reduce beside the conv-stack backward
            split = self._dp_split_offset()
            w_fc = dist.all_reduce(flat[split:], async_op=True)  # RCCL's stream, after graph A1
            graphs[1].replay()  # the conv-stack backward, concurrent with w_fc
            w_conv = dist.all_reduce(flat[:split], async_op=True)
            w_fc.wait()  # the compute stream waits on RCCL's (the host does not block)
            w_conv.wait()
            graphs[2].replay()
        elif len(graphs) == 2:  # the all-reduce of the flat fp32 gradient buffer (RCCL over xGMI), then the step
            work = dist.all_reduce(flat, async_op=True)  # graph B waits on it on the device, the host goes on
            work.wait()
            graphs[1].replay()
        return static_stats

    def minibatch_inputs(self, batch: int):
        """The captured optimizer step's 6 input tensors for a packed minibatch
        of ``batch`` rows (x, masks, actions, old log-probs, advantages,
        returns), for PackedRolloutBuffer.get_minibatches(out=...) to gather
        into; None until that step has been captured (or without graphs)."""
        if not (self.use_graphs and self.device.type == "cuda"):
            return None
        shapes = ((batch, 4, 8, 8), (batch, 192), (batch,), (batch,), (batch,), (batch,))
        ent = self._graphs.get((tuple(torch.Size(s) for s in shapes), self.autocast_dtype, self.network.training))
        if ent is None:
            return None
        st = ent[1]
        want = (torch.float32, torch.float32, torch.int64, torch.float32, torch.float32, torch.float32)
        if any(t.dtype != d or not t.is_contiguous() for t, d in zip(st, want)):
            return None
        return st

    def _capture_step(self, inputs):
        """Capture one optimizer step.  The warm-up steps that graph capture
        needs would change weights, BatchNorm statistics and Adam moments, so
        those are snapshotted first and restored after the capture."""
        static_in = [t.detach().clone() for t in inputs]
        with torch.no_grad():
            params = [p.detach().clone() for p in self.network.parameters()]
            bufs = [b.detach().clone() for b in self.network.buffers()]
            # the Linear tails' dropout generator word too, so the first replay draws the masks the first
            # eager step would have (models/network.py _dropout_rng)
            rng = self.network._dropout_rng(self.device) if hasattr(self.network, "_dropout_rng") else None
            rng0 = rng.clone() if rng is not None else None
            opt = {p: {k: v.detach().clone() for k, v in st.items() if torch.is_tensor(v)}
                   for p, st in self.optimizer.state.items()}
        dev_stream = torch.cuda.current_stream(self.device)
        # the hand-off kernels' counters: a block of this capture's own (zeroed on dev_stream, before the side
        # stream's fork), kept alive with its graphs
        own = K.own_counters(self.device).__enter__()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(dev_stream)
        world = _world()
        try:
            return self._capture_on(side, dev_stream, world, static_in, params, bufs, rng, rng0, opt, own)
        finally:
            own.__exit__(None, None, None)

    def _capture_on(self, side, dev_stream, world, static_in, params, bufs, rng, rng0, opt, own):
        with torch.cuda.stream(side):
            for _ in range(3):
                loss, _ = self._minibatch_loss(*static_in)
                self._optimizer_step(loss)
            # no autograd graph of the warm-up may outlive it: its AccumulateGrad nodes would be reused
            # by the capture's backward and flagged as a stream mismatch
            del loss
        graphs = [torch.cuda.CUDAGraph()]
        flat = self._flat_grad
        if world > 1 and self.dp_overlap == "graph-segments":
            flat = self._grad_buffer()
            self._remove_dp_hooks()
            graphs += [torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()]
            with torch.cuda.graph(graphs[0], stream=side):  # A1: zero, forward, loss, heads + FC backward
                flat.zero_()
                loss, stats = self._minibatch_loss(*static_in)
                self._backward_loss(loss)
                del loss
            h, hd = self._seg
            self._seg = None
            with torch.cuda.graph(graphs[1], stream=side, pool=graphs[0].pool()):  # A2: conv-stack backward
                with K.deferred_wgrad(self.device):
                    h.backward(hd.grad)
            del h, hd
            with torch.cuda.graph(graphs[2], stream=side, pool=graphs[0].pool()):  # B: average, clip, Adam
                flat.div_(world)
                self._clip_and_step()
        elif world == 1 or self.dp_overlap == "capture":
            # one graph per step; data parallel: the bucketed all-reduces issued by the backward hooks are
            # captured with it (RCCL collectives in a HIP graph)
            with torch.cuda.graph(graphs[0], stream=side):
                loss, stats = self._minibatch_loss(*static_in)
                self._optimizer_step(loss)
                del loss
            flat = self._flat_grad
        else:
            flat = self._grad_buffer()  # every .grad a view into it (made by the warm-up's eager steps)
            graphs.append(torch.cuda.CUDAGraph())
            self._dp_hooks_on = False  # graph A holds no collective: the all-reduce runs between the replays
            try:
                with torch.cuda.graph(graphs[0], stream=side):
                    flat.zero_()
                    loss, stats = self._minibatch_loss(*static_in)
                    with K.deferred_wgrad(self.device):
                        self._backward_loss(loss)
                    del loss
            finally:
                self._dp_hooks_on = True
            with torch.cuda.graph(graphs[1], stream=side, pool=graphs[0].pool()):
                flat.div_(world)
                self._clip_and_step()
        dev_stream.wait_stream(side)
        with torch.no_grad():
            for p, v in zip(self.network.parameters(), params):
                p.copy_(v)
            for b, v in zip(self.network.buffers(), bufs):
                b.copy_(v)
            if rng is not None:
                rng.copy_(rng0)
            for p, st in self.optimizer.state.items():
                old = opt.get(p)
                for k, v in st.items():
                    if torch.is_tensor(v):
                        if old is not None and k in old:
                            v.copy_(old[k])
                        else:  # fresh Adam state == zero moments at step 0
                            v.zero_()
        graphs[0].bb_counters = own.block  # the graphs embed its address
        return graphs, static_in, stats, flat

    def update(self, buffer, last_values, batch_size: Optional[int] = None) -> Dict[str, float]:
        """ppo.py:330-423.  Metrics are accumulated on the device and read once.
        ``batch_size`` overrides the per-rank minibatch (data-parallel runs
        pass config.batch_size // world so the global minibatch is unchanged)."""
        cfg = self.config
        bs = int(batch_size or cfg.batch_size)
        if isinstance(last_values, np.ndarray):
            last_values = torch.from_numpy(last_values)
        buffer.compute_returns_and_advantages(last_values, cfg.gamma, cfg.gae_lambda)
        acc = torch.zeros(6, dtype=torch.float32, device=self.device)
        n = 0
        self.minibatch_stats = []
        packed = hasattr(buffer, "get_minibatches")
        for _ in range(cfg.num_epochs):
            batches = buffer.get_minibatches(bs, out=self.minibatch_inputs) if packed else buffer.get_samples(bs)
            for batch in batches:
                if packed:
                    x, masks, actions, old_lp, adv, ret = batch
                else:
                    boards, pieces, masks, actions, old_lp, adv, ret = batch
                    x = BlockBlastNetwork.stack_input(boards.to(self.device), pieces.to(self.device))
                    masks, actions, old_lp, adv, ret = (t.to(self.device) for t in (masks, actions, old_lp, adv, ret))
                st = self.train_minibatch(x, masks, actions, old_lp, adv, ret)
                acc += st
                if self.record_minibatch_stats:  # a replayed step rewrites its stats tensor: keep a copy
                    self.minibatch_stats.append(st.clone())
                if self.minibatch_callback is not None:
                    self.minibatch_callback(n, st)
                n += 1
        m = (acc / max(n, 1)).tolist()
        self.check_optimizer_guard()
        keys = ("policy_loss", "value_loss", "entropy", "total_loss", "approx_kl", "clip_fraction")
        return dict(zip(keys, m))

    # ----------------------------------------------------------- checkpoint
    def save(self, path: str) -> None:
        """ppo.py:425-431 (same dict keys).  Saved as a plain Adam (capturable
        and fused off), so the reference's own Adam loads it on any device."""
        opt = self.optimizer.state_dict()
        opt["param_groups"] = [dict(g, capturable=False, fused=None) for g in opt["param_groups"]]
        torch.save({"network_state_dict": self.network.state_dict(),
                    "optimizer_state_dict": opt,
                    "config": self.config.to_dict()}, path)

    def load(self, path: str) -> None:
        """ppo.py:433-439 (safe loader: tensors and plain containers only)."""
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        self.network.load_state_dict(ckpt["network_state_dict"])
        if "optimizer_state_dict" in ckpt:
            self.optimizer.load_state_dict(ckpt["optimizer_state_dict"])
            cap = self.device.type == "cuda"
            for g in self.optimizer.param_groups:
                g["capturable"] = cap
                g["fused"] = True if cap else None
            for st in self.optimizer.state.values():  # capturable Adam keeps its step count on the device
                if "step" in st and torch.is_tensor(st["step"]):
                    st["step"] = st["step"].to(self.device if cap else "cpu", torch.float32)
        self._graphs = {}  # captured graphs reference the replaced optimizer state
        self.graph_epoch += 1
        if "config" in ckpt:
            self.config = PPOConfig.from_dict(ckpt["config"])
        self._flat_grad = None
        self._remove_dp_hooks()

    def train(self) -> None:
        super().train()
        self.network.train()

    def eval(self) -> None:
        super().eval()
        self.network.eval()


def broadcast_parameters(agent: PPOAgent, src: int = 0) -> None:
    """Start every data-parallel rank from rank src's weights."""
    if _world() > 1:
        for p in agent.network.state_dict().values():
            dist.broadcast(p, src)
