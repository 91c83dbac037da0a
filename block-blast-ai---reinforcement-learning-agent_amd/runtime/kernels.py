"""torch-facing wrappers of the rollout-side HIP kernels (csrc/bb_ppo.hip,
csrc/bb_env.hip expand).  Inputs/outputs are device tensors; launches go on
torch's current stream; nothing here falls back to CPU."""
from __future__ import annotations

import ctypes as C
import os
import struct
import weakref
from typing import Optional, Tuple

import torch

from . import lib as L

_BIT = None


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _s(dev: torch.device):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise L.BBNativeError("HIP kernel inputs must be device tensors (no CPU fallback)")


def pack_mask(mask: torch.Tensor) -> torch.Tensor:
    """(N, 192) bool/int/float mask -> (N, 3) int64 bit words (bbvec.h layout)."""
    global _BIT
    _need_cuda(mask)
    if _BIT is None or _BIT.device != mask.device:
        _BIT = (torch.ones(64, dtype=torch.int64, device=mask.device) << torch.arange(64, device=mask.device))
    m = (mask.reshape(mask.shape[0], 3, 64) != 0).to(torch.int64)
    return (m * _BIT).sum(dim=-1)


def masked_sample(
    logits: torch.Tensor,
    mask_bits: torch.Tensor,
    uniform: Optional[torch.Tensor] = None,
    seed: int = 0,
    step: int = 0,
    env_offset: int = 0,
    deterministic: bool = False,
    action_in: Optional[torch.Tensor] = None,
    want_entropy: bool = True,
    step_base: Optional[torch.Tensor] = None,
) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
    """Fused masked softmax / Categorical / sample / log-prob / masked entropy
    (network.py:173-180, 210-262).  logits f32 (N,192) unmasked; mask_bits
    int64 (N,3).  Returns (action int64, log_prob f32, entropy f32).
    ``step_base``: an int64 device tensor of one element; the Philox step is
    then ``step_base[0] + step``, read by the kernel (bb_masked_sample_dstep),
    so a launch captured in a HIP graph samples afresh on every replay."""
    _need_cuda(logits, mask_bits, uniform, action_in, step_base)
    logits = logits.contiguous().float()
    n = logits.shape[0]
    dev = logits.device
    act = torch.empty(n, dtype=torch.int64, device=dev)
    logp = torch.empty(n, dtype=torch.float32, device=dev)
    ent = torch.empty(n, dtype=torch.float32, device=dev) if want_entropy else None
    if step_base is not None:
        if uniform is not None or action_in is not None:
            raise ValueError("masked_sample: step_base excludes uniform / action_in")
        assert step_base.dtype == torch.int64 and step_base.numel() == 1
        L.check(
            L.load().bb_masked_sample_dstep(_p(logits), _p(mask_bits.contiguous()), n, seed, _p(step_base), step,
                                            env_offset, int(bool(deterministic)), _p(act), _p(logp), _p(ent),
                                            _s(dev)),
            "bb_masked_sample_dstep",
        )
        return act, logp, ent
    if uniform is not None:
        uniform = uniform.contiguous().float()
    if action_in is not None:
        action_in = action_in.contiguous().long()
    L.check(
        L.load().bb_masked_sample(_p(logits), _p(mask_bits.contiguous()), n, _p(uniform), seed, step, env_offset,
                                  int(bool(deterministic)), _p(action_in), _p(act), _p(logp), _p(ent), _s(dev)),
        "bb_masked_sample",
    )
    return (action_in if action_in is not None else act), logp, ent


def gae(rewards: torch.Tensor, values: torch.Tensor, dones: torch.Tensor, last_values: torch.Tensor,
        gamma: float, gae_lambda: float, adv: Optional[torch.Tensor] = None,
        ret: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """RolloutBuffer.compute_returns_and_advantages (ppo.py:141-169) on [T, N]
    f32 device tensors, numpy-2 float32 op order (gamma*lambda multiplied in
    double first, as Python does, then rounded to f32)."""
    _need_cuda(rewards, values, dones, last_values)
    T, N = rewards.shape
    adv = torch.empty_like(rewards) if adv is None else adv
    ret = torch.empty_like(rewards) if ret is None else ret
    g32 = float(torch.tensor(gamma, dtype=torch.float32))
    gl32 = float(torch.tensor(gamma * gae_lambda, dtype=torch.float32))
    L.check(
        L.load().bb_gae(_p(rewards.contiguous()), _p(values.contiguous()), _p(dones.contiguous()),
                        _p(last_values.contiguous()), T, N, g32, gl32, _p(adv), _p(ret), _s(rewards.device)),
        "bb_gae",
    )
    return adv, ret


def gather_obs(board: torch.Tensor, hand: torch.Tensor, mask_bits: torch.Tensor, index: torch.Tensor,
               want_x: bool = True, want_mask: bool = True, out_x: Optional[torch.Tensor] = None,
               out_mask: Optional[torch.Tensor] = None):
    """Packed rollout records -> network input x (n,4,8,8) f32 and f32 mask
    (n,192) for the rows in `index` (RolloutBuffer.get_samples, ppo.py:171-213),
    into out_x / out_mask when given (contiguous f32 of those shapes)."""
    _need_cuda(board, hand, mask_bits, index)
    n = index.numel()
    dev = board.device
    for o, shp in ((out_x, (n, 4, 8, 8)), (out_mask, (n, 192))):
        if o is not None and not (o.is_cuda and o.dtype == torch.float32 and tuple(o.shape) == shp
                                  and o.is_contiguous()):
            raise L.BBNativeError(f"gather_obs: output must be a contiguous f32 device tensor of shape {shp}")
    x = (out_x if out_x is not None else torch.empty((n, 4, 8, 8), dtype=torch.float32, device=dev)) \
        if want_x else None
    mf = (out_mask if out_mask is not None else torch.empty((n, 192), dtype=torch.float32, device=dev)) \
        if want_mask else None
    L.check(
        L.load().bb_gather_obs(_p(board), _p(hand), _p(mask_bits), _p(index.contiguous().long()), n, _p(x), _p(mf),
                               _s(dev)),
        "bb_gather_obs",
    )
    return x, mf


# ---------------------------------------------------------------------------
# Training-mode BatchNorm2d (+ fused ReLU) on the HIP kernels of csrc/bb_nn.hip
# ---------------------------------------------------------------------------
_BN_DTYPES = {torch.float32: 0, torch.bfloat16: 1}


def _bn_layout(x: torch.Tensor) -> int:
    """1 when x is laid out channels_last (NHWC) and not also NCHW-contiguous."""
    return int(x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous())


def bn_fusable(x: torch.Tensor) -> bool:
    """f32/bf16 device tensor, NCHW with HW rows or NHWC with C rows of whole
    16-byte vectors."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype in _BN_DTYPES and x.numel() > 0):
        return False
    if _bn_layout(x):
        row = x.shape[1] * x.element_size()  # bytes per NHWC row: 16 x a power of two <= 256
        return row % 16 == 0 and 256 % (row // 16) == 0
    return (x.shape[2] * x.shape[3] * x.element_size()) % 16 == 0


# BatchNorm batch statistics from the producing convolution's store pass (bb_conv3x3_forward_stats ->
# bb_bn_forward_part): no reduction pass over the convolution's output (0: bb_bn_forward's own pass, for A/B)
CONV_STATS = os.environ.get("BB_CONV_STATS", "1") != "0"
# ... and a ResidualBlock's bn1 backward sums from conv2's data-gradient store pass (bb_conv3x3_forward_bstats).
# Off: 1.510 against 1.503 ms per update step (the store pass's +11.5 us per launch outweighs the 13.6 us
# reduction it replaces plus the extra partials; profiles/r05/ab/convstats)
CONV_BSTATS = os.environ.get("BB_CONV_BSTATS", "0") != "0"


class StatsSlot:
    """Carries BatchNorm reduction partials from a board convolution's store pass to a BatchNorm: forward, the
    statistics of the convolution's output (bb_conv3x3_forward_stats); backward, the reduction sums of the
    BatchNorm whose output the convolution read, from the convolution's data gradient
    (bb_conv3x3_forward_bstats; ``bn`` = that BatchNorm's input and coefficients, set by its forward)."""

    __slots__ = ("part", "nb", "ptr", "bn")

    def __init__(self):
        self.part, self.nb, self.ptr, self.bn = None, 0, 0, None


def _stats_for(slot, x: torch.Tensor):
    """(partials, blocks) when ``slot`` holds the statistics of exactly x (bf16 NHWC), else None."""
    if slot is None or slot.part is None or slot.ptr != x.data_ptr() or x.dtype != torch.bfloat16 \
            or not _bn_layout(x):
        return None
    return slot.part, slot.nb


def _bn_workspace(x: torch.Tensor, nhwc: int) -> torch.Tensor:
    n, c, h, w = x.shape
    nbytes = L.load().bb_bn_workspace_bytes(_BN_DTYPES[x.dtype], nhwc, n, c, h * w)
    if nbytes < 0:
        raise L.BBNativeError(f"bb_bn_workspace_bytes rejected shape {tuple(x.shape)} {x.dtype} nhwc={nhwc}")
    return torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=x.device)


def _bn_backward_call(x, dy, nhwc, pre_bias, weight, bias, mean, invstd, relu: int, ws, dx, dw, db, dpb, dev,
                      part=None):
    """bb_bn_backward, or bb_bn_backward_red carrying a board convolution's pending weight-gradient reduction
    (wgrad_piggyback) in its finalisation launch; part = (partials, blocks): bb_bn_backward_part (the reduction
    sums from the convolution that produced dy)."""
    n, c, h, w = x.shape
    lib = L.load()
    job = _take_pending_reduce(dev)
    args = (_p(x), _p(dy), _BN_DTYPES[x.dtype], nhwc, n, c, h * w, _p(pre_bias), _p(weight), _p(bias), _p(mean),
            _p(invstd), int(relu), _p(ws), _p(dx), _p(dw), _p(db), _p(dpb))
    if part is not None:
        cws, chunks, cin, cout, wl, cdw = job if job is not None else (None, 0, 0, 0, 0, None)
        L.check(lib.bb_bn_backward_part(*args, _p(cws), chunks, cin, cout, wl, C.c_void_p(cdw), _p(part[0]), part[1],
                                        _s(dev)), "bb_bn_backward_part")
    elif job is None:
        L.check(lib.bb_bn_backward(*args, _s(dev)), "bb_bn_backward")
    else:
        cws, chunks, cin, cout, wl, cdw = job
        L.check(lib.bb_bn_backward_red(*args, _p(cws), chunks, cin, cout, wl, C.c_void_p(cdw), _s(dev)),
                "bb_bn_backward_red")


class BatchNormReLUFunction(torch.autograd.Function):
    """y = [relu](batch_norm(x + pre_bias, batch statistics)) with running-stat
    update; backward from x and the saved mean / inverse std
    (bb_bn_forward/backward).  ``pre_bias`` is the preceding convolution's
    bias (None = none), so conv(x) without bias -> this == conv(x) + bias ->
    nn.BatchNorm2d [-> ReLU]; its gradient is the per-channel sum of dx."""

    @staticmethod
    def forward(ctx, x, pre_bias, weight, bias, running_mean, running_var, momentum: float, eps: float, relu: bool,
                num_batches_tracked=None, stats=None, bwd_slot=None):
        nhwc = _bn_layout(x)
        x = x.contiguous(memory_format=torch.channels_last if nhwc else torch.contiguous_format)
        n, c, h, w = x.shape
        dev = x.device
        y = torch.empty_like(x)
        ws = _bn_workspace(x, nhwc)
        mean = torch.empty(c, dtype=torch.float32, device=dev)
        invstd = torch.empty(c, dtype=torch.float32, device=dev)
        args = (_p(x), _BN_DTYPES[x.dtype], nhwc, n, c, h * w, _p(pre_bias), _p(weight), _p(bias), float(eps),
                int(relu), _p(ws), _p(mean), _p(invstd), _p(running_mean), _p(running_var), float(momentum),
                _p(num_batches_tracked), _p(y))
        st = _stats_for(stats, x)
        if st is None:
            L.check(L.load().bb_bn_forward(*args, _s(dev)), "bb_bn_forward")
        else:  # the statistics came out of the convolution's store pass
            L.check(L.load().bb_bn_forward_part(args[0], None, *args[1:], _p(st[0]), st[1], _s(dev)),
                    "bb_bn_forward_part")
        ctx.save_for_backward(x, pre_bias, weight, bias, mean, invstd)
        ctx.relu = bool(relu)
        ctx.nhwc = nhwc
        ctx.bwd_slot = None
        if bwd_slot is not None and nhwc and x.dtype == torch.bfloat16:  # for the next convolution's backward
            bwd_slot.bn = (x, weight, bias, mean, invstd, int(relu))
            ctx.bwd_slot = bwd_slot
        return y

    @staticmethod
    def backward(ctx, dy):
        x, pre_bias, weight, bias, mean, invstd = ctx.saved_tensors
        fmt = torch.channels_last if ctx.nhwc else torch.contiguous_format
        dy = dy.to(x.dtype).contiguous(memory_format=fmt)
        n, c, h, w = x.shape
        dev = x.device
        dx = torch.empty_like(x)
        dw = torch.empty_like(weight)
        db = torch.empty_like(bias)
        dpb = torch.empty_like(pre_bias) if pre_bias is not None else None
        ws = _bn_workspace(x, ctx.nhwc)
        slot = ctx.bwd_slot
        part = _stats_for(slot, dy)
        if slot is not None:
            slot.part, slot.bn = None, None  # used once
        _bn_backward_call(x, dy, ctx.nhwc, pre_bias, weight, bias, mean, invstd, int(ctx.relu), ws, dx, dw, db, dpb,
                          dev, part)
        return dx, dpb, dw, db, None, None, None, None, None, None, None, None


# ResidualBlock tail backward on bb_bn_backward_res: the ReLU mask applied in the BatchNorm reduction, which
# writes the masked gradient for the elementwise pass (0: threshold_backward + bb_bn_backward, for A/B).
# 1.575-1.579 against 1.579-1.583 ms per step, three interleaved repeats, 2 launches fewer
# (profiles/r05/rm/r05rm2_ab.log; the first form, mask applied in both passes, was 1.619 against 1.613)
RES_MASK = os.environ.get("BB_RES_MASK", "1") != "0"


class BatchNormAddReLUFunction(torch.autograd.Function):
    """relu(batch_norm(x + pre_bias) + res) with running-stat update: the tail
    of ResidualBlock (network.py:14-30, bn2 -> + identity -> relu) in the
    BatchNorm apply pass (bb_bn_forward_res) instead of two more elementwise
    passes.  Backward: bb_bn_backward_res -- the ReLU mask from the saved
    output (torch's threshold_backward, as F.relu's backward) applied inside
    the BatchNorm passes, the masked gradient (the residual's) written by the
    elementwise pass."""

    @staticmethod
    def forward(ctx, x, pre_bias, res, weight, bias, running_mean, running_var, momentum: float, eps: float,
                num_batches_tracked=None, grad_mailbox=None, stats=None):
        ctx.mailbox = grad_mailbox
        nhwc = _bn_layout(x)
        fmt = torch.channels_last if nhwc else torch.contiguous_format
        x = x.contiguous(memory_format=fmt)
        res = res.contiguous(memory_format=fmt)
        n, c, h, w = x.shape
        dev = x.device
        y = torch.empty_like(x)
        ws = _bn_workspace(x, nhwc)
        mean = torch.empty(c, dtype=torch.float32, device=dev)
        invstd = torch.empty(c, dtype=torch.float32, device=dev)
        args = (_p(x), _p(res), _BN_DTYPES[x.dtype], nhwc, n, c, h * w, _p(pre_bias), _p(weight), _p(bias),
                float(eps), 1, _p(ws), _p(mean), _p(invstd), _p(running_mean), _p(running_var), float(momentum),
                _p(num_batches_tracked), _p(y))
        st = _stats_for(stats, x)
        if st is None:
            L.check(L.load().bb_bn_forward_res(*args, _s(dev)), "bb_bn_forward_res")
        else:  # the statistics came out of the convolution's store pass
            L.check(L.load().bb_bn_forward_part(*args, _p(st[0]), st[1], _s(dev)), "bb_bn_forward_part")
        ctx.save_for_backward(x, pre_bias, weight, bias, mean, invstd, y)
        ctx.nhwc = nhwc
        return y

    @staticmethod
    def backward(ctx, dy):
        x, pre_bias, weight, bias, mean, invstd, y = ctx.saved_tensors
        fmt = torch.channels_last if ctx.nhwc else torch.contiguous_format
        dy = dy.to(x.dtype).contiguous(memory_format=fmt)
        n, c, h, w = x.shape
        dev = x.device
        dx = torch.empty_like(x)
        dw = torch.empty_like(weight)
        db = torch.empty_like(bias)
        dpb = torch.empty_like(pre_bias) if pre_bias is not None else None
        ws = _bn_workspace(x, ctx.nhwc)
        if RES_MASK:  # the ReLU's mask from the saved output inside the BatchNorm passes (threshold_backward)
            g = torch.empty_like(x)  # the masked gradient: the residual's, and the elementwise pass's input
            job = _take_pending_reduce(dev)  # a convolution's weight-gradient reduction, carried along
            red = (None, 0, 0, 0, 0, None) if job is None else job
            L.check(L.load().bb_bn_backward_res(_p(x), _p(dy), _p(y), _BN_DTYPES[x.dtype], ctx.nhwc, n, c, h * w,
                                                _p(pre_bias), _p(weight), _p(bias), _p(mean), _p(invstd), _p(ws),
                                                _p(dx), _p(dw), _p(db), _p(dpb), _p(g), _p(red[0]), red[1], red[2],
                                                red[3], red[4], None if red[5] is None else C.c_void_p(red[5]),
                                                _s(dev)),
                    "bb_bn_backward_res")
        else:
            g = torch.ops.aten.threshold_backward(dy, y, 0).contiguous(memory_format=fmt)
            _bn_backward_call(x, g, ctx.nhwc, pre_bias, weight, bias, mean, invstd, 0, ws, dx, dw, db, dpb, dev)
        gres = g
        if ctx.mailbox is not None and ctx.needs_input_grad[2]:
            ctx.mailbox.put(g)  # the block's first convolution adds it to its data gradient
            gres = None
        return dx, dpb, gres, dw, db, None, None, None, None, None, None, None


# ---------------------------------------------------------------------------
# 3x3 / pad-1 convolutions over 8x8 boards, bf16 MFMA (csrc/bb_conv.hip)
# ---------------------------------------------------------------------------
_CONV_CH = (64, 128)

# ---------------------------------------------------------------------------
# Deferred convolution weight gradients: inside ``deferred_wgrad(device)`` the
# board convolutions' weight-gradient kernels run on a side stream forked from
# the current one and accumulate into ``weight.grad`` there, off autograd's
# critical path (dgrad -> BatchNorm backward -> dgrad ...): the MFMA-bound
# weight gradients overlap the HBM-bound BatchNorm passes of the rest of the
# backward.  On exit the current stream waits for the side stream, so every
# weight gradient is complete before anything after the block reads it
# (clip + Adam, the data-parallel all-reduce).  Captured HIP graphs record the
# fork / join.  Outside the block the weight gradient is autograd's as usual.
# ---------------------------------------------------------------------------
# opt-in: measured slower (bf16 optimizer step 1.885 ms with the side stream against 1.711 ms without, two
# interleaved repeats each, profiles/r05/pu/): the weight gradients and the BatchNorm backward passes slow each other
# down more than the overlap saves (bn_reduce_nhwc backward 21 -> 35 us, conv_wgrad 38 -> 46 us per call)
ASYNC_WGRAD = os.environ.get("BB_ASYNC_WGRAD", "0") == "1"
_wg_streams = {}
_wg_active = {}  # device -> [depth, used]


class deferred_wgrad:
    def __init__(self, device: torch.device, enabled: bool = True):
        self.dev = _dev_key(device)
        self.on = bool(enabled and ASYNC_WGRAD and self.dev.type == "cuda")

    def __enter__(self):
        if self.on:
            st = _wg_active.setdefault(self.dev, [0, False])
            st[0] += 1
        return self

    def __exit__(self, *exc):
        if self.on:
            st = _wg_active[self.dev]
            st[0] -= 1
            if st[1]:
                torch.cuda.current_stream(self.dev).wait_stream(_wg_streams[self.dev])
                st[1] = st[0] > 0
        return False


def _wgrad_deferred(weight: torch.Tensor, dev: torch.device, saved, compute) -> bool:
    """Run compute() -> dw on the side stream and add it into weight.grad there when a deferred_wgrad block
    is open on ``dev``; False (nothing done) otherwise.  ``saved``: tensors of the current stream that the
    side stream reads (kept from reuse until it has)."""
    dev = _dev_key(dev)
    st = _wg_active.get(dev)
    if not st or st[0] <= 0 or weight.grad is not None and weight.grad.is_sparse:
        return False
    side = _wg_streams.get(dev)
    if side is None:
        side = _wg_streams[dev] = torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        dw = compute()
        g = weight.grad
        if g is None:
            weight.grad = dw
        else:
            g.add_(dw)
    for t in saved:
        t.record_stream(side)
    st[1] = True
    return True


# ---------------------------------------------------------------------------
# Weight-gradient reductions carried by the next BatchNorm backward: inside ``wgrad_piggyback(device)`` a board
# convolution's backward launches only the weight-gradient partial-sum kernel and leaves its fixed-order reduction
# pending; the next BatchNorm backward on the device (the one that always follows a convolution in the CNN's
# backward) runs it as extra workgroups of its finalisation launch (bb_bn_backward_red): two small launches become
# one.  Whatever is still pending when the block closes (or when a second convolution comes first) is reduced in
# a launch of its own, so every weight gradient is complete at the block's exit -- before clip + Adam or a
# data-parallel all-reduce reads it.  Only for backward passes with no gradient hooks in between (a hook would see
# the weight gradient before its reduction): PPOAgent opens the block on one rank, or around a data-parallel
# backward whose all-reduce runs after it.
# ---------------------------------------------------------------------------
# A pending job holds the weight gradient by address only: a Python reference would make autograd's
# AccumulateGrad copy the (not yet reduced) tensor into .grad instead of keeping it; the block's exit checks that
# every such .grad is the tensor the reduction wrote.
WGRAD_PIGGYBACK = os.environ.get("BB_WGRAD_PIGGYBACK", "1") != "0"
_pending_red = {}  # device -> [depth, pending job or None, [(weight, dw address)]]


def _flush_reduce(dev, job) -> None:
    cws, chunks, cin, cout, wl, cdw = job
    L.check(L.load().bb_conv3x3_wgrad_reduce(_p(cws), chunks, cin, cout, wl, C.c_void_p(cdw), _s(dev)),
            "bb_conv3x3_wgrad_reduce")


def _take_pending_reduce(dev):
    st = _pending_red.get(_dev_key(dev))
    if not st or st[1] is None:
        return None
    job, st[1] = st[1], None
    return job


class wgrad_piggyback:
    """``params``: the parameters whose gradients the backward inside produces; every .grad must be None at
    entry (autograd then keeps the tensors the reductions write instead of adding them into old ones)."""

    def __init__(self, device: torch.device, enabled: bool = True, params=None):
        self.dev = _dev_key(device)
        self.on = bool(enabled and WGRAD_PIGGYBACK and self.dev.type == "cuda")
        self.params = params

    def __enter__(self):
        if self.on:
            if self.params is not None and any(p.grad is not None for p in self.params):
                raise L.BBNativeError("wgrad_piggyback: every parameter's .grad must be None when the block opens")
            _pending_red.setdefault(self.dev, [0, None, []])[0] += 1
        return self

    def __exit__(self, *exc):
        if self.on:
            st = _pending_red[self.dev]
            st[0] -= 1
            job = _take_pending_reduce(self.dev)
            if job is not None:
                _flush_reduce(self.dev, job)
            checks, st[2] = st[2], []
            for weight, addr in checks:
                if exc[0] is None and (weight.grad is None or weight.grad.data_ptr() != addr):
                    raise L.BBNativeError("wgrad_piggyback: autograd copied a pending weight gradient; open the "
                                          "block only around a backward whose parameters' .grad are all None")
        return False


def conv3x3_fusable(x: torch.Tensor, conv) -> bool:
    """An nn.Conv2d 3x3 / stride 1 / pad 1 with 64 or 128 channels in and out,
    applied to a device tensor of 8x8 boards."""
    return (x.is_cuda and x.dim() == 4 and x.shape[2] == 8 and x.shape[3] == 8 and x.shape[0] > 0
            and conv.in_channels in _CONV_CH and conv.out_channels in _CONV_CH and conv.groups == 1
            and tuple(conv.kernel_size) == (3, 3) and tuple(conv.stride) == (1, 1)
            and tuple(conv.padding) == (1, 1) and tuple(conv.dilation) == (1, 1) and conv.padding_mode == "zeros")


def _w_layout(w: torch.Tensor) -> int:
    if w.is_contiguous():
        return 0
    if w.is_contiguous(memory_format=torch.channels_last):
        return 1
    raise L.BBNativeError("conv weight must be contiguous or channels_last")


# the input layer (conv 4 -> 64) on bb_conv_in_forward / _wgrad under bf16 autocast (0: MIOpen's, for A/B)
CONV_IN = os.environ.get("BB_CONV_IN", "1") != "0"


def conv_in_fusable(x: torch.Tensor, conv) -> bool:
    """The input layer: an nn.Conv2d 4 -> 64, 3x3 / stride 1 / pad 1, on f32 8x8 boards (NCHW or channels_last)."""
    return (CONV_IN and x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and x.shape[1:] == (4, 8, 8)
            and x.shape[0] > 0 and conv.in_channels == 4 and conv.out_channels == 64 and conv.groups == 1
            and tuple(conv.kernel_size) == (3, 3) and tuple(conv.stride) == (1, 1)
            and tuple(conv.padding) == (1, 1) and tuple(conv.dilation) == (1, 1) and conv.padding_mode == "zeros"
            and conv.weight.dtype == torch.float32
            and (x.is_contiguous() or x.is_contiguous(memory_format=torch.channels_last)))


class ConvInFunction(torch.autograd.Function):
    """conv2d(x, weight, padding=1) without bias for the 4 -> 64 input layer under bf16 autocast: f32 input and
    weight rounded to bf16 (autocast's casts), f32 sums, bf16 NHWC output; backward: the f32 weight gradient
    only (the input is data)."""

    @staticmethod
    def forward(ctx, x, weight, prep: Optional["PrepJob"] = None):
        _need_cuda(x, weight)
        nhwc = 0 if x.is_contiguous() else 1
        wl = _w_layout(weight)
        n = x.shape[0]
        y = torch.empty((n, 64, 8, 8), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        if prep is not None and not prep.done:  # the other layers' weight images in the same launch
            L.check(L.load().bb_conv_in_forward_prep(_p(x), nhwc, _p(weight), wl, n, _p(y), *prep.args, _s(x.device)),
                    "bb_conv_in_forward_prep")
            prep.done = True
        else:
            L.check(L.load().bb_conv_in_forward(_p(x), nhwc, _p(weight), wl, n, _p(y), _s(x.device)),
                    "bb_conv_in_forward")
        ctx.save_for_backward(x, weight)
        ctx.nhwc, ctx.wl = nhwc, wl
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        if not ctx.needs_input_grad[1]:
            return None, None, None
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n = x.shape[0]
        lib = L.load()
        ws = torch.empty((lib.bb_conv_in_wgrad_workspace_bytes(n) + 3) // 4, dtype=torch.float32, device=x.device)
        dw = torch.empty_like(weight)
        L.check(lib.bb_conv_in_wgrad(_p(x), ctx.nhwc, _p(dy), n, _p(ws), ctx.wl, _p(dw), _s(x.device)),
                "bb_conv_in_wgrad")
        return None, dw, None


class Conv3x3Function(torch.autograd.Function):
    """conv2d(x, weight, padding=1) without bias under bf16 autocast:
    bf16 NHWC activations, f32 accumulation, bf16 output, f32 weight gradient
    (bb_conv3x3_prep / _forward / _wgrad; the data gradient is the forward
    kernel over dy with the tap-reversed, transposed weight image)."""

    @staticmethod
    def forward(ctx, x, weight, images=None, grad_mailbox=None, stats=None, bwd_slot=None):
        _need_cuda(x, weight)
        ctx.mailbox = grad_mailbox
        ctx.bwd_slot = bwd_slot
        x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        n, cin = x.shape[0], x.shape[1]
        cout = weight.shape[0]
        dev = x.device
        lib = L.load()
        if images is not None:  # from conv3x3_prep_multi (all layers in one launch)
            wf, wd = images
        else:
            wl = _w_layout(weight)
            wf = torch.empty(9 * cout * cin, dtype=torch.bfloat16, device=dev)
            wd = torch.empty(9 * cout * cin, dtype=torch.bfloat16, device=dev)
            L.check(lib.bb_conv3x3_prep(_p(weight), cin, cout, wl, _p(wf), _p(wd), _s(dev)), "bb_conv3x3_prep")
        y = torch.empty((n, cout, 8, 8), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        if stats is not None and CONV_STATS:  # + the following BatchNorm's statistics partials (StatsSlot)
            nbp = lib.bb_conv3x3_stats_blocks(n, cout)
            part = torch.empty(nbp * cout * 3, dtype=torch.float64, device=dev)
            L.check(lib.bb_conv3x3_forward_stats(_p(x), _p(wf), n, cin, cout, _p(y), _p(part), _s(dev)),
                    "bb_conv3x3_forward_stats")
            stats.part, stats.nb, stats.ptr = part, nbp, y.data_ptr()
        else:
            L.check(lib.bb_conv3x3_forward(_p(x), _p(wf), n, cin, cout, _p(y), _s(dev)), "bb_conv3x3_forward")
        ctx.save_for_backward(x, wd, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wd, weight = ctx.saved_tensors
        n, cin = x.shape[0], x.shape[1]
        cout = weight.shape[0]
        dev = x.device
        lib = L.load()
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            extra = ctx.mailbox.take() if ctx.mailbox is not None else None
            if extra is not None:  # + the identity path's gradient of x, in the store pass
                extra = extra.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
                L.check(lib.bb_conv3x3_forward_add(_p(dy), _p(wd), n, cout, cin, _p(extra), _p(dx), _s(dev)),
                        "bb_conv3x3_forward_add")
            else:
                slot = ctx.bwd_slot
                bn = slot.bn if slot is not None and CONV_STATS and CONV_BSTATS else None
                if bn is not None and bn[0].shape == dx.shape and bn[0].dtype == torch.bfloat16 \
                        and bn[0].is_contiguous(memory_format=torch.channels_last):
                    # + the reduction sums of the BatchNorm whose output x is (its backward skips its own pass)
                    nbp = lib.bb_conv3x3_stats_blocks(n, cin)
                    part = torch.empty(nbp * cin * 3, dtype=torch.float64, device=dev)
                    bx, bw, bb, bmean, binv, brelu = bn
                    L.check(lib.bb_conv3x3_forward_bstats(_p(dy), _p(wd), n, cout, cin, _p(dx), _p(bx), _p(bmean),
                                                          _p(binv), _p(bw), _p(bb), brelu, _p(part), _s(dev)),
                            "bb_conv3x3_forward_bstats")
                    slot.part, slot.nb, slot.ptr = part, nbp, dx.data_ptr()
                else:
                    L.check(lib.bb_conv3x3_forward(_p(dy), _p(wd), n, cout, cin, _p(dx), _s(dev)),
                            "bb_conv3x3_forward")
        if ctx.needs_input_grad[1]:
            nbytes = lib.bb_conv3x3_workspace_bytes(n, cin, cout)
            if nbytes < 0:
                raise L.BBNativeError(f"bb_conv3x3_workspace_bytes rejected {n}x{cin}->{cout}")

            def wgrad():
                ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
                g = torch.empty_like(weight, dtype=torch.float32)
                L.check(lib.bb_conv3x3_wgrad(_p(x), _p(dy), n, cin, cout, _p(ws), _w_layout(g), _p(g), _s(dev)),
                        "bb_conv3x3_wgrad")
                return g

            st = _pending_red.get(_dev_key(dev))
            if st and st[0] > 0 and not _wg_active.get(_dev_key(dev), [0])[0] > 0:
                # partial sums now, their reduction in the next BatchNorm backward's finalisation launch
                prev = _take_pending_reduce(dev)
                if prev is not None:
                    _flush_reduce(dev, prev)
                ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=dev)
                dw = torch.empty_like(weight, dtype=torch.float32)
                L.check(lib.bb_conv3x3_wgrad_partial(_p(x), _p(dy), n, cin, cout, _p(ws), _s(dev)),
                        "bb_conv3x3_wgrad_partial")
                st[1] = (ws, lib.bb_conv3x3_wgrad_chunks(n, cin, cout), cin, cout, _w_layout(dw), dw.data_ptr())
                st[2].append((weight, dw.data_ptr()))
            elif not _wgrad_deferred(weight, dev, (x, dy), wgrad):
                dw = wgrad()
        return dx, dw, None, None, None, None


_CONV32_PAIRS = ((128, 128), (64, 128))  # forward layers; the 64 -> 128 layer's data gradient runs (128, 64)


def conv3x3_f32_fusable(x: torch.Tensor, conv) -> bool:
    """conv3x3_fusable, fp32 activations and weights, (cin, cout) in _CONV32_PAIRS."""
    return (x.dtype == torch.float32 and conv.weight.dtype == torch.float32 and conv3x3_fusable(x, conv)
            and (conv.in_channels, conv.out_channels) in _CONV32_PAIRS)


class Conv3x3F32Function(torch.autograd.Function):
    """conv2d(x, weight, padding=1) without bias in fp32 (no autocast) on csrc/bb_conv32.hip: f32 NHWC
    activations, every output the fp64 sum of 16-product fp32 MFMA chains rounded once (bb_conv3x3_f32_prep
    / _forward).  Backward: the data gradient on the same kernel with the tap-reversed, transposed weight
    image; the weight gradient from aten's convolution_backward (MIOpen)."""

    @staticmethod
    def forward(ctx, x, weight):
        _need_cuda(x, weight)
        x = x.contiguous(memory_format=torch.channels_last)
        n, cin = x.shape[0], x.shape[1]
        cout = weight.shape[0]
        dev = x.device
        lib = L.load()
        need_dx = ctx.needs_input_grad[0]
        wf = torch.empty(9 * cout * cin, dtype=torch.float32, device=dev)
        wd = torch.empty(9 * cout * cin, dtype=torch.float32, device=dev) if need_dx else None
        L.check(lib.bb_conv3x3_f32_prep(_p(weight), cin, cout, _w_layout(weight), _p(wf), _p(wd), _s(dev)),
                "bb_conv3x3_f32_prep")
        y = torch.empty((n, cout, 8, 8), dtype=torch.float32, device=dev, memory_format=torch.channels_last)
        L.check(lib.bb_conv3x3_f32_forward(_p(x), _p(wf), n, cin, cout, _p(y), _s(dev)), "bb_conv3x3_f32_forward")
        ctx.save_for_backward(x, wd, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wd, weight = ctx.saved_tensors
        n, cin = x.shape[0], x.shape[1]
        cout = weight.shape[0]
        dev = x.device
        dy = dy.float().contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            L.check(L.load().bb_conv3x3_f32_forward(_p(dy), _p(wd), n, cout, cin, _p(dx), _s(dev)),
                    "bb_conv3x3_f32_forward")
        if ctx.needs_input_grad[1]:
            def wgrad():
                return torch.ops.aten.convolution_backward(dy, x, weight, None, [1, 1], [1, 1], [1, 1], False,
                                                           [0, 0], 1, [False, True, False])[1]

            if not _wgrad_deferred(weight, dev, (x, dy), wgrad):
                dw = wgrad()
        return dx, dw


def linear_f32(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """nn.Linear's forward in fp32 with blocked fp32 MFMA chains summed in fp64 (bb_linear_f32); no autograd."""
    _need_cuda(x, weight)
    x = x.contiguous()
    weight = weight.contiguous()
    m, k = x.shape
    n = weight.shape[0]
    y = torch.empty((m, n), dtype=torch.float32, device=x.device)
    L.check(L.load().bb_linear_f32(_p(x), _p(weight), _p(bias.contiguous() if bias is not None else None), m, n, k,
                                   _p(y), _s(x.device)), "bb_linear_f32")
    return y


class GradMailbox:
    """Hands the identity path's gradient of a ResidualBlock input from
    BatchNormAddReLUFunction.backward to the block's first Conv3x3Function
    backward (which autograd runs later: it is upstream), so that the sum of the
    two input gradients is formed in the data-gradient convolution's store pass
    instead of a separate add kernel."""

    def __init__(self):
        self.g = None

    def put(self, g):
        self.g = g

    def take(self):
        g, self.g = self.g, None
        return g


class PrepJob:
    """The table of a bb_conv3x3_prep_multi launch not yet made (conv3x3_prep_multi(..., defer=True)): the input
    layer's forward launch carries it (bb_conv_in_forward_prep), or run() launches it on its own."""

    def __init__(self, weights, imgs):
        k = len(weights)
        i32 = C.c_int32 * k
        self.dev = weights[0].device
        self.keep = (weights, imgs)
        self.args = (k, _ptrs(weights), i32(*[w.shape[1] for w in weights]), i32(*[w.shape[0] for w in weights]),
                     i32(*[_w_layout(w) for w in weights]), _ptrs([a for a, _ in imgs]), _ptrs([b for _, b in imgs]))
        self.done = False

    def run(self) -> None:
        if not self.done:
            L.check(L.load().bb_conv3x3_prep_multi(*self.args, _s(self.dev)), "bb_conv3x3_prep_multi")
            self.done = True


def conv3x3_prep_multi(weights, defer: bool = False):
    """bb_conv3x3_prep of every weight in one launch (bb_conv3x3_prep_multi):
    [(forward image, data-gradient image)] per weight, bf16.  defer: return (images, PrepJob) with nothing
    launched yet."""
    k = len(weights)
    if not 0 < k <= 16:
        raise L.BBNativeError("conv3x3_prep_multi: 1 to 16 layers")
    _need_cuda(*weights)
    dev = weights[0].device
    imgs = []
    for w in weights:
        n = w.shape[0] * w.shape[1] * 9
        imgs.append((torch.empty(n, dtype=torch.bfloat16, device=dev), torch.empty(n, dtype=torch.bfloat16, device=dev)))
    job = PrepJob(weights, imgs)
    if defer:
        return imgs, job
    job.run()
    return imgs


# ---------------------------------------------------------------------------
# PPO minibatch loss, forward and backward (csrc/bb_loss.hip)
# ---------------------------------------------------------------------------
class PPOLossFunction(torch.autograd.Function):
    """PPOAgent's minibatch loss (ppo.py:362-401) with the masked Categorical
    tail (network.py:173-180, 210-262) on bb_ppo_loss_forward/backward.
    Returns (total loss, stats[6] = policy / value / entropy / total loss,
    approx_kl, clip_fraction); stats carry no gradient.  ``seed``: the tensor
    the caller will backpropagate the loss with (its value read on the device
    when the forward runs): forward and backward then run as one launch
    (bb_ppo_loss_fused), and the backward hands those gradients over when
    autograd passes that same tensor; any other gradient runs bb_ppo_loss_backward."""

    @staticmethod
    def forward(ctx, logits, values, masks, actions, old_log_probs, advantages, returns, clip: float,
                value_coef: float, entropy_coef: float, seed: Optional[torch.Tensor] = None):
        _need_cuda(logits, values, masks, actions, old_log_probs, advantages, returns)
        # bf16 logits and values (the autocast network's) are read as they are and get bf16 gradients
        # (bb_ppo_loss_*_bf16: the values of autograd's casts, without the cast launches)
        bf16 = logits.dtype == torch.bfloat16 and values.dtype == torch.bfloat16
        act = torch.bfloat16 if bf16 else torch.float32
        ins = (logits.contiguous().to(act), values.contiguous().to(act), masks.contiguous().float(),
               actions.contiguous().long(), old_log_probs.contiguous().float(), advantages.contiguous().float(),
               returns.contiguous().float())
        b = ins[0].shape[0]
        dev = ins[0].device
        lib = L.load()
        ws = torch.empty((lib.bb_ppo_loss_workspace_bytes(b) + 7) // 8, dtype=torch.float64, device=dev)
        cnt = _bgrad_counters(dev, 1)
        stats = torch.empty(6, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        coef = (float(clip), float(value_coef), float(entropy_coef))
        ctx.seed, ctx.grads = None, None
        if seed is not None and seed.is_cuda and seed.dtype == torch.float32 and seed.numel() == 1:
            dlogits, dvalues = torch.empty_like(ins[0]), torch.empty_like(ins[1])
            L.check(lib.bb_ppo_loss_fused(_p(ins[0]), _p(ins[1]), int(bf16), *[_p(t) for t in ins[2:]], b, *coef,
                                          _p(seed), _p(dlogits), _p(dvalues), _p(ws), _p(cnt), _p(stats), _p(loss),
                                          _s(dev)), "bb_ppo_loss_fused")
            ctx.seed, ctx.grads = seed, (dlogits, dvalues)
        else:
            fn = lib.bb_ppo_loss_forward_bf16 if bf16 else lib.bb_ppo_loss_forward
            L.check(fn(*[_p(t) for t in ins], b, *coef, _p(ws), _p(cnt), _p(stats), _p(loss), _s(dev)),
                    "bb_ppo_loss_forward")
        ctx.save_for_backward(*ins)
        ctx.coef = coef
        ctx.bf16 = bf16
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics
        return loss, stats

    @staticmethod
    def backward(ctx, grad_loss, grad_stats):
        if grad_loss is None:
            return (None,) * 11
        if ctx.grads is not None and grad_loss is ctx.seed:  # computed by the forward's launch
            dlogits, dvalues = ctx.grads
            ctx.grads = None
            return dlogits, dvalues, None, None, None, None, None, None, None, None, None
        ins = ctx.saved_tensors
        b = ins[0].shape[0]
        dev = ins[0].device
        g = grad_loss.float().reshape(1).contiguous()
        dlogits = torch.empty_like(ins[0])
        dvalues = torch.empty_like(ins[1])
        fn = L.load().bb_ppo_loss_backward_bf16 if ctx.bf16 else L.load().bb_ppo_loss_backward
        L.check(fn(*[_p(t) for t in ins], b, *ctx.coef, _p(g), _p(dlogits), _p(dvalues), _s(dev)),
                "bb_ppo_loss_backward")
        return dlogits, dvalues, None, None, None, None, None, None, None, None, None


# ---------------------------------------------------------------------------
# clip_grad_norm_ + Adam, and the Linear layers' autocast casts (csrc/bb_optim.hip)
# ---------------------------------------------------------------------------
OPT_MAX_TENSORS = 48  # BB_OPT_MAX_TENSORS


def _ptrs(ts):
    return (C.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


def adam_clip_workspace(numels, device) -> torch.Tensor:
    """bb_adam_clip_step's scratch, zeroed: its header holds the guard word (ADAM_GUARD_WORD) the finaliser
    sets and adam_guard_check reads."""
    n = (C.c_int64 * len(numels))(*numels)
    nbytes = L.load().bb_adam_clip_workspace_bytes(len(numels), n)
    if nbytes < 0:
        raise L.BBNativeError(f"bb_adam_clip_workspace_bytes rejected {len(numels)} tensors")
    return torch.zeros((nbytes + 7) // 8, dtype=torch.float64, device=device)


ADAM_GUARD_WORD = 2  # BB_ADAM_GUARD_WORD: uint32 words 2 (first bad chunk + 1) and 3 (count) of the header
ADAM_CHUNK = 2048  # elements per gradient-norm chunk


def adam_guard_check(ws: torch.Tensor, numels, names=None, clear: bool = True) -> None:
    """Raise BBNativeError when bb_adam_clip_step's finaliser flagged a gradient-norm chunk partial that was
    not finite or above 1e16 (sum of g^2 over 2,048 elements), naming the tensor and the element range.  One
    device read (a sync); ``clear`` re-arms the word."""
    w = ws.view(torch.int32)[ADAM_GUARD_WORD:ADAM_GUARD_WORD + 2]
    first, count = (int(v) for v in w.tolist())
    if first == 0:
        return
    if clear:
        w.zero_()
    chunk = first - 1
    t, c0 = 0, 0
    for t, n in enumerate(numels):
        nc = -(-int(n) // ADAM_CHUNK)
        if chunk < c0 + nc:
            break
        c0 += nc
    lo = (chunk - c0) * ADAM_CHUNK
    name = names[t] if names is not None and t < len(names) else f"tensor {t}"
    raise L.BBNativeError(f"bb_adam_clip_step guard: {count} gradient-norm chunk partial(s) non-finite or above "
                          f"1e16; first: {name} elements [{lo}, {min(lo + ADAM_CHUNK, int(numels[t]))}) "
                          f"(chunk {chunk})")


def adam_clip_step(params, grads, exp_avgs, exp_avg_sqs, steps, lr: float, beta1: float, beta2: float, eps: float,
                   max_norm: float, ws: torch.Tensor, total_norm: Optional[torch.Tensor] = None) -> None:
    """nn.utils.clip_grad_norm_(params, max_norm) + torch.optim.Adam.step()
    (weight decay 0) in three launches (bb_adam_clip_step): gradients are
    clipped in place, parameters / moments / step counts updated in place."""
    k = len(params)
    if not (len(grads) == len(exp_avgs) == len(exp_avg_sqs) == len(steps) == k) or not 0 < k <= OPT_MAX_TENSORS:
        raise L.BBNativeError(f"adam_clip_step: 1..{OPT_MAX_TENSORS} tensors with all four states")
    for p, g, m, v, s in zip(params, grads, exp_avgs, exp_avg_sqs, steps):
        _need_cuda(p, g, m, v, s)
        if not (p.dtype == g.dtype == m.dtype == v.dtype == s.dtype == torch.float32):
            raise L.BBNativeError("adam_clip_step: f32 tensors only")
        dense = p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))
        if not (dense and p.shape == g.shape and p.stride() == g.stride() == m.stride() == v.stride()):
            raise L.BBNativeError("adam_clip_step: parameter, gradient and moments must share one dense layout")
    numel = (C.c_int64 * k)(*[p.numel() for p in params])
    dev = params[0].device
    L.check(L.load().bb_adam_clip_step(k, _ptrs(params), _ptrs(grads), _ptrs(exp_avgs), _ptrs(exp_avg_sqs),
                                       _ptrs(steps), numel, float(lr), float(beta1), float(beta2), float(eps),
                                       float(max_norm), _p(ws), _p(total_norm), _s(dev)),
            "bb_adam_clip_step")


def cast_multi(dir_: int, srcs, dsts, perms) -> None:
    """bb_cast_multi: dir 0 f32 -> bf16, 1 bf16 -> f32, all tensors in one launch."""
    k = len(srcs)
    numel = (C.c_int64 * k)(*[t.numel() for t in srcs])
    pc = (C.c_int32 * k)(*[p[0] for p in perms])
    ph = (C.c_int32 * k)(*[p[1] for p in perms])
    L.check(L.load().bb_cast_multi(k, int(dir_), _ptrs(srcs), _ptrs(dsts), numel, pc, ph, _s(srcs[0].device)),
            "bb_cast_multi")


# bf16 Linear tails on bb_dropout_forward / bb_linear_bgrad (0: torch's dropout, threshold_backward and bias
# reductions, for A/B)
LINEAR_TAIL = os.environ.get("BB_LINEAR_TAIL", "1") != "0"


def _bgrad_ok(t: torch.Tensor) -> bool:
    return LINEAR_TAIL and t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.is_contiguous()


def _rows_ok(t: torch.Tensor) -> bool:
    """A bf16 matrix whose rows are contiguous and 16-byte aligned (a column slice of a wider one allowed)."""
    return (LINEAR_TAIL and t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2 and t.stride(1) == 1
            and t.stride(0) >= t.shape[1] and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0)


_bgrad_cnt = {}  # (device, stream) -> zeroed uint32 counters of bb_linear_bgrad (re-armed by every launch)
_BGRAD_CNT = 4096
_cnt_owned = {}  # device key -> the counter block of the capture in progress (own_counters)
_cnt_live = weakref.WeakValueDictionary()  # id -> every capture-owned block still referenced (by its graph)


def _dev_key(dev) -> torch.device:
    """A device with its index ('cuda' -> 'cuda:<current>'), the key every per-device table here uses."""
    d = torch.device(dev)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


class own_counters:
    """A counter block of its own for the launches issued inside (a graph capture and its warm-up): the
    hand-off kernels of a captured graph embed its address, so two graphs never share counters through a
    pooled stream handle.  ``block`` is the tensor; keep it alive as long as the graph (PPOAgent stores it with
    the captured entry).  Created zeroed, before any capture starts."""

    def __init__(self, device):
        self.dev = _dev_key(device)
        self.block = None
        self._prev = None

    def __enter__(self):
        if self.dev.type == "cuda":
            self.block = torch.zeros(_BGRAD_CNT, dtype=torch.int32, device=self.dev)
            _cnt_live[id(self.block)] = self.block
            self._prev = _cnt_owned.get(self.dev)
            _cnt_owned[self.dev] = self.block
        return self

    def __exit__(self, *exc):
        if self.dev.type == "cuda":
            if self._prev is None:
                _cnt_owned.pop(self.dev, None)
            else:
                _cnt_owned[self.dev] = self._prev
        return False


def counter_blocks():
    """Every counter block handed out so far (stream-keyed and capture-owned ones alike are re-armed by the
    launches that used them: all zero between steps -- tests check it)."""
    return list(_bgrad_cnt.values()) + list(_cnt_live.values())


def _bgrad_counters(dev: torch.device, need: int) -> torch.Tensor:
    """The zeroed counter block for a hand-off launch: the capture's own (own_counters) when one is open on
    the device, else the stream's (launches on one stream are ordered, and each re-arms the counters it used)."""
    if need > _BGRAD_CNT:
        raise L.BBNativeError(f"linear tails: {need} counters needed (> {_BGRAD_CNT})")
    dk = _dev_key(dev)
    own = _cnt_owned.get(dk)
    if own is not None:
        return own
    stream = torch.cuda.current_stream(dk)
    key = (str(dk), stream.cuda_stream)
    cnt = _bgrad_cnt.get(key)
    if cnt is None:
        if torch.cuda.is_current_stream_capturing():  # zeroed outside capture: a captured fill would re-zero
            raise L.BBNativeError("linear_bgrad: run one eager backward on this stream before capturing")
        cnt = _bgrad_cnt[key] = torch.zeros(_BGRAD_CNT, dtype=torch.int32, device=dk)
    return cnt


def linear_bgrad(gy: torch.Tensor, yd: Optional[torch.Tensor], scale: float = 1.0):
    """(g, db) of bb_linear_bgrad: g = gy * scale where yd > 0 else 0 (yd None: g = gy), db = g.sum(0)."""
    rows, cols = gy.shape
    dev = gy.device
    lib = L.load()
    g = torch.empty_like(gy) if yd is not None else gy
    db = torch.empty(cols, dtype=gy.dtype, device=dev)
    ws = torch.empty((lib.bb_linear_bgrad_workspace_bytes(rows, cols) + 3) // 4, dtype=torch.float32, device=dev)
    cnt = _bgrad_counters(dev, lib.bb_linear_bgrad_counters(cols))
    L.check(lib.bb_linear_bgrad(_p(gy), _p(yd) if yd is not None else None, rows, cols, float(scale), _p(g), _p(db),
                                _p(ws), _p(cnt), _s(dev)), "bb_linear_bgrad")
    return g, db


def linear_bgrad2(gy: torch.Tensor, gy2: torch.Tensor, yd: torch.Tensor):
    """bb_linear_bgrad2: (g, db) of bb_linear_bgrad over [gy | gy2] (two layers' output gradients side by
    side, yd the two layers' joint output), without concatenating them."""
    rows, split = gy.shape
    cols = yd.shape[1]
    if not (_bgrad_ok(gy) and _bgrad_ok(gy2) and _bgrad_ok(yd) and gy2.shape == (rows, cols - split)
            and yd.shape[0] == rows):
        raise L.BBNativeError("linear_bgrad2: contiguous bf16 [rows][split], [rows][cols - split], [rows][cols]")
    dev = gy.device
    lib = L.load()
    g = torch.empty_like(yd)
    db = torch.empty(cols, dtype=gy.dtype, device=dev)
    ws = torch.empty((lib.bb_linear_bgrad_workspace_bytes(rows, cols) + 3) // 4, dtype=torch.float32, device=dev)
    cnt = _bgrad_counters(dev, lib.bb_linear_bgrad_counters(cols))
    L.check(lib.bb_linear_bgrad2(_p(gy), _p(gy2), split, _p(yd), rows, cols, 1.0, _p(g), _p(db), _p(ws), _p(cnt),
                                 _s(dev)), "bb_linear_bgrad2")
    return g, db


WGRAD_MAX = 512 * 512  # bb_linear_wgrad for weights up to this size (the 8,192-column first FC stays hipBLASLt's)


def linear_wgrad(g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """g^T x (autograd's weight gradient of F.linear) on bb_linear_wgrad when the shapes fit, else torch's mm."""
    rows, n = g.shape
    k = x.shape[1]
    if (_bgrad_ok(g) and _rows_ok(x) and x.shape[0] == rows and n % 32 == 0 and k % 32 == 0 and n * k <= WGRAD_MAX
            and 0 < rows <= 16384):
        lib = L.load()
        dev = g.device
        dw = torch.empty((n, k), dtype=g.dtype, device=dev)
        ws = torch.empty((lib.bb_linear_wgrad_workspace_bytes(rows, n, k) + 3) // 4, dtype=torch.float32, device=dev)
        cnt = _bgrad_counters(dev, lib.bb_linear_wgrad_counters(n, k))
        L.check(lib.bb_linear_wgrad(_p(g), _p(x), rows, n, k, x.stride(0), _p(dw), _p(ws), _p(cnt), _s(dev)),
                "bb_linear_wgrad")
        return dw
    return g.t().mm(x)


class LinearReLUFunction(torch.autograd.Function):
    """dropout(relu(F.linear(x, w, b)), p) for 2-D x: the ReLU in hipBLASLt's GEMM epilogue
    (torch._addmm_activation), then -- p > 0, nn.Dropout in training -- bb_dropout_forward in place (its
    Philox generator word ``rng``, advanced on the device by every launch).  Backward: bb_linear_bgrad
    (dropout's masked scale, threshold_backward from the saved output, the bias gradient's sum: one pass),
    then dx = g w, dw = g^T x."""

    @staticmethod
    def forward(ctx, x, weight, bias, p: float = 0.0, rng: Optional[torch.Tensor] = None):
        y = torch._addmm_activation(bias, x, weight.t())
        scale = 1.0
        if p > 0.0:
            if rng is None or y.numel() % 8 or not _bgrad_ok(y):
                raise L.BBNativeError("LinearReLUFunction: dropout needs a bf16 output of 8k elements and rng")
            L.check(L.load().bb_dropout_forward(_p(y), y.numel(), float(p), _p(rng), _s(y.device)),
                    "bb_dropout_forward")
            scale = 1.0 / struct.unpack("f", struct.pack("f", 1.0 - p))[0]  # bb_optim.hip launch_dropout_fwd
        ctx.save_for_backward(x, weight, y)
        ctx.scale = scale
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, y = ctx.saved_tensors
        gy = gy.contiguous()
        if _bgrad_ok(gy) and _bgrad_ok(y) and gy.shape == y.shape:
            g, db = linear_bgrad(gy, y, ctx.scale)
        else:  # (f32 / CPU operands: torch's ops; dropout was applied only on the bf16 path)
            g = torch.ops.aten.threshold_backward(gy, y, 0)
            db = g.sum(0)
        db = db if ctx.needs_input_grad[2] else None
        dx = g.mm(weight) if ctx.needs_input_grad[0] else None
        dw = linear_wgrad(g, x) if ctx.needs_input_grad[1] else None
        return dx, dw, db, None, None


class LinearBiasFunction(torch.autograd.Function):
    """F.linear(x, w, b) for 2-D bf16 x whose backward takes the bias gradient from bb_linear_bgrad (one pass
    over dy) instead of torch's semaphore memset + reduction."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        return torch.addmm(bias, x, weight.t())

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy = gy.contiguous()
        db = None
        if ctx.needs_input_grad[2]:
            db = linear_bgrad(gy, None)[1] if _bgrad_ok(gy) else gy.sum(0)
        dx = gy.mm(weight) if ctx.needs_input_grad[0] else None
        dw = linear_wgrad(gy, x) if ctx.needs_input_grad[1] else None
        return dx, dw, db


class LinearF32Function(torch.autograd.Function):
    """F.linear(x, w, b) for 2-D fp32 x in a training forward (no autocast), with the bias gradient as a GEMV
    (dy^T 1) instead of autograd's dy.sum(0).  torch's sum over the batch runs as a global-memory reduction whose
    semaphores are zeroed by a hipMemsetAsync before each launch; replayed from PPOAgent's captured optimizer step
    that reduction sporadically left its output unwritten (a NaN canary in .grad survived the replay, the
    semaphore counts 16 / 32 sat in its first words) and the Adam guard flagged it -- tools/diag_graph_grad.py:
    95 of 100 replays flagged with the reduction, 0 of 100 (twice) with the GEMV."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        return torch.addmm(bias, x, weight.t())

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gy = gy.contiguous()
        dx = gy.mm(weight) if ctx.needs_input_grad[0] else None
        dw = gy.t().mm(x) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.needs_input_grad[2]:
            db = gy.t().mv(torch.ones(gy.shape[0], dtype=gy.dtype, device=gy.device))
        return dx, dw, db


def linear_f32_train_ok(x: torch.Tensor, weight: torch.Tensor, bias) -> bool:
    """LinearF32Function applies: a 2-D fp32 device input, fp32 weight and bias, gradients recorded."""
    return (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and weight.dtype == torch.float32
            and bias is not None and bias.dtype == torch.float32 and torch.is_grad_enabled()
            and not torch.is_autocast_enabled("cuda"))


class LinearN1Function(torch.autograd.Function):
    """F.linear(x, w, b) for a one-output bf16 Linear (the value head's last layer) on bb_linear_n1_forward /
    _backward: one launch each way instead of torch's bias copy + GEMM and two GEMMs + a reduction."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        _need_cuda(x, weight)
        rows, k = x.shape
        y = torch.empty((rows, 1), dtype=x.dtype, device=x.device)
        L.check(L.load().bb_linear_n1_forward(_p(x), _p(weight), _p(bias), rows, k, x.stride(0), _p(y),
                                              _s(x.device)), "bb_linear_n1_forward")
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        rows, k = x.shape
        dev = x.device
        lib = L.load()
        gy = gy.contiguous()
        dx, dw, db = _n1_backward(gy, x, weight, ctx.has_bias)
        return dx, dw, db


def _n1_backward(gy, x, weight, has_bias: bool):
    """(dx, dW, db) of bb_linear_n1_backward; x may be a column slice (row stride x.stride(0))."""
    rows, k = x.shape
    dev = x.device
    lib = L.load()
    dx = torch.empty((rows, k), dtype=x.dtype, device=dev)
    dw = torch.empty_like(weight)
    db = torch.empty(1, dtype=x.dtype, device=dev) if has_bias else None
    ws = torch.empty((lib.bb_linear_n1_workspace_bytes(rows, k) + 3) // 4, dtype=torch.float32, device=dev)
    cnt = _bgrad_counters(dev, lib.bb_linear_n1_counters(k))
    L.check(lib.bb_linear_n1_backward(_p(gy), _p(x), _p(weight), rows, k, x.stride(0), _p(dx), _p(dw), _p(db), _p(ws),
                                      _p(cnt), _s(dev)), "bb_linear_n1_backward")
    return dx, dw, db


class HeadsFunction(torch.autograd.Function):
    """The policy and value heads (src/models/network.py:106-120 of the reference: Linear(F, 256) -> ReLU -> Linear(256, 192)
    and Linear(F, 128) -> ReLU -> Linear(128, 1)) on the same features h, their first layers as ONE GEMM with
    the ReLU in its epilogue: wp0 / wv0 and bp0 / bv0 must lie back to back in memory (the Linear shadows of
    network.py allocate them so), read as one [384][F] weight and [384] bias.  Then the policy's last layer
    on hipBLASLt (a column slice of the joint output) and the value's on bb_linear_n1_forward.  Backward:
    bb_linear_bgrad (policy bias), bb_linear_wgrad, one GEMM for the policy's hidden gradient,
    bb_linear_n1_backward, bb_linear_bgrad2 (both hidden layers' ReLU masks and biases in one pass), then one
    GEMM for dh (both heads' input gradients summed inside it) and one bb_linear_wgrad for both first-layer
    weights: 7 launches for the 11 the separate layers take (and 3 for 4 forward)."""

    @staticmethod
    def forward(ctx, h, wp0, bp0, wv0, bv0, wp2, bp2, wv2, bv2):
        _need_cuda(h, wp0)
        n0, k = wp0.shape
        n = n0 + wv0.shape[0]
        w_cat = wp0.as_strided((n, k), (k, 1))
        b_cat = bp0.as_strided((n,), (1,))
        y = torch._addmm_activation(b_cat, h, w_cat.t())
        logits = torch.addmm(bp2, y[:, :n0], wp2.t())
        yv = y[:, n0:]
        value = torch.empty((h.shape[0], 1), dtype=h.dtype, device=h.device)
        L.check(L.load().bb_linear_n1_forward(_p(yv), _p(wv2), _p(bv2), h.shape[0], n - n0, n, _p(value),
                                              _s(h.device)), "bb_linear_n1_forward")
        ctx.save_for_backward(h, wp0, wp2, wv2, y)
        ctx.n0 = n0
        ctx.has_bv2 = bv2 is not None
        return logits, value

    @staticmethod
    def backward(ctx, glog, gval):
        h, wp0, wp2, wv2, y = ctx.saved_tensors
        n0 = ctx.n0
        n, k = y.shape[1], h.shape[1]
        glog = glog.contiguous()
        gval = gval.contiguous()
        dbp2 = linear_bgrad(glog, None)[1]
        dwp2 = linear_wgrad(glog, y[:, :n0])
        dyp = glog.mm(wp2)
        dyv, dwv2, dbv2 = _n1_backward(gval, y[:, n0:], wv2, ctx.has_bv2)
        g, db_cat = linear_bgrad2(dyp, dyv, y)
        dh = g.mm(wp0.as_strided((n, k), (k, 1))) if ctx.needs_input_grad[0] else None
        dw_cat = linear_wgrad(g, h)
        return dh, dw_cat[:n0], db_cat[:n0], dw_cat[n0:], db_cat[n0:], dwp2, dbp2, dwv2, dbv2


def heads_ok(h: torch.Tensor, wp0, bp0, wv0, bv0, wp2, bp2, wv2, bv2) -> bool:
    """HeadsFunction applies: bf16 features and shadows, the first layers' weights and biases adjacent."""
    if not (_bgrad_ok(h) and h.shape[0] > 0 and bp0 is not None and bv0 is not None and bp2 is not None):
        return False
    ts = (wp0, bp0, wv0, bv0, wp2, bp2, wv2)
    if any(t.dtype != torch.bfloat16 or not t.is_contiguous() or not t.is_cuda for t in ts):
        return False
    n0, k = wp0.shape
    nv = wv0.shape[0]
    return (wv0.shape[1] == k == h.shape[1] and bp0.numel() == n0 and bv0.numel() == nv
            and wv0.untyped_storage().data_ptr() == wp0.untyped_storage().data_ptr()
            and bv0.untyped_storage().data_ptr() == bp0.untyped_storage().data_ptr()
            and wv0.data_ptr() == wp0.data_ptr() + 2 * n0 * k and bv0.data_ptr() == bp0.data_ptr() + 2 * n0
            and n0 % 32 == 0 and nv % 32 == 0 and k % 32 == 0 and wp2.shape[1] == n0 and wp2.shape[0] % 32 == 0
            and tuple(wv2.shape) == (1, nv) and (n0 + nv) * k <= WGRAD_MAX and h.shape[0] <= 16384)


def linear_n1_ok(x: torch.Tensor, weight: torch.Tensor) -> bool:
    return (_bgrad_ok(x) and weight.dim() == 2 and weight.shape[0] == 1 and weight.shape[1] == x.shape[1]
            and weight.dtype == torch.bfloat16 and weight.is_contiguous() and x.shape[1] % 8 == 0 and x.shape[0] > 0)


class LinearCastFunction(torch.autograd.Function):
    """autocast's f32 -> bf16 casts of the CNN's Linear weights and biases, all
    in one launch, and the bf16 -> f32 casts of their gradients in one launch
    (values identical to autocast's per-tensor casts).  perms[i] = (c, hw)
    stores parameter i's columns, read as [c][hw], in [hw][c] order (the first
    FC weight against the channels_last flatten); (0, 0) = as is."""

    @staticmethod
    def forward(ctx, perms, *params):
        _need_cuda(*params)
        for p in params:
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise L.BBNativeError("LinearCastFunction: contiguous f32 parameters only")
        # one buffer, each slot 256-byte aligned: consecutive parameters whose sizes are multiples of 128
        # elements lie back to back (HeadsFunction reads two heads' layers as one)
        offs, tot = [], 0
        for p in params:
            offs.append(tot)
            tot += (p.numel() + 127) // 128 * 128
        buf = torch.empty(tot, dtype=torch.bfloat16, device=params[0].device)
        outs = [buf[o:o + p.numel()].view(p.shape) for o, p in zip(offs, params)]
        cast_multi(0, params, outs, perms)
        ctx.perms = perms
        ctx.set_materialize_grads(False)  # an unused output leaves its parameter's .grad None, as autocast does
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        idx = [i for i, g in enumerate(grads) if g is not None]
        res = [None] * len(grads)
        if idx:
            gin = [grads[i].to(torch.bfloat16).contiguous() for i in idx]
            outs = [torch.empty(g.shape, dtype=torch.float32, device=g.device) for g in gin]
            cast_multi(1, gin, outs, [ctx.perms[i] for i in idx])
            for i, o in zip(idx, outs):
                res[i] = o
        return (None, *res)
