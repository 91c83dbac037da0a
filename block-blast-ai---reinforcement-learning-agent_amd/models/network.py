"""Policy/value CNN of the Block Blast agent (stays PyTorch-ROCm).

Same architecture, parameter names (``conv_encoder.N.*``, ``fc_encoder.N.*``,
``policy_head.N.*``, ``value_head.N.*``), initialisation and forward semantics
as the reference ``src/models/network.py::BlockBlastNetwork`` (network.py:33-271),
so checkpoints load both ways.  The conv/linear GEMMs run on MFMA through
PyTorch; the masking / softmax / Categorical / sample / entropy tail of
``get_action_and_value`` has a fused HIP kernel (``masked_sample`` below,
csrc/bb_ppo.hip) used on the rollout path.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.distributions import Categorical

N_PARAMS_DEFAULT = 5_290_113  # parameter count of the default net


class BatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d (same parameters, buffers and semantics) whose
    training-mode forward/backward on the GPU are the HIP kernels of
    csrc/bb_nn.hip, with the following ReLU fused when ``relu``.  Other modes
    (eval, CPU, momentum=None) are nn.BatchNorm2d [+ ReLU] itself."""

    use_fused = True

    def __init__(self, num_features: int, relu: bool = False, **kw):
        super().__init__(num_features, **kw)
        self.fuse_relu = relu

    def fusable(self, x: torch.Tensor) -> bool:
        if not (self.use_fused and self.training and self.affine and self.track_running_stats
                and self.momentum is not None):
            return False
        from runtime.kernels import bn_fusable

        return bn_fusable(x)

    def forward(self, x: torch.Tensor, pre_bias: Optional[torch.Tensor] = None, stats=None,
                bwd_slot=None) -> torch.Tensor:
        """BatchNorm2d(x + pre_bias) [-> ReLU]; ``pre_bias`` is a preceding
        convolution's bias that was left out of the convolution; ``stats`` its
        runtime.kernels.StatsSlot (the batch statistics from its store pass);
        ``bwd_slot`` the slot of the convolution reading this output (its data
        gradient's store pass makes this backward's reduction sums)."""
        if self.fusable(x):
            from runtime.kernels import BatchNormReLUFunction

            return BatchNormReLUFunction.apply(x, pre_bias, self.weight, self.bias, self.running_mean,
                                               self.running_var, self.momentum, self.eps, self.fuse_relu,
                                               self.num_batches_tracked, stats, bwd_slot)  # nbt += 1 on device
        if pre_bias is not None:
            x = x + pre_bias.view(1, -1, 1, 1).to(x.dtype)
        y = super().forward(x)
        return F.relu(y) if self.fuse_relu else y


HIP_CONV = os.environ.get("BB_HIP_CONV", "1") != "0"  # 3x3 64/128-channel convs on csrc/bb_conv.hip under bf16
NHWC_FLATTEN = os.environ.get("BB_NHWC_FLATTEN", "1") != "0"  # channels_last trunk: flatten without the layout copy
FUSED_CASTS = os.environ.get("BB_FUSED_CASTS", "1") != "0"  # bf16 Linear weights/biases cast in one launch each way
CAST_PERM_ROW_MAX = 8192  # bb_cast_multi's permuted-row limit (perm_c * perm_hw, include/bbvec.h)
LINEAR_RELU = os.environ.get("BB_LINEAR_RELU", "1") != "0"  # bf16 Linear -> ReLU: the ReLU in the GEMM epilogue
HEADS_FUSED = os.environ.get("BB_HEADS_FUSED", "1") != "0"  # both heads' first layers as one GEMM (HeadsFunction)
PREP_MULTI = os.environ.get("BB_PREP_MULTI", "1") != "0"  # the HIP convs' weight images in one launch
RES_FUSED = os.environ.get("BB_RES_FUSED", "1") != "0"  # ResidualBlock's bn2 + identity + relu in one BatchNorm pass
# ... and the identity path's input gradient added in conv1's data-gradient store pass (no add kernel)
RES_GRAD_FUSED = os.environ.get("BB_RES_GRAD_FUSED", "1") != "0"


# fp32 (no autocast) 64/128-channel 3x3 convs on csrc/bb_conv32.hip (blocked fp32 chains summed in fp64):
# the rollout's train-mode forward stays within north_star's 1e-5 of the fp64 network.  By
# default only where autograd records nothing (the rollout / value forwards); BB_F32_CONV_GRAD=1 also runs
# the update's forward + data gradient on it.
F32_CONV = os.environ.get("BB_F32_CONV", "1") != "0"
F32_CONV_GRAD = os.environ.get("BB_F32_CONV_GRAD", "0") == "1"
# fp32 training Linear layers with the bias gradient as a GEMV (runtime.kernels.LinearF32Function); 0: F.linear,
# whose batch-sum bias gradient is NOT safe under PPOAgent's graph replay (kept only to measure the cost)
F32_LINEAR_GEMV = os.environ.get("BB_F32_LINEAR_GEMV", "1") != "0"


def _f32_conv_on(x: torch.Tensor, conv: nn.Conv2d) -> bool:
    if not (F32_CONV and x.is_cuda and x.dtype == torch.float32 and not torch.is_autocast_enabled("cuda")):
        return False
    if torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad) and not F32_CONV_GRAD:
        return False
    from runtime.kernels import conv3x3_f32_fusable

    return conv3x3_f32_fusable(x, conv)


def _linear(x: torch.Tensor, lin: nn.Linear, weight: Optional[torch.Tensor] = None) -> torch.Tensor:
    """lin(x) (``weight`` replaces lin.weight: the permuted first FC weight).  In the same fp32 forwards as the
    fp32 convolutions (no autocast, nothing recorded for autograd) it runs on bb_linear_f32, whose blocked
    fp32 chains summed in fp64 keep the K = 8,192 first layer's sums within one rounding (hipBLASLt's order
    cost the rollout's logits more than north_star's 1e-5, tools/diag_net_fp32.py)."""
    w = lin.weight if weight is None else weight
    if (F32_CONV and x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 2
            and not torch.is_autocast_enabled("cuda")
            and not (torch.is_grad_enabled() and (x.requires_grad or w.requires_grad))
            and w.shape[0] % 128 == 0 and w.shape[1] % 32 == 0):
        from runtime.kernels import linear_f32

        return linear_f32(x, w, lin.bias)
    if x.is_cuda and F32_LINEAR_GEMV:
        from runtime.kernels import LinearF32Function, linear_f32_train_ok

        if linear_f32_train_ok(x, w, lin.bias):  # the bias gradient as a GEMV (graph-replay safe)
            return LinearF32Function.apply(x, w, lin.bias)
    return F.linear(x, w, lin.bias)


def _hip_conv_on(x: torch.Tensor) -> bool:
    return HIP_CONV and x.is_cuda and torch.is_autocast_enabled("cuda") \
        and torch.get_autocast_dtype("cuda") == torch.bfloat16


def conv_nobias(conv: nn.Conv2d, x: torch.Tensor, images=None, mailbox=None, stats=None,
                bwd_slot=None) -> torch.Tensor:
    """conv(x) without its bias.  Under bf16 autocast on the GPU the 3x3
    layers with 64 or 128 channels in and out run on the HIP kernels
    (runtime.kernels.Conv3x3Function): bf16 NHWC, f32 accumulation, as
    autocast's conv2d.  ``images``: {conv: bf16 weight images} prepared for all
    layers in one launch (BlockBlastNetwork._conv_images)."""
    if _hip_conv_on(x):
        from runtime.kernels import ConvInFunction, Conv3x3Function, conv3x3_fusable, conv_in_fusable

        prep = images.get("prep") if images else None  # the weight images' launch, if not made yet
        if conv3x3_fusable(x, conv):
            if prep is not None:
                prep.run()
            return Conv3x3Function.apply(x, conv.weight, images.get(conv) if images else None, mailbox, stats,
                                         bwd_slot)
        if conv_in_fusable(x, conv):  # the 4 -> 64 input layer: f32 boards in, bf16 NHWC out (+ the images)
            return ConvInFunction.apply(x, conv.weight, prep)
    elif _f32_conv_on(x, conv):
        from runtime.kernels import Conv3x3F32Function

        return Conv3x3F32Function.apply(x, conv.weight)
    return conv._conv_forward(x, conv.weight, None)


def _stats_slot(x: torch.Tensor):
    """A StatsSlot for a HIP board convolution feeding one of our BatchNorms (None off that path)."""
    if not _hip_conv_on(x):
        return None
    from runtime.kernels import StatsSlot

    return StatsSlot()


def conv_bn(conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor, images=None, mailbox=None,
            bwd_slot=None) -> torch.Tensor:
    """bn(conv(x)).  When the BatchNorm runs on the HIP kernels the
    convolution's bias is added inside them (one add on load instead of a
    separate pass, and its gradient comes out of the BatchNorm backward instead
    of a reduction over dy)."""
    if isinstance(bn, BatchNorm2d) and conv.bias is not None and bn.training and x.is_cuda and bn.use_fused:
        slot = _stats_slot(x)
        z = conv_nobias(conv, x, images, mailbox, slot)
        if bn.fusable(z):
            return bn(z, pre_bias=conv.bias, stats=slot, bwd_slot=bwd_slot)
        return bn(z + conv.bias.view(1, -1, 1, 1).to(z.dtype))
    return bn(conv(x))


class ConvStack(nn.Sequential):
    """nn.Sequential (same module indices, so the same state_dict keys) that
    runs each Conv2d -> BatchNorm2d pair through conv_bn."""

    def forward(self, x: torch.Tensor, images=None) -> torch.Tensor:
        mods = list(self)
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, nn.Conv2d) and i + 1 < len(mods) and isinstance(mods[i + 1], BatchNorm2d):
                x = conv_bn(m, mods[i + 1], x, images)
                i += 2
                continue
            x = m(x, images) if isinstance(m, ResidualBlock) else m(x)
            i += 1
        return x


class ResidualBlock(nn.Module):
    """network.py:14-30: conv-bn-relu-conv-bn + identity, relu (the first ReLU
    fused into bn1)."""

    def __init__(self, channels: int):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, channels, kernel_size=3, padding=1)
        self.bn1 = BatchNorm2d(channels, relu=True)
        self.conv2 = nn.Conv2d(channels, channels, kernel_size=3, padding=1)
        self.bn2 = BatchNorm2d(channels)

    def forward(self, x: torch.Tensor, images=None) -> torch.Tensor:
        bn2, conv2 = self.bn2, self.conv2
        fused = (RES_FUSED and isinstance(bn2, BatchNorm2d) and conv2.bias is not None and bn2.training and x.is_cuda
                 and bn2.use_fused)
        mailbox = None
        if fused and RES_GRAD_FUSED and _hip_conv_on(x) and isinstance(self.bn1, BatchNorm2d) \
                and self.conv1.bias is not None and self.bn1.training and self.bn1.use_fused:
            from runtime.kernels import GradMailbox, conv3x3_fusable

            if conv3x3_fusable(x, self.conv1):  # conv1's data gradient adds the identity path's gradient
                mailbox = GradMailbox()
        bslot = _stats_slot(x)  # bn1's backward sums from conv2's data-gradient store pass
        y = conv_bn(self.conv1, self.bn1, x, images, mailbox, bslot)
        if fused:
            slot = _stats_slot(y)
            z = conv_nobias(conv2, y, images, None, slot, bslot)
            from runtime.kernels import BatchNormAddReLUFunction, _bn_layout

            if bn2.fusable(z) and x.dtype == z.dtype and x.shape == z.shape and _bn_layout(x) == _bn_layout(z):
                # bn2 -> + identity -> relu in the BatchNorm apply pass
                return BatchNormAddReLUFunction.apply(z, conv2.bias, x, bn2.weight, bn2.bias, bn2.running_mean,
                                                      bn2.running_var, bn2.momentum, bn2.eps,
                                                      bn2.num_batches_tracked, mailbox, slot)
            # (an unused mailbox stays empty: conv1's data gradient is then the plain one, and autograd adds)
            return F.relu(bn2(z, pre_bias=conv2.bias, stats=slot) + x)
        y = conv_bn(conv2, bn2, y, images)
        return F.relu(y + x)


def _conv_stack(in_ch: int, channels: Sequence[int], batch_norm: bool, residual: bool) -> nn.Sequential:
    layers = []
    for i, out_ch in enumerate(channels):
        layers.append(nn.Conv2d(in_ch, out_ch, kernel_size=3, padding=1))
        if batch_norm:  # ReLU fused into the BatchNorm; the Identity keeps the reference's module indices
            layers.append(BatchNorm2d(out_ch, relu=True))
            layers.append(nn.Identity())
        else:
            layers.append(nn.ReLU())
        if residual and i > 0:  # network.py:86-87
            layers.append(ResidualBlock(out_ch))
        in_ch = out_ch
    return ConvStack(*layers)


def _mlp(in_f: int, hidden: Sequence[int]) -> nn.Sequential:
    layers = []
    for h in hidden:
        layers += [nn.Linear(in_f, h), nn.ReLU(), nn.Dropout(0.1)]
        in_f = h
    return nn.Sequential(*layers)


class BlockBlastNetwork(nn.Module):
    def __init__(
        self,
        board_size: int = 8,
        num_pieces: int = 3,
        conv_channels: Tuple[int, ...] = (64, 128, 128),
        fc_hidden: Tuple[int, ...] = (512, 256),
        action_space_size: int = 192,
        use_residual: bool = True,
        use_batch_norm: bool = True,
    ):
        super().__init__()
        self.board_size = board_size
        self.num_pieces = num_pieces
        self.action_space_size = action_space_size
        self.conv_encoder = _conv_stack(1 + num_pieces, conv_channels, use_batch_norm, use_residual)
        self.fc_encoder = _mlp(conv_channels[-1] * board_size * board_size, fc_hidden)
        self.policy_head = nn.Sequential(nn.Linear(fc_hidden[-1], 256), nn.ReLU(), nn.Linear(256, action_space_size))
        self.value_head = nn.Sequential(nn.Linear(fc_hidden[-1], 128), nn.ReLU(), nn.Linear(128, 1))
        self.apply(self._init_weights)
        # set to a list by PPOAgent's segmented data-parallel step: the next recorded forward cuts autograd at
        # the conv stack's output and appends (output, detached leaf), so backward runs in two segments --
        # heads + FC (which own ~85% of the gradient floats), then the conv stack (which owns ~85% of the
        # backward's FLOPs) -- with the first segment's all-reduce overlapping the second
        self.grad_split: Optional[list] = None

    @staticmethod
    def _init_weights(m: nn.Module) -> None:
        """network.py:122-133: kaiming-uniform (relu) weights, zero biases."""
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            nn.init.kaiming_uniform_(m.weight, nonlinearity="relu")
            if m.bias is not None:
                nn.init.zeros_(m.bias)

    # ------------------------------------------------------------------ core
    def _linears(self):
        return [m for seq in (self.fc_encoder, self.policy_head, self.value_head) for m in seq
                if isinstance(m, nn.Linear)]

    def _linear_shadows(self, h: torch.Tensor, perm0: Optional[Tuple[int, int]]):
        """Under bf16 autocast on the GPU: bf16 copies of every Linear weight and
        bias from one launch (runtime.kernels.LinearCastFunction; autocast
        otherwise casts them one kernel each, and their gradients back one kernel
        each).  perm0 = (c, hw): the first FC weight's columns in (hw, c) order
        for the channels_last flatten.  None when not applicable."""
        if not (FUSED_CASTS and h.is_cuda and torch.is_autocast_enabled("cuda")
                and torch.get_autocast_dtype("cuda") == torch.bfloat16):
            return None
        if perm0 is not None and perm0[0] * perm0[1] > CAST_PERM_ROW_MAX:
            return None  # bb_cast_multi permutes one row per workgroup through LDS: autocast's path instead
        lins = self._linears()
        entries = [(m, kind) for m in lins for kind in (("w", "b") if m.bias is not None else ("w",))]
        heads = self._head_pair()
        if heads is not None:  # the heads' first weights, then their biases, back to back (HeadsFunction)
            p0, v0 = heads
            tail = [(p0, "w"), (v0, "w"), (p0, "b"), (v0, "b")]
            entries = [e for e in entries if e not in tail] + tail
        params, perms = [], []
        for m, kind in entries:
            first = perm0 is not None and len(self.fc_encoder) and m is self.fc_encoder[0] and kind == "w"
            params.append(m.weight if kind == "w" else m.bias)
            perms.append(perm0 if first else (0, 0))
        if not params or len(params) > 48 or any(p.dtype != torch.float32 or not p.is_contiguous() for p in params):
            return None
        from runtime.kernels import LinearCastFunction

        outs = dict(zip(entries, LinearCastFunction.apply(tuple(perms), *params)))
        return {m: (outs[(m, "w")], outs.get((m, "b"))) for m in lins}

    def _head_pair(self):
        """(policy_head[0], value_head[0]) when both heads are Linear -> ReLU -> Linear with biases (the
        reference's heads) and HeadsFunction may run them, else None."""
        p, v = list(self.policy_head), list(self.value_head)
        shape = lambda s: (len(s) == 3 and isinstance(s[0], nn.Linear) and isinstance(s[1], nn.ReLU)
                           and isinstance(s[2], nn.Linear) and s[0].bias is not None and s[2].bias is not None)
        if HEADS_FUSED and LINEAR_RELU and shape(p) and shape(v) and v[2].out_features == 1:
            return p[0], v[0]
        return None

    def _heads(self, h: torch.Tensor, sh):
        """(logits, value (B, 1)) from HeadsFunction when it applies, else None."""
        pair = self._head_pair() if sh is not None and h.dim() == 2 else None
        if pair is None:
            return None
        from runtime import kernels as K

        args = (*sh[pair[0]], *sh[pair[1]], *sh[self.policy_head[2]], *sh[self.value_head[2]])
        if not K.heads_ok(h, *args):
            return None
        return K.HeadsFunction.apply(h, *args)

    def _dropout_after(self, mods, i: int, z: torch.Tensor):
        """(p, rng) when mods[i] is an nn.Dropout the bf16 Linear tail applies itself (bb_dropout_forward),
        else None.  p = 0 in eval mode (nothing drawn)."""
        from runtime.kernels import LINEAR_TAIL

        if not (LINEAR_TAIL and i < len(mods) and isinstance(mods[i], nn.Dropout) and z.is_cuda):
            return None
        d = mods[i]
        p = float(d.p) if d.training else 0.0
        if not 0.0 <= p < 1.0:
            return None
        return p, (self._dropout_rng(z.device) if p > 0.0 else None)

    def _dropout_rng(self, dev: torch.device) -> torch.Tensor:
        """The device generator word {seed, offset, 0, 0} of bb_dropout_forward (one per network and
        device; the launches advance the offset).  Seeded from torch.initial_seed(), so torch.manual_seed
        reproduces the masks.  Made outside graph capture (the first training step's eager run)."""
        rngs = self.__dict__.setdefault("_drop_rngs", {})
        dev = torch.device(dev)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        key = str(dev)
        if key not in rngs:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("BlockBlastNetwork: run one eager training step before capturing (dropout state)")
            seed = (torch.initial_seed() * 0x9E3779B97F4A7C15 + len(rngs) + 1) & ((1 << 63) - 1)
            rngs[key] = torch.tensor([seed, 0, 0, 0], dtype=torch.int64, device=dev)
        return rngs[key]

    def _run(self, seq: nn.Sequential, z: torch.Tensor, sh, skip: int = 0) -> torch.Tensor:
        """seq(z), its Linear layers on the bf16 shadows ``sh`` when given; a
        Linear followed by a ReLU then runs as one GEMM with the ReLU in its
        epilogue (LinearReLUFunction), with a following Dropout applied by the same
        function.  skip: modules seq[:skip] were applied already."""
        mods = list(seq)
        i = skip
        while i < len(mods):
            m = mods[i]
            if sh is not None and isinstance(m, nn.Linear):
                if LINEAR_RELU and i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU) and z.dim() == 2:
                    from runtime.kernels import LinearReLUFunction

                    drop = self._dropout_after(mods, i + 2, z)
                    z = LinearReLUFunction.apply(z, *sh[m], *(drop or ()))
                    i += 3 if drop is not None else 2
                    continue
                from runtime import kernels as K

                if K.LINEAR_TAIL and z.dim() == 2 and K.linear_n1_ok(z, sh[m][0]):
                    z = K.LinearN1Function.apply(z, *sh[m])  # the value head's one-output layer
                elif K.LINEAR_TAIL and z.dim() == 2 and sh[m][1] is not None:
                    z = K.LinearBiasFunction.apply(z, *sh[m])
                else:
                    z = F.linear(z, *sh[m])
            elif isinstance(m, nn.Linear):
                z = _linear(z, m)
            else:
                z = m(z)
            i += 1
        return z

    def _conv_images(self, x: torch.Tensor):
        """Under bf16 autocast on the GPU: the bf16 weight images of every HIP
        board convolution, all layers in one launch (bb_conv3x3_prep_multi)
        instead of one prep launch per layer.  None when not applicable."""
        if not (PREP_MULTI and self.training and _hip_conv_on(x)):  # eval: conv_bn runs torch's convolutions
            return None
        from runtime.kernels import conv3x3_fusable, conv3x3_prep_multi

        probe = x[:1]  # 8x8 boards: every layer sees the same geometry
        convs = [m for m in self.conv_encoder.modules() if isinstance(m, nn.Conv2d) and conv3x3_fusable(probe, m)]
        if not convs or len(convs) > 16:
            return None
        from runtime.kernels import conv_in_fusable

        first = self.conv_encoder[0] if len(self.conv_encoder) else None
        if isinstance(first, nn.Conv2d) and conv_in_fusable(x, first):
            # the input layer's forward launch builds the images too (bb_conv_in_forward_prep); a HIP
            # convolution reached first launches them on its own
            imgs, job = conv3x3_prep_multi([c.weight for c in convs], defer=True)
            out = dict(zip(convs, imgs))
            out["prep"] = job
            return out
        return dict(zip(convs, conv3x3_prep_multi([c.weight for c in convs])))

    def _trunk(self, x: torch.Tensor):
        """x: (B, 4, 8, 8) -> (fc features (B, fc_hidden[-1]), Linear shadows or None)."""
        h = self.conv_encoder(x, self._conv_images(x))
        if self.grad_split is not None and torch.is_grad_enabled() and h.requires_grad:
            hd = h.detach().requires_grad_(True)
            self.grad_split.append((h, hd))
            h = hd
        lin0 = self.fc_encoder[0] if len(self.fc_encoder) else None
        if (NHWC_FLATTEN and isinstance(lin0, nn.Linear) and h.is_cuda
                and h.is_contiguous(memory_format=torch.channels_last) and not h.is_contiguous()):
            # channels_last activations: flatten in (h, w, c) order (a view, no copy) against the
            # first FC weight's columns permuted the same way -- the reference's (c, h, w) flatten
            # (network.py:163) copied 33.5 MB per minibatch forward and left its gradient in the
            # other layout for the ReLU backward of the last residual block
            n, c, hh, ww = h.shape
            o = lin0.out_features
            flat = h.permute(0, 2, 3, 1).reshape(n, hh * ww * c)
            sh = self._linear_shadows(h, (c, hh * ww))
            if sh is not None:  # the permuted bf16 weight comes out of the multi-tensor cast
                mods = list(self.fc_encoder)
                fuse = LINEAR_RELU and len(mods) > 1 and isinstance(mods[1], nn.ReLU)
                if fuse:
                    from runtime.kernels import LinearReLUFunction

                    drop = self._dropout_after(mods, 2, flat)
                    z = LinearReLUFunction.apply(flat, *sh[lin0], *(drop or ()))
                    skip = 3 if drop is not None else 2
                else:
                    z, skip = F.linear(flat, *sh[lin0]), 1
                return self._run(self.fc_encoder, z, sh, skip), sh
            wp = lin0.weight.view(o, c, hh, ww).permute(0, 2, 3, 1)
            if torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16:
                wp = wp.to(torch.bfloat16, memory_format=torch.contiguous_format)  # autocast's cast + the permute, one pass
            w = wp.reshape(o, hh * ww * c)
            return self._run(self.fc_encoder, _linear(flat, lin0, w), None, 1), None
        sh = self._linear_shadows(h, None)
        return self._run(self.fc_encoder, h.reshape(h.shape[0], -1), sh), sh

    def trunk(self, x: torch.Tensor) -> torch.Tensor:
        """x: (B, 4, 8, 8) -> fc features (B, fc_hidden[-1])."""
        return self._trunk(x)[0]

    def raw(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Unmasked logits (B, 192) and value (B,) from the stacked input."""
        h, sh = self._trunk(x)
        heads = self._heads(h, sh)
        if heads is not None:
            return heads[0], heads[1].squeeze(-1)
        return self._run(self.policy_head, h, sh), self._run(self.value_head, h, sh).squeeze(-1)

    @staticmethod
    def stack_input(board: torch.Tensor, pieces: torch.Tensor) -> torch.Tensor:
        if board.dim() == 3:
            board = board.unsqueeze(1)
        return torch.cat([board, pieces], dim=1)

    # ------------------------------------------------- reference interface
    def forward(self, board: torch.Tensor, pieces: torch.Tensor,
                action_mask: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        """network.py:135-182: masked logits (invalid -> -inf) and value."""
        logits, value = self.raw(self.stack_input(board, pieces))
        if action_mask is not None:
            logits = logits + torch.where(action_mask.bool(), torch.zeros_like(logits),
                                          torch.full_like(logits, float("-inf")))
        return logits, value

    def get_action_and_value(self, board, pieces, action_mask, action=None, deterministic: bool = False):
        """network.py:184-230 (torch path; differentiable, used by the update)."""
        logits, value = self.forward(board, pieces, action_mask)
        action, log_prob, entropy = categorical_tail(logits, action_mask, action, deterministic)
        return action, log_prob, entropy, value

    def _masked_entropy(self, probs: torch.Tensor, action_mask: torch.Tensor) -> torch.Tensor:
        return masked_entropy(probs, action_mask)

    def get_value(self, board: torch.Tensor, pieces: torch.Tensor) -> torch.Tensor:
        """network.py:264-271."""
        return self.forward(board, pieces)[1]


def masked_entropy(probs: torch.Tensor, action_mask: torch.Tensor) -> torch.Tensor:
    """network.py:232-262: entropy of the mask-renormalised distribution."""
    mask = action_mask.bool().float()
    masked = probs * mask
    norm = masked / masked.sum(dim=-1, keepdim=True).clamp(min=1e-10)
    return -(norm * torch.log(norm.clamp(min=1e-10)) * mask).sum(dim=-1)


def categorical_tail(masked_logits: torch.Tensor, action_mask: torch.Tensor, action=None,
                     deterministic: bool = False):
    """softmax -> Categorical(probs) -> sample/argmax -> log_prob, masked entropy
    (network.py:210-230), differentiable torch ops."""
    probs = F.softmax(masked_logits, dim=-1)
    dist = Categorical(probs=probs)
    if action is None:
        action = torch.argmax(probs, dim=-1) if deterministic else dist.sample()
    return action, dist.log_prob(action), masked_entropy(probs, action_mask)


def count_params(net: nn.Module) -> int:
    return sum(p.numel() for p in net.parameters())
