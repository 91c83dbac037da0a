#!/usr/bin/env python3
"""Micro-benchmark of the HIP BatchNorm kernels (csrc/bb_nn.hip): forward and
backward at the CNN's shapes, NCHW vs NHWC, with and without the folded conv
bias; HIP-event timing, us per call and effective GB/s."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import torch  # noqa: E402

from runtime.kernels import BatchNormReLUFunction  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    N, C = 2048, 128
    for dtype in (torch.bfloat16, torch.float32):
        for nhwc in (False, True):
            for pb in (False, True):
                fmt = torch.channels_last if nhwc else torch.contiguous_format
                x = torch.randn(N, C, 8, 8, device=dev).to(dtype).contiguous(memory_format=fmt).requires_grad_(True)
                w = torch.rand(C, device=dev, requires_grad=True)
                b = torch.randn(C, device=dev, requires_grad=True)
                bias = torch.randn(C, device=dev, requires_grad=True) if pb else None
                rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
                fwd = lambda: BatchNormReLUFunction.apply(x, bias, w, b, rm, rv, 0.1, 1e-5, True)
                y = fwd()
                g = torch.randn_like(y)
                t_f = timeit(fwd)
                t_b = timeit(lambda: torch.autograd.grad(y, [x, w, b] + ([bias] if pb else []), g, retain_graph=True))
                nbytes = x.numel() * x.element_size()
                print(json.dumps({"dtype": str(dtype), "nhwc": nhwc, "pre_bias": pb, "fwd_us": round(t_f, 1),
                                  "bwd_us": round(t_b, 1), "fwd_GBs": round(3 * nbytes / t_f / 1e3, 1),
                                  "bwd_GBs": round(5 * nbytes / t_b / 1e3, 1)}))


if __name__ == "__main__":
    main()
