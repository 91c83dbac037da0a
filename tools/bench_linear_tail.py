#!/usr/bin/env python3
"""Diagnostics (not product): per-launch time of bb_linear_bgrad / bb_dropout_forward at the update step's
shapes (batch 2048: fc 512 / 256, heads 256 / 128 / 192 / 1) against torch's kernels for the same work, HIP
100 launches captured in a HIP graph.  BBVEC_LIB selects a tuning build (tools/variants.py)."""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"))
from runtime import kernels as K  # noqa: E402
from runtime import lib as L  # noqa: E402


def timed(fn, n=100):
    """GPU time per call: n calls captured in a HIP graph, replayed (host overhead out of the picture)."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        for _ in range(n):
            fn()
    graph.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(5):
        graph.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (5 * n)


def main():
    dev = torch.device("cuda", 0)
    out = {"lib": os.environ.get("BBVEC_LIB", "shipped")}
    for rows, cols, masked in [(2048, 512, True), (2048, 256, True), (2048, 128, True), (2048, 192, False),
                               (2048, 1, False)]:
        gy = torch.randn((rows, cols), device=dev).to(torch.bfloat16)
        yd = torch.randn((rows, cols), device=dev).to(torch.bfloat16).clamp_min(0) if masked else None
        ours = timed(lambda: K.linear_bgrad(gy, yd, 1.1111))
        if masked:
            def ref():
                g = torch.ops.aten.threshold_backward(gy * 1.1111, yd, 0)
                return g.sum(0)
        else:
            def ref():
                return gy.sum(0)
        out[f"bgrad_{cols}{'m' if masked else ''}"] = [round(ours, 2), round(timed(ref), 2)]
    rng = torch.tensor([5, 0, 0, 0], dtype=torch.int64, device=dev)
    for cols in (512, 256):
        y = torch.rand((2048, cols), device=dev).to(torch.bfloat16)

        def ours():
            L.check(L.load().bb_dropout_forward(K._p(y), y.numel(), 0.1, K._p(rng), K._s(dev)), "dropout")
        out[f"dropout_{cols}"] = [round(timed(ours), 2),
                                  round(timed(lambda: torch.nn.functional.dropout(y, 0.1, True)), 2)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
