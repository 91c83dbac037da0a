#!/usr/bin/env python3
"""Time the HIP 3x3 board convolutions (csrc/bb_conv.hip) against torch's
(MIOpen) bf16 channels_last convolution at the PPO minibatch shape: forward,
data gradient and weight gradient per layer shape, HIP events around R
back-to-back launches.  Prints one JSON line per shape."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import torch  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--shapes", default="128x128,64x128")
    args = ap.parse_args()
    from runtime import lib as L
    from runtime.kernels import _p, _s

    lib = L.load()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    for sh in args.shapes.split(","):
        cin, cout = (int(v) for v in sh.split("x"))
        n = args.n
        x = torch.randn((n, cin, 8, 8), device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn((n, cout, 8, 8), device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn((cout, cin, 3, 3), device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        wb = w.bfloat16()
        wf = torch.empty(9 * cin * cout, dtype=torch.bfloat16, device=dev)
        wd = torch.empty_like(wf)
        y = torch.empty((n, cout, 8, 8), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        ws = torch.empty(lib.bb_conv3x3_workspace_bytes(n, cin, cout) // 4, dtype=torch.float32, device=dev)
        dw = torch.empty_like(w)
        s = _s(dev)
        hip = {
            "prep": lambda: lib.bb_conv3x3_prep(_p(w), cin, cout, 1, _p(wf), _p(wd), s),
            "fwd": lambda: lib.bb_conv3x3_forward(_p(x), _p(wf), n, cin, cout, _p(y), s),
            "dgrad": lambda: lib.bb_conv3x3_forward(_p(dy), _p(wd), n, cout, cin, _p(dx), s),
            "wgrad": lambda: lib.bb_conv3x3_wgrad(_p(x), _p(dy), n, cin, cout, _p(ws), 1, _p(dw), s),
        }
        ref = {
            "fwd": lambda: torch.nn.functional.conv2d(x, wb, padding=1),
            "dgrad": lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [1, 1], [1, 1], [1, 1], False,
                                                                 [0, 0], 1, [True, False, False]),
            "wgrad": lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [1, 1], [1, 1], [1, 1], False,
                                                                 [0, 0], 1, [False, True, False]),
        }
        flop = 2.0 * n * 64 * cin * cout * 9
        out = {"shape": f"{cin}->{cout}", "n": n, "gflop_per_op": round(flop / 1e9, 2)}
        for k, fn in hip.items():
            us = timeit(fn, args.reps)
            out[f"hip_{k}_us"] = round(us, 2)
            if k != "prep":
                out[f"hip_{k}_tflops"] = round(flop / us / 1e6, 1)
        for k, fn in ref.items():
            us = timeit(fn, args.reps)
            out[f"miopen_{k}_us"] = round(us, 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
