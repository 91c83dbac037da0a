#!/usr/bin/env python3
"""Diagnostics (not product): do torch's own bias-gradient reductions (sum over the batch, a global-memory
semaphore reduction) survive HIP graph replay?  A pure-torch fp32 MLP shaped like the CNN's FC encoder and heads
(8192 -> 512 -> 256 -> 256/128 -> 192/1, batch 1024) is captured forward + backward (every .grad None before
the captured backward, as PPOAgent's step), then replayed R times with every .grad filled with NaN before each
replay; a replay whose gradients differ from the first replay's (or keep a NaN) is counted, per parameter.
    python tools/diag_graph_reduce.py [replays] [mode]
mode "plain": as above; "noise": an unrelated eager allocation churn between replays; "zero" / "keep": fill
with zeros / leave the gradients as the last replay left them.  The first four replays are checked against an
eager step run at the end ("first_replays_vs_eager": max relative deviations above 1e-4).  Third argument
"pre": one eager step on the default stream before the side-stream warm-up; "prenone": every .grad set to None before
the capture begins (PyTorch's documented whole-network pattern) instead of inside it.
"""
import json
import sys

import torch
import torch.nn as nn


def sum_only(reps: int, shape):
    """The bias-gradient reduction alone: y = g.sum(0) captured, replayed with a clone of y kept after each replay
    (the "keep" pattern); every replay against eager."""
    dev = torch.device("cuda")
    torch.manual_seed(0)
    g = torch.randn(shape, device=dev)
    ref = g.sum(0)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            y = g.sum(0)
    torch.cuda.current_stream().wait_stream(side)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=side):
        y = g.sum(0)
    keep, bad = [], []
    for k in range(reps):
        gr.replay()
        torch.cuda.synchronize()
        d = float((y - ref).abs().max() / ref.abs().max())
        if d > 1e-5:
            bad.append((k + 1, d))
        keep.append(y.clone())
    print(json.dumps({"mode": "sumonly", "shape": list(shape), "bad_replays": bad[:10], "n_bad": len(bad)}), flush=True)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    mode = sys.argv[2] if len(sys.argv) > 2 else "plain"
    if mode == "sumonly":
        for shape in ((1024, 512), (1024, 256), (4096, 512), (1024, 8192)):
            sum_only(reps, shape)
        return
    if "mv" in sys.argv[3:]:  # the bias gradients as GEMVs (tools/diag_graph_grad.py _LinearMV)
        sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
        from diag_graph_grad import _patch_linear

        _patch_linear()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    trunk = nn.Sequential(nn.Linear(8192, 512), nn.ReLU(), nn.Linear(512, 256), nn.ReLU()).to(dev)
    ph = nn.Sequential(nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 192)).to(dev)
    vh = nn.Sequential(nn.Linear(256, 128), nn.ReLU(), nn.Linear(128, 1)).to(dev)
    params = [p for m in (trunk, ph, vh) for p in m.parameters()]
    names = [f"{k}.{n}" for k, m in (("trunk", trunk), ("ph", ph), ("vh", vh)) for n, _ in m.named_parameters()]
    x = torch.randn(1024, 8192, device=dev)
    w = torch.randn(1024, 192, device=dev)
    r = torch.randn(1024, device=dev)

    def step():
        for p in params:
            p.grad = None
        h = trunk(x)
        loss = (ph(h) * w).sum() / 1024 + ((vh(h).squeeze(-1) - r) ** 2).mean()
        loss.backward()

    if "pre" in sys.argv[3:]:  # one eager step on the default stream first (allocator history)
        step()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(side)
    if "prenone" in sys.argv[3:]:  # the warm-up's gradients freed before the capture, not inside it
        for p in params:
            p.grad = None
        torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        step()
    g.replay()
    torch.cuda.synchronize()
    if mode in ("quiet", "alloc"):
        # quiet: replays with no allocation in between; alloc: one eager allocation churn after the first replay
        if mode == "alloc":
            junk = [torch.full((s,), 7.0, device=dev) for s in (512, 256, 65536, 256, 49152, 192, 4194304, 131072)]
            del junk
        for _ in range(9):
            g.replay()
        torch.cuda.synchronize()
        got = [p.grad.clone() for p in params]
        for p in params:
            p.grad = None
        step()
        torch.cuda.synchronize()
        dev_ = {n: float((a - p.grad).abs().max() / (p.grad.abs().max() + 1e-30)) for n, a, p in zip(names, got, params)}
        print(json.dumps({"mode": mode, "replay10_vs_eager": {n: v for n, v in dev_.items() if v > 1e-4}}), flush=True)
        return
    ref = [p.grad.clone() for p in params]
    hist = [ref]
    bad, worst = {}, {}
    nan_left = {}
    for k in range(reps):
        with torch.no_grad():
            for p in params:
                if mode in ("plain", "noise"):
                    p.grad.fill_(float("nan"))
                elif mode == "zero":
                    p.grad.zero_()
        if mode == "noise":
            junk = [torch.empty(1 << s, device=dev).fill_(3.0) for s in range(8, 20)]
            del junk
        g.replay()
        torch.cuda.synchronize()
        for n, p, q in zip(names, params, ref):
            if not torch.isfinite(p.grad).all():
                nan_left[n] = nan_left.get(n, 0) + 1
            elif not torch.equal(p.grad, q):
                bad[n] = bad.get(n, 0) + 1
                d = float((p.grad - q).abs().max() / (q.abs().max() + 1e-30))
                worst[n] = max(worst.get(n, 0.0), d)
        ref = [p.grad.clone() for p in params]  # each replay against the one before
        if len(hist) < 4:
            hist.append(ref)
    # the eager reference last, with the graph's gradient tensors set aside (the replays keep writing theirs)
    gsave = [p.grad for p in params]
    step()
    torch.cuda.synchronize()
    eager = [p.grad.clone() for p in params]
    first = {}
    for i, h in enumerate(hist):
        for n, a, e in zip(names, h, eager):
            d = float((a - e).abs().max() / (e.abs().max() + 1e-30))
            if d > 1e-4:
                first[f"replay{i + 1}:{n}"] = d
    del gsave
    print(json.dumps({"replays": reps, "mode": mode, "nan_left": nan_left, "not_bit_equal": bad,
                      "max_rel_diff": worst,
                      "first_replays_vs_eager": first}), flush=True)


if __name__ == "__main__":
    main()
