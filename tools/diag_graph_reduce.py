#!/usr/bin/env python3
"""Diagnostics (not product): do torch's own bias-gradient reductions (sum over the batch, a global-memory
semaphore reduction) survive HIP graph replay?  A pure-torch fp32 MLP shaped like the CNN's FC encoder and heads
(8192 -> 512 -> 256 -> 256/128 -> 192/1, batch 1024) is captured forward + backward (every .grad None before
the captured backward, as PPOAgent's step), then replayed R times with every .grad filled with NaN before each
replay; a replay whose gradients differ from the first replay's (or keep a NaN) is counted, per parameter.
    python tools/diag_graph_reduce.py [replays] [mode]
mode "plain": as above; "noise": an unrelated eager allocation churn between replays; "zero" / "keep": fill
with zeros / leave the gradients as the last replay left them.  Every replay is also checked against an eager
step (rtol 1e-4): "vs_eager" counts replays outside it, per parameter.
"""
import json
import sys

import torch
import torch.nn as nn


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    mode = sys.argv[2] if len(sys.argv) > 2 else "plain"
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

    step()
    torch.cuda.synchronize()
    eager = [p.grad.clone() for p in params]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        step()
    g.replay()
    torch.cuda.synchronize()
    ref = [p.grad.clone() for p in params]
    bad, worst, vs_eager = {}, {}, {}
    first = {n: float((p.grad - e).abs().max() / (e.abs().max() + 1e-30)) for n, p, e in zip(names, params, eager)}
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
        for n, p, q, e in zip(names, params, ref, eager):
            if not torch.allclose(p.grad, e, rtol=1e-4, atol=1e-6):
                vs_eager[n] = vs_eager.get(n, 0) + 1
            if not torch.isfinite(p.grad).all():
                nan_left[n] = nan_left.get(n, 0) + 1
            elif not torch.equal(p.grad, q):
                bad[n] = bad.get(n, 0) + 1
                d = float((p.grad - q).abs().max() / (q.abs().max() + 1e-30))
                worst[n] = max(worst.get(n, 0.0), d)
        ref = [p.grad.clone() for p in params]  # each replay against the one before
    print(json.dumps({"replays": reps, "mode": mode, "nan_left": nan_left, "not_bit_equal": bad,
                      "max_rel_diff": worst,
                      "vs_eager": vs_eager, "first_replay_vs_eager": {n: v for n, v in first.items() if v > 1e-4}}), flush=True)


if __name__ == "__main__":
    main()
