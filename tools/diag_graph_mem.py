#!/usr/bin/env python3
"""Diagnostics (not product): which earlier allocations the tensors made after a graph's second replay reuse,
for tools/diag_graph_reduce.py's "keep" pattern (the third replay onward then computes trunk.0.bias wrong).
The allocator's history (torch.cuda.memory._record_memory_history, C++ and Python frames) is searched for
allocations made before or during the capture whose address ranges overlap the clones made after replay 2;
their stacks name the op whose memory the graph still reads."""
import json
import sys

import torch
import torch.nn as nn


def main():
    dev = torch.device("cuda")
    torch.cuda.memory._record_memory_history(max_entries=200000, context="all", stacks="all")
    torch.manual_seed(0)
    trunk = nn.Sequential(nn.Linear(8192, 512), nn.ReLU(), nn.Linear(512, 256), nn.ReLU()).to(dev)
    ph = nn.Sequential(nn.Linear(256, 256), nn.ReLU(), nn.Linear(256, 192)).to(dev)
    vh = nn.Sequential(nn.Linear(256, 128), nn.ReLU(), nn.Linear(128, 1)).to(dev)
    params = [p for m in (trunk, ph, vh) for p in m.parameters()]
    x = torch.randn(1024, 8192, device=dev)
    w = torch.randn(1024, 192, device=dev)
    r = torch.randn(1024, device=dev)

    def step():
        for p in params:
            p.grad = None
        h = trunk(x)
        loss = (ph(h) * w).sum() / 1024 + ((vh(h).squeeze(-1) - r) ** 2).mean()
        loss.backward()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        step()
    n_before = len(torch.cuda.memory._snapshot()["device_traces"][0])
    g.replay()
    torch.cuda.synchronize()
    keep = [[p.grad.clone() for p in params]]
    g.replay()
    torch.cuda.synchronize()
    keep.append([p.grad.clone() for p in params])
    ranges = [(t.data_ptr(), t.data_ptr() + t.numel() * 4) for t in keep[1]]
    g.replay()
    torch.cuda.synchronize()
    b = trunk[0].bias.grad.clone()
    for p in params:
        p.grad = None
    step()
    ok = float((b - trunk[0].bias.grad).abs().max() / trunk[0].bias.grad.abs().max())
    snap = torch.cuda.memory._snapshot()
    tr = snap["device_traces"][0][:n_before]
    hits = []
    for ev in tr:
        if ev["action"] != "alloc":
            continue
        a0, a1 = ev["addr"], ev["addr"] + ev["size"]
        for i, (c0, c1) in enumerate(ranges):
            if a0 < c1 and c0 < a1:
                frames = [f"{f['name']} ({f['filename'].split('/')[-1]}:{f['line']})" for f in ev.get("frames", [])]
                keyf = [f for f in frames if any(k in f for k in ("at::", "c10::", "hip", ".py", "blas", "Blas"))]
                hits.append({"clone": i, "addr": hex(a0), "size": ev["size"], "stream": ev.get("stream"),
                             "frames": keyf[:14]})
    print(json.dumps({"replay3_trunk0_bias_rel": ok, "hits": hits}, indent=1))


if __name__ == "__main__":
    main()
