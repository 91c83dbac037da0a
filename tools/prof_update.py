#!/usr/bin/env python3
"""Steady-state kernel breakdown of one PPO optimizer step (config 3 shape).

Runs ``--warm`` graph-replayed minibatch steps on synthetic inputs, launches a
marker kernel (torch.cuda._sleep), then ``--steps`` timed steps.  Under
``rocprofv3 --kernel-trace`` the kernels after the marker are the steady state;
``--summarize <kernel_trace.csv>`` prints the per-kernel breakdown per step.
"""
import argparse
import collections
import csv
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

FWD_FLOP = 113_049_856


def summarize(path, steps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [k for k, r in enumerate(rows) if "sleep" in r["Kernel_Name"].lower() or "spin" in r["Kernel_Name"].lower()]
    sel = rows[marks[-1] + 1:] if marks else rows[-len(rows) // 3:]
    span = int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])
    acc = collections.defaultdict(lambda: [0, 0])
    for r in sel:
        acc[r["Kernel_Name"]][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        acc[r["Kernel_Name"]][1] += 1
    busy = sum(v[0] for v in acc.values())
    print(f"marker found: {bool(marks)}; window {span/1e6:.2f} ms over {steps} steps = {span/1e3/steps:.1f} us/step; "
          f"kernel busy {100*busy/span:.1f}%; {len(sel)/steps:.1f} kernels/step")
    for k, (d, c) in sorted(acc.items(), key=lambda kv: -kv[1][0])[:40]:
        print(f"{100*d/busy:6.2f}% {c/steps:6.1f}/step {d/c/1e3:8.1f}us {d/1e3/steps:8.1f}us/step  {k[:230]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--warm", type=int, default=20)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--autocast", choices=["none", "bf16"], default="bf16")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--summarize", default=None)
    args = ap.parse_args()
    if args.summarize:
        summarize(args.summarize, args.steps)
        return
    import torch

    from agents import PPOAgent, PPOConfig

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    agent = PPOAgent(PPOConfig(batch_size=args.batch), device=dev, sample_seed=1)
    if args.autocast == "bf16":
        agent.autocast_dtype = torch.bfloat16
    agent.use_graphs = not args.no_graph
    if args.channels_last:
        agent.set_channels_last(True)
    agent.train()
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.rand((B, 4, 8, 8), device=dev, generator=g) < 0.4).float()
    m = (torch.rand((B, 192), device=dev, generator=g) < 0.3).float()
    m[:, 0] = 1.0
    a = torch.multinomial(m, 1, generator=g).squeeze(1)
    lp = -torch.rand(B, device=dev, generator=g) * 4
    adv = torch.randn(B, device=dev, generator=g)
    ret = torch.randn(B, device=dev, generator=g)
    for _ in range(args.warm):
        agent.train_minibatch(x, m, a, lp, adv, ret)
    st = agent.minibatch_inputs(B)  # the captured step's own inputs (PPOAgent.update gathers into them)
    if st is not None:
        for dst, src in zip(st, (x, m, a, lp, adv, ret)):
            dst.copy_(src)
        x, m, a, lp, adv, ret = st
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        agent.train_minibatch(x, m, a, lp, adv, ret)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({"batch": B, "autocast": args.autocast, "graph": not args.no_graph, "channels_last": args.channels_last,
                      "update_step_ms": round(dt * 1e3, 3),
                      "cnn_tflops": round(3 * FWD_FLOP * B / dt / 1e12, 2)}))


if __name__ == "__main__":
    main()
