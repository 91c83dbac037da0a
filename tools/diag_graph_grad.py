#!/usr/bin/env python3
"""Diagnostics (not product): the gradients a replayed fp32 optimizer-step graph leaves, after another agent's
graphed steps ran in the same process (tools/diag_guard.py reproduces the Adam guard that way).

max_grad_norm is set to 1e30, so bb_adam_clip_step's in-place clip multiplies by 1 and every .grad after a
replay is the raw gradient.  A twin agent runs the same minibatches eagerly; per step, the parameters whose
gradient differs from the twin's by more than 1e-2 relative (or is non-finite) are printed with a few values.
    python tools/diag_graph_grad.py [none|graphed|graphed_keep|eager] [steps] [noloss]
Before every replay after the first the graphed agent's .grad tensors (the graph's own) are filled with NaN: a
NaN left after the replay is an output no kernel wrote.
"""
import gc
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import torch  # noqa: E402

from agents import PPOAgent, PPOConfig  # noqa: E402

DEV = torch.device("cuda")
KEEP = []


def batches(n, B, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    out = []
    for _ in range(n):
        x = (torch.rand((B, 4, 8, 8), device=DEV, generator=g) < 0.4).float()
        m = (torch.rand((B, 192), device=DEV, generator=g) < 0.3).float()
        m[:, 0] = 1.0
        a = torch.multinomial(m, 1, generator=g).squeeze(1)
        out.append((x, m, a, -torch.rand(B, device=DEV, generator=g) * 4, torch.randn(B, device=DEV, generator=g),
                    torch.randn(B, device=DEV, generator=g)))
    return out


def make(graphs, batch, **kw):
    torch.manual_seed(3)
    a = PPOAgent(PPOConfig(batch_size=batch, **kw), device=DEV, sample_seed=1)
    for m in a.network.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    a.use_graphs = graphs
    a.train()
    return a


def poison(kind):
    if kind == "none":
        return
    agents = [make(kind != "eager", 256)] if kind != "eager" else [make(False, 256)]
    if kind.startswith("graphed"):
        agents.append(make(False, 256))
    for b in batches(5, 256, 9):
        for ag in agents:
            ag.train_minibatch(*b)
    torch.cuda.synchronize()
    if kind == "graphed_keep":
        KEEP.append(agents)
    del agents
    gc.collect()


class _LinearMV(torch.autograd.Function):
    """F.linear for 2-D fp32 input whose bias gradient is a GEMV (g^T 1) instead of torch's sum(0) reduction."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w.t())

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        ones = torch.ones(g.shape[0], dtype=g.dtype, device=g.device)
        return g.mm(w), g.t().mm(x), g.t().mv(ones)


def _patch_linear():
    orig = torch.nn.functional.linear

    def lin(x, w, b=None):
        if b is not None and x.dim() == 2 and x.is_cuda and x.dtype == torch.float32 and torch.is_grad_enabled():
            return _LinearMV.apply(x, w, b)
        return orig(x, w, b)

    torch.nn.functional.linear = lin


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "graphed"
    if "mvlinear" in sys.argv[3:]:
        _patch_linear()
    poison(kind)
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    # lr 0: the parameters never move, so the graphed and eager agents stay comparable step after step
    g_ag = make(True, 1024, max_grad_norm=1e30, learning_rate=0.0)
    e_ag = make(False, 1024, max_grad_norm=1e30, learning_rate=0.0)
    if "noloss" in sys.argv[3:]:
        g_ag.fused_loss = e_ag.fused_loss = False
    report = {"poison": kind, "steps": []}
    for k, b in enumerate(batches(steps, 1024, 11)):
        if k:
            with torch.no_grad():
                for p in g_ag.network.parameters():
                    if p.grad is not None:
                        p.grad.fill_(float("nan"))
        g_ag.train_minibatch(*b)
        e_ag.train_minibatch(*b)
        torch.cuda.synchronize()
        bad = []
        for (n, p), q in zip(g_ag.network.named_parameters(), e_ag.network.parameters()):
            if p.grad is None or q.grad is None:
                continue
            gg, ge = p.grad.double(), q.grad.double()
            fin = bool(torch.isfinite(gg).all())
            rel = float((gg - ge).norm() / (ge.norm() + 1e-30)) if fin else float("inf")
            if rel > 0.05 and not (fin and gg.norm() < 1e-4):
                flat = gg.flatten()
                idx = torch.nonzero(~torch.isclose(flat, ge.flatten(), rtol=1e-2, atol=1e-6)).flatten()
                bad.append({"param": n, "rel": rel, "n_diff": int(idx.numel()), "numel": flat.numel(),
                            "first_idx": idx[:8].tolist(), "graph_vals": flat[idx[:4]].tolist(),
                            "eager_vals": ge.flatten()[idx[:4]].tolist(), "ptr": hex(p.grad.data_ptr())})
        report["steps"].append({"step": k, "bad": bad})
        print(json.dumps(report["steps"][-1])[:3000], flush=True)


if __name__ == "__main__":
    main()
