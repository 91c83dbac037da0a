"""Every gradient a replayed optimizer-step graph leaves is written by that replay and equals the eager step's.

Regression test for the Adam guard trip of round 6: torch's batch-sum reduction for the fp32 Linear bias
gradients (a global-memory semaphore reduction zeroed by a hipMemsetAsync) sporadically left its output
unwritten when replayed from PPOAgent's captured step.  The fp32 Linear layers now take their bias gradient as a
GEMV (runtime.kernels.LinearF32Function).  Here every .grad the graph owns is filled with NaN before each
replay (a NaN left afterwards is an output no kernel wrote), lr is 0 and the clip threshold 1e30 (the graphed
and eager twins stay comparable and the in-place clip multiplies by 1), and each replay's gradients are compared
with the eager twin's."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _batches(n, B, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    out = []
    for _ in range(n):
        x = (torch.rand((B, 4, 8, 8), device=dev, generator=g) < 0.4).float()
        m = (torch.rand((B, 192), device=dev, generator=g) < 0.3).float()
        m[:, 0] = 1.0
        a = torch.multinomial(m, 1, generator=g).squeeze(1)
        out.append((x, m, a, -torch.rand(B, device=dev, generator=g) * 4, torch.randn(B, device=dev, generator=g),
                    torch.randn(B, device=dev, generator=g)))
    return out


def _agent(dev, graphs, autocast):
    from agents import PPOAgent, PPOConfig

    torch.manual_seed(3)
    a = PPOAgent(PPOConfig(batch_size=1024, max_grad_norm=1e30, learning_rate=0.0), device=dev, sample_seed=1)
    for m in a.network.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    a.use_graphs = graphs
    a.autocast_dtype = autocast
    a.train()
    return a


@pytest.mark.parametrize("autocast", [None, torch.bfloat16])
def test_replayed_step_writes_every_gradient(cuda, autocast):
    g_ag, e_ag = _agent(cuda, True, autocast), _agent(cuda, False, autocast)
    tol = 1e-2 if autocast is None else 5e-2
    for k, b in enumerate(_batches(24, 1024, 11, cuda)):
        if k:
            with torch.no_grad():
                for p in g_ag.network.parameters():
                    if p.grad is not None:
                        p.grad.fill_(float("nan"))
        g_ag.train_minibatch(*b)
        e_ag.train_minibatch(*b)
        torch.cuda.synchronize()
        for (n, p), q in zip(g_ag.network.named_parameters(), e_ag.network.parameters()):
            assert p.grad is not None and q.grad is not None, n
            assert bool(torch.isfinite(p.grad).all()), f"step {k}: {n} keeps unwritten (NaN canary) elements"
            ref = q.grad.double()
            scale = float(ref.norm())
            if scale < 1e-4:  # the conv biases folded into BatchNorm: zero up to rounding
                continue
            rel = float((p.grad.double() - ref).norm()) / scale
            assert rel < tol, f"step {k}: {n} graph vs eager rel {rel:.3g}"
    g_ag.check_optimizer_guard()
