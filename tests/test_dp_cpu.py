"""Data-parallel optimizer step on a 2-rank gloo group (CPU): the bucketed all-reduce that backward issues
(PPOAgent._dp_buckets: post-accumulate-grad hooks, one async all-reduce per bucket of the flat gradient
buffer) against the gradient of the concatenated minibatch on one process.

With the network in eval mode (BatchNorm on running statistics, dropout off) every sample's loss term is
independent of the others, and the PPO loss is a mean over the minibatch (ppo.py:372-392), so the average
of the two ranks' minibatch gradients equals the gradient of their concatenation: the per-rank minibatch
of training.minibatch_scope per_gpu reproduces one step on a world x batch_size
minibatch.  (In train mode the BatchNorm batch statistics are per rank: a documented deviation.)"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B = 48


def _data(n):
    g = torch.Generator().manual_seed(7)
    x = (torch.rand(n, 4, 8, 8, generator=g) < 0.4).float()
    mask = (torch.rand(n, 192, generator=g) < 0.3).float()
    mask[:, 5] = 1.0
    act = torch.multinomial(mask, 1, generator=g).squeeze(1)
    old = -3.0 * torch.rand(n, generator=g)
    adv, ret = torch.randn(n, generator=g), torch.randn(n, generator=g)
    return x, mask, act, old, adv, ret


def _agent():
    from agents import PPOAgent, PPOConfig

    torch.manual_seed(0)
    agent = PPOAgent(PPOConfig(batch_size=B), device=torch.device("cpu"), sample_seed=1)
    agent.eval()
    return agent


def _worker(rank, world, port, q, mode="graph-split"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    agent = _agent()
    agent.dp_overlap = mode
    agent.dp_bucket_floats = 1 << 19  # several buckets over the 5.29 M gradient floats
    full = _data(world * B)
    mine = tuple(t[rank * B:(rank + 1) * B] for t in full)
    seen = {}
    orig_finish, orig_clip = agent._dp_finish, agent._clip_and_step

    def finish(w):  # every bucket must have been issued by the hooks, during backward
        st = agent._dp_hooks[1]
        seen["buckets"], seen["issued_in_backward"] = len(st), sum(1 for b in st if b[4])
        orig_finish(w)

    def clip():
        seen["grad"] = agent._flat_grad.clone()
        orig_clip()

    agent._dp_finish, agent._clip_and_step = finish, clip
    if mode == "graph-segments":  # record the order: FC bucket issued before the conv-stack backward ran
        calls = []
        real_ar = dist.all_reduce

        def all_reduce(t, *a, **k):
            calls.append(("all_reduce", t.numel(), agent.network.conv_encoder[0].weight.grad is not None
                          and bool(agent.network.conv_encoder[0].weight.grad.abs().sum() > 0)))
            return real_ar(t, *a, **k)

        import agents.ppo as P
        P.dist.all_reduce = all_reduce
    loss, _ = agent._minibatch_loss(*mine)
    agent._optimizer_step(loss)
    # the reference: one process, the concatenated minibatch, plain autograd
    ref = _agent()
    ref.dp_overlap = "graph-split"  # plain autograd: no segment cut in the reference's forward
    ref_loss, _ = ref._minibatch_loss(*full)
    params = [p for p in ref.network.parameters() if p.requires_grad]
    grads = torch.autograd.grad(ref_loss, params)
    err, scale = 0.0, 0.0
    for (p, off, _n), g in zip(agent._flat_layout, grads):
        got = torch.as_strided(seen["grad"], p.size(), p.stride(), off)
        err = max(err, float((got - g).abs().max()))
        scale = max(scale, float(g.abs().max()))
    w = torch.cat([p.detach().reshape(-1) for p in agent.network.parameters()])
    if mode == "graph-segments":
        P.dist.all_reduce = real_ar
        # two buckets: the heads + FC one issued before any conv-stack gradient existed, then the conv one
        split = agent._dp_split_offset()
        n = agent._flat_grad.numel()
        ok = [c[1] for c in calls] == [n - split, split] and calls[0][2] is False and calls[1][2] is True
        seen["buckets"], seen["issued_in_backward"] = (2, 2) if ok else (len(calls), -1)
    q.put((rank, seen["buckets"], seen["issued_in_backward"], err, scale, float(w.double().sum())))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_segmented_backward_equals_concatenated_minibatch(world):
    """dp_overlap "graph-segments" (the default) in its eager form: backward cut at the conv stack's output,
    the heads + FC bucket all-reduced before the conv-stack backward runs, then the conv bucket; the averaged
    gradient equals the concatenated minibatch's and the replicas stay identical (2 and 4 gloo ranks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29200 + world * 7 + (os.getpid() % 400)
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "graph-segments")) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, nb, issued, err, scale, _ in res:
        assert nb == 2 and issued == 2, (rank, nb, issued)
        assert err <= 1e-5 * scale + 1e-7, (rank, err, scale)
    assert all(r[5] == res[0][5] for r in res)  # replicas identical after the step


def test_bucketed_allreduce_equals_concatenated_minibatch():
    """dp_overlap "graph-split" / "capture" in their eager form: the post-accumulate-grad hooks' buckets."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 500)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for rank, nb, issued, err, scale, _ in res:
        assert nb > 2 and issued == nb, (rank, nb, issued)  # all buckets overlapped with backward
        assert err <= 1e-5 * scale + 1e-7, (rank, err, scale)  # == the concatenated minibatch's gradient
    assert res[0][5] == pytest.approx(res[1][5], rel=0, abs=0)  # replicas identical after the step
