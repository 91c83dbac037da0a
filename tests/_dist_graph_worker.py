"""Worker for test_gpu_train.py's data-parallel graph test (torch.distributed.run,
2 ranks sharing the card over gloo): the HIP-graph-replayed data-parallel
optimizer step (forward + backward graph, all-reduce, clip + Adam graph) against
the eager data-parallel step on the same per-rank minibatches, for dp_overlap "graph-segments" (three graphs:
heads + FC backward, conv-stack backward beside the first bucket's all-reduce, clip + Adam) and "graph-split"
(two graphs around one all-reduce)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from agents import PPOAgent, PPOConfig  # noqa: E402


def _batches(rank, n=6, b=256):
    g = torch.Generator().manual_seed(100 + rank)  # each rank its own samples
    out = []
    for _ in range(n):
        x = (torch.rand(b, 4, 8, 8, generator=g) < 0.4).float()
        mask = (torch.rand(b, 192, generator=g) < 0.3).float()
        mask[:, 0] = 1.0
        act = torch.multinomial(mask, 1, generator=g).squeeze(1)
        old = -3.0 * torch.rand(b, generator=g)
        adv, ret = torch.randn(b, generator=g), torch.randn(b, generator=g)
        out.append((x, mask, act, old, adv, ret))
    return out


def main():
    out = os.environ["BB_TEST_OUT"]
    torch.cuda.set_device(0)  # both ranks on the one GPU of the test box
    # deterministic MIOpen algorithms: its default fp32 weight gradients accumulate split-K partials with
    # atomics, and the two runs compared here would drift apart by that alone
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    cuda = torch.device("cuda", 0)
    report = {}
    for mode, ngraphs in (("graph-segments", 3), ("graph-split", 2)):
        res = {}
        for graphs in (True, False):
            torch.manual_seed(0)
            agent = PPOAgent(PPOConfig(batch_size=512), device=cuda, sample_seed=1)
            agent.dp_overlap = mode
            agent.use_graphs = graphs
            agent.train()
            for m in agent.network.modules():
                if isinstance(m, torch.nn.Dropout):
                    m.p = 0.0
            stats = []
            for batch in _batches(rank):
                stats.append(agent.train_minibatch(*(t.to(cuda) for t in batch)).clone())
            torch.cuda.synchronize()
            flat = torch.cat([p.detach().double().reshape(-1).cpu() for p in agent.network.parameters()])
            res[graphs] = (flat, torch.stack(stats).double().cpu())
            if graphs:
                assert len(agent._graphs) == 1 and len(next(iter(agent._graphs.values()))[0]) == ngraphs
        (fg, sg), (fe, se) = res[True], res[False]
        rel = float((fg - fe).norm() / fe.norm())
        report[mode] = {"checksum": float(fg.sum()), "checksum_eager": float(fe.sum()), "weights_rel": rel,
                        "weights_maxabs": float((fg - fe).abs().max()),
                        "stats_maxabs": float((sg - se).abs().max()), "flat": fg}
    # the two modes compute the same step: segmented and unsegmented weights agree
    a, b = report["graph-segments"].pop("flat"), report["graph-split"].pop("flat")
    report["modes_rel"] = float((a - b).norm() / b.norm())
    with open(os.path.join(out, f"graph_rank{rank}.json"), "w") as f:
        json.dump(report, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
