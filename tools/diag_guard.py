#!/usr/bin/env python3
"""Diagnostics (not product): which gradient trips bb_adam_clip_step's guard in the training driver.

Runs training.train on tests/test_gpu_train.py's config (512 envs, fp32, 16 optimizer steps per update) with
PPOAgent._clip_and_step wrapped: before every eager clip + Adam (warm-up / capture steps with graphs, every
step without) it records each parameter gradient's norm, max |g| and non-finite count.  Prints one JSON object
per mode: the records of tensors whose norm is non-finite or above 1e6, and the guard's verdict.
    python tools/diag_guard.py [graphs|eager|both] [none|nan|graphed]
The second argument first poisons the process: "nan" fills ~8 GB of the caching allocator's blocks with NaN and
frees them (a read of unwritten memory then sees NaN), "graphed" runs tests/test_gpu_ppo_agent.py's fp32 graphed
step test body (two agents, five minibatch steps).
"""
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import torch  # noqa: E402

from agents import ppo as P  # noqa: E402


def run(graphs: bool):
    from training import train

    bad, seen = [], {"steps": 0}
    orig_clip = P.PPOAgent._clip_and_step
    orig_init = P.PPOAgent.__init__

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        self.use_graphs = graphs and self.device.type == "cuda"

    def clip(self):
        capturing = torch.cuda.is_current_stream_capturing()
        if not capturing:
            torch.cuda.synchronize()
            for name, p in self.network.named_parameters():
                if p.grad is None:
                    continue
                g = p.grad.detach().double()
                nf = int((~torch.isfinite(g)).sum())
                nrm = float(torch.linalg.vector_norm(torch.nan_to_num(g, nan=0.0, posinf=0.0, neginf=0.0)))
                mx = float(torch.nan_to_num(g, nan=0.0, posinf=0.0, neginf=0.0).abs().max())
                if nf or nrm > 1e6:
                    bad.append({"step": seen["steps"], "param": name, "nonfinite": nf, "norm": nrm, "max": mx,
                                "stride": list(p.grad.stride()), "grad_ptr_mod256": p.grad.data_ptr() % 256})
            seen["steps"] += 1
        return orig_clip(self)

    P.PPOAgent.__init__ = init
    P.PPOAgent._clip_and_step = clip
    err = None
    try:
        with tempfile.TemporaryDirectory() as tmp:
            cfg = {"ppo": {"num_epochs": 2},
                   "training": {"num_envs": 512, "batch_size": 1024, "rollout_steps": 16, "total_timesteps": 10 ** 9},
                   "rewards": {}, "logging": {"log_interval": 1, "save_interval": 100},
                   "paths": {"checkpoint_dir": tmp + "/ck", "log_dir": tmp + "/logs", "results_dir": tmp + "/res"}}
            train(cfg, seed=42, max_updates=2)
    except Exception as exc:  # noqa: BLE001
        err = f"{type(exc).__name__}: {exc}"[:400]
    finally:
        P.PPOAgent.__init__ = orig_init
        P.PPOAgent._clip_and_step = orig_clip
    return {"graphs": graphs, "eager_clip_calls": seen["steps"], "bad": bad[:40], "n_bad": len(bad), "error": err}


def poison(kind: str):
    if kind == "nan":
        blocks = [torch.full((n,), float("nan"), device="cuda") for n in [1 << s for s in range(6, 28)] for _ in range(4)]
        torch.cuda.synchronize()
        del blocks
    elif kind == "graphed":
        from agents import PPOAgent, PPOConfig

        def make(graphs):
            torch.manual_seed(3)
            a = PPOAgent(PPOConfig(batch_size=256), device=torch.device("cuda"), sample_seed=1)
            a.use_graphs = graphs
            a.train()
            return a

        g = torch.Generator(device="cuda").manual_seed(9)
        B = 256
        agents = (make(False), make(True))
        for _ in range(5):
            x = (torch.rand((B, 4, 8, 8), device="cuda", generator=g) < 0.4).float()
            m = (torch.rand((B, 192), device="cuda", generator=g) < 0.3).float()
            m[:, 0] = 1.0
            a = torch.multinomial(m, 1, generator=g).squeeze(1)
            b = (x, m, a, -torch.rand(B, device="cuda", generator=g) * 4, torch.randn(B, device="cuda", generator=g),
                 torch.randn(B, device="cuda", generator=g))
            for ag in agents:
                ag.train_minibatch(*b)
        torch.cuda.synchronize()
        del agents


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    poison(sys.argv[2] if len(sys.argv) > 2 else "none")
    for g in ((True, False) if mode == "both" else ((mode == "graphs"),)):
        print(json.dumps(run(g)), flush=True)


if __name__ == "__main__":
    main()
