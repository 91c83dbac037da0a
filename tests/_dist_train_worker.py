"""Worker for test_gpu_train.py's 2-rank run (launched by torch.distributed.run)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from training import trainer  # noqa: E402


def main():
    out = os.environ["BB_TEST_OUT"]
    os.environ["LOCAL_RANK"] = "0"  # both ranks share the one GPU of the test box
    captured = {}
    orig = trainer.PPOAgent

    class Spy(orig):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            captured["agent"] = self
            captured["steps"] = 0

            def count(_n, _st):
                captured["steps"] += 1
            self.minibatch_callback = count

    trainer.PPOAgent = Spy
    cfg = {"ppo": {"num_epochs": 1}, "training": {"num_envs": 512, "batch_size": 1024, "rollout_steps": 16,
                                                  "total_timesteps": 10 ** 9,
                                                  "minibatch_scope": os.environ.get("BB_TEST_SCOPE", "global")},
           "logging": {"log_interval": 1, "save_interval": 1000},
           "paths": {"checkpoint_dir": os.path.join(out, "ck"), "log_dir": os.path.join(out, "logs"),
                     "results_dir": os.path.join(out, "res")}}
    s = trainer.train(cfg, seed=42, max_updates=1)
    agent = captured["agent"]
    with torch.no_grad():
        checksum = float(sum(p.double().sum() for p in agent.network.parameters()))
    rank = dist.get_rank()
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump({"checksum": checksum, "total_steps": s["total_steps"], "episodes": s["episodes"],
                   "optimizer_steps": captured["steps"]}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
