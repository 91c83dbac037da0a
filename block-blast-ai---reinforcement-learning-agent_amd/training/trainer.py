"""Device-resident PPO training driver: drop-in for the reference
``scripts/train.py`` (load_config 39-42, create_directories 45-58, train
61-312) behind the same CLI (``run_train.py --config --resume --seed``).

What stays identical: config sections and their reading quirks (``num_epochs``
comes from ``ppo``, ``batch_size`` / ``num_envs`` / ``rollout_steps`` /
``total_timesteps`` from ``training``, the ``network`` section is ignored),
env i seeded ``seed + i``, the agent kept in train mode for rollouts
(BatchNorm batch statistics), ``global_step += num_envs`` per rollout step,
FPS = global_step / wall time, the 100-episode score window, the
``best.pt`` / ``latest.pt`` / ``checkpoint_{step}.pt`` / ``final.pt`` names,
JSONL + summary logs, and the progress callback contract.

What changes: nothing crosses PCIe inside the rollout.  Per step the env
shard snapshots its packed state (board bits, hand word, mask bits) into the
``PackedRolloutBuffer``, expands the CNN input in HBM, the fused masked-sample
kernel picks actions, and ``bb_step`` advances every env with in-kernel
auto-reset.  Episode statistics are gathered on the device and read once per
update.

Data parallel (one process per GPU, ``torch.distributed.run``): the
``num_envs`` envs are split into contiguous shards by global index (seeds
``seed + global_index`` as on one GPU); each rank trains on its shard's
samples with minibatch ``batch_size // world`` (``training.minibatch_scope:
global``, the default: the global minibatch is the reference's) or
``batch_size`` (``per_gpu``, SURVEY 8(d) C4: the optimizer steps per update
are one GPU's); gradients are averaged by an RCCL all-reduce of the flat
gradient buffer per optimizer step, in two buckets: the heads + FC gradients'
all-reduce is issued when their backward segment ends and runs while the
conv stack's backward replays (``training.dp_overlap: graph-segments``, the
default), and advantage moments are global.  BatchNorm statistics stay per rank
(documented deviation).
"""
from __future__ import annotations

import os
import sys
import time
from datetime import datetime
from pathlib import Path
from typing import Any, Callable, Dict, Optional

import numpy as np
import torch
import torch.distributed as dist
import yaml

from agents.ppo import DP_OVERLAP_MODES, PackedRolloutBuffer, PPOAgent, PPOConfig, broadcast_parameters
from runtime.device_env import DeviceEnvBatch
from utils.device import get_device, set_seed
from utils.logger import Logger, MetricsTracker, TensorBoardLogger

WINDOW = 100  # MetricsTracker(window_size=100), train.py:96

DEFAULT_CONFIG: Dict[str, Any] = {  # train.py:263-296 fallback when the YAML is missing
    "environment": {"board_size": 8},
    "ppo": {"learning_rate": 3e-4, "gamma": 0.99, "gae_lambda": 0.95, "clip_epsilon": 0.2,
            "entropy_coef": 0.01, "value_coef": 0.5, "max_grad_norm": 0.5},
    "training": {"num_envs": 64, "batch_size": 2048, "num_epochs": 10, "rollout_steps": 128,
                 "total_timesteps": 10_000_000},
    "rewards": {"line_clear_base": 100, "block_placed": 1, "game_over_penalty": -500},
    "logging": {"log_interval": 10, "save_interval": 100, "eval_interval": 50},
    "paths": {"checkpoint_dir": "checkpoints", "log_dir": "logs", "results_dir": "results"},
}


def load_config(config_path: str) -> Dict[str, Any]:
    """train.py:39-42 (yaml.safe_load)."""
    with open(config_path, "r") as f:
        return yaml.safe_load(f)


def create_directories(config: Dict[str, Any], make: bool = True) -> Dict[str, Path]:
    """train.py:45-58."""
    paths = config.get("paths", {})
    dirs = {"checkpoint": Path(paths.get("checkpoint_dir", "checkpoints")),
            "log": Path(paths.get("log_dir", "logs")),
            "results": Path(paths.get("results_dir", "results"))}
    if make:
        for d in dirs.values():
            d.mkdir(parents=True, exist_ok=True)
    return dirs


def ppo_config_from(config: Dict[str, Any]) -> PPOConfig:
    """train.py:110-119, including where each field is read from."""
    p, t = config.get("ppo", {}), config.get("training", {})
    return PPOConfig(
        learning_rate=p.get("learning_rate", 3e-4), gamma=p.get("gamma", 0.99),
        gae_lambda=p.get("gae_lambda", 0.95), clip_epsilon=p.get("clip_epsilon", 0.2),
        entropy_coef=p.get("entropy_coef", 0.01), value_coef=p.get("value_coef", 0.5),
        max_grad_norm=p.get("max_grad_norm", 0.5), num_epochs=p.get("num_epochs", 10),
        batch_size=t.get("batch_size", 2048))


def _dist_setup():
    """(rank, world) — initialises the process group when launched by
    torch.distributed.run (RCCL on the GPU; gloo when asked via BB_DIST_BACKEND)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1 and not dist.is_initialized():
        backend = os.environ.get("BB_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        dist.init_process_group(backend)
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class DeviceRollout:
    """One rank's env shard + packed rollout storage + episode bookkeeping."""

    def __init__(self, num_envs: int, env_offset: int, global_envs: int, seed: int, reward_config,
                 rollout_steps: int, device: torch.device):
        self.n, self.offset, self.global_envs, self.T = num_envs, env_offset, global_envs, rollout_steps
        self.device = device
        self.env = DeviceEnvBatch(num_envs, [seed + env_offset + i for i in range(num_envs)], reward_config,
                                  autoreset=True, device=device, env_offset=env_offset)
        self.buffer = PackedRolloutBuffer(rollout_steps, num_envs, device)
        self.x = torch.zeros((num_envs, 4, 8, 8), dtype=torch.float32, device=device)
        self.mask_bits = torch.zeros((num_envs, 3), dtype=torch.int64, device=device)
        self.actions32 = torch.zeros(num_envs, dtype=torch.int32, device=device)
        # final score / moves of episodes ending at (t, i); valid where dones[t, i] == 1 (stale elsewhere)
        self.ep_score = torch.zeros((rollout_steps, num_envs), dtype=torch.int64, device=device)
        self.ep_moves = torch.zeros((rollout_steps, num_envs), dtype=torch.int32, device=device)
        self._graph = None          # captured rollout (collect(graph=True))
        self._graph_warm = False
        self._graph_key = None      # (agent, agent.graph_epoch, train mode) the graph was captured for
        self._step_base = None

    def reset(self) -> None:
        self.env.reset()
        self.env.obs(x=self.x, mask_bits=self.mask_bits)

    def collect(self, agent: PPOAgent, graph: bool = False) -> None:
        """scripts/train.py:173-203 for this shard, entirely on the device.

        ``graph=True`` (BASELINE config 5): the T rollout steps -- snapshot,
        CNN forward, fused masked sample, bb_step, buffer writes, observation
        expansion -- are captured once into one HIP graph and replayed on later
        calls (the first call runs eagerly and warms MIOpen / hipBLASLt up).
        The sampling step comes from a device counter (bb_masked_sample_dstep)
        so replays draw fresh uniforms; outputs equal the eager loop's for the
        same counter value."""
        if not graph or not self.env.device.type == "cuda":
            self._collect_steps(agent)
            return
        key = (id(agent), agent.graph_epoch, agent.network.training)
        if self._graph_key != key:  # new agent, parameter storage, layout, precision or mode: recapture
            self._graph, self._graph_warm, self._graph_key = None, False, key
        if self._graph is None and not self._graph_warm:
            self._collect_steps(agent)  # eager warm-up: library algorithm selection, workspaces
            self._graph_warm = True
            return
        if self._graph is None:
            self._step_base = torch.zeros(1, dtype=torch.int64, device=self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._collect_steps(agent, step_base=self._step_base)
            self._graph = g
        self._step_base.fill_(agent.sample_step)
        self._graph.replay()
        agent.sample_step += self.T
        self.buffer.ptr, self.buffer.full = self.T, True

    def _collect_steps(self, agent: PPOAgent, step_base: Optional[torch.Tensor] = None) -> None:
        buf, env = self.buffer, self.env
        buf.reset()
        for t in range(self.T):
            env.snapshot(board=buf.board[t], hand=buf.hand[t], mask_bits=buf.mask_bits[t])
            a, lp, v = agent.act_device(self.x, buf.mask_bits[t], env_offset=self.offset, step_base=step_base,
                                        step_add=t)
            buf.actions[t].copy_(a)
            buf.log_probs[t].copy_(lp)
            buf.values[t].copy_(v)
            self.actions32.copy_(a)
            # final score / moves written by bb_step straight into row t for the envs that ended (the
            # reference reads info['final_score'] / info['moves'] of terminated envs only, train.py:196-201)
            env.step(self.actions32, final_score=self.ep_score[t], final_moves=self.ep_moves[t])
            buf.rewards[t].copy_(env.reward)
            buf.dones[t].copy_(env.terminated)
            env.obs(x=self.x)
            buf.advance()

    def episodes(self, world: int):
        """Episodes finished in this rollout, ordered like the reference's
        append order (step-major, then global env index), reduced over ranks:
        (count, max score, last <=WINDOW (score, moves) pairs)."""
        d = self.buffer.dones.reshape(-1) > 0
        idx = torch.nonzero(d).squeeze(-1)
        count = torch.tensor([idx.numel()], dtype=torch.int64, device=self.device)
        tail = idx[-WINDOW:]
        t = torch.div(tail, self.n, rounding_mode="floor")
        key = t * self.global_envs + self.offset + (tail - t * self.n)
        rec = torch.full((WINDOW, 3), -1, dtype=torch.int64, device=self.device)
        k = tail.numel()
        if k:
            rec[WINDOW - k:, 0] = key
            rec[WINDOW - k:, 1] = self.ep_score.reshape(-1)[tail]
            rec[WINDOW - k:, 2] = self.ep_moves.reshape(-1)[tail].long()
        smax = torch.where(d, self.ep_score.reshape(-1), torch.full_like(self.ep_score.reshape(-1), -1)).max()
        smax = smax.reshape(1)
        if world > 1:
            dist.all_reduce(count)
            dist.all_reduce(smax, op=dist.ReduceOp.MAX)
            parts = [torch.empty_like(rec) for _ in range(world)]
            dist.all_gather(parts, rec)
            rec = torch.cat(parts)
        rec = rec.cpu().numpy()
        rec = rec[rec[:, 0] >= 0]
        rec = rec[np.argsort(rec[:, 0], kind="stable")][-WINDOW:]
        return int(count.item()), int(smax.item()), rec[:, 1].tolist(), rec[:, 2].tolist()

    def close(self) -> None:
        self.env.close()


def train(config: Dict[str, Any], resume_path: Optional[str] = None, seed: int = 42,
          progress_callback: Optional[Callable[[Dict[str, Any]], bool]] = None,
          max_updates: Optional[int] = None) -> Dict[str, Any]:
    """train.py:61-254.  Returns the final statistics (the reference prints them)."""
    rank, world = _dist_setup()
    main = rank == 0
    set_seed(seed)
    device = get_device(verbose=main)
    dirs = create_directories(config, make=main)

    ppo_cfg, train_cfg = config.get("ppo", {}), config.get("training", {})
    # set_seed turns on cudnn.deterministic like the reference (device.py:74-90).  Under MIOpen
    # that excludes the split-K weight-gradient convolutions and made a 65,536-env PPO update
    # several times slower, so the trainer turns it back off unless training.deterministic is set;
    # env streams, rollouts and sampling stay deterministic either way, only the CNN gradients'
    # last bits vary run to run.
    if torch.cuda.is_available():
        torch.backends.cudnn.deterministic = bool(train_cfg.get("deterministic", False))
    reward_cfg, log_cfg = config.get("rewards", {}), config.get("logging", {})
    name = f"ppo_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
    logger = Logger(str(dirs["log"]), name, enabled=main)
    tb = TensorBoardLogger(str(dirs["log"]), name, enabled=main)
    tracker = MetricsTracker(window_size=WINDOW)

    num_envs = int(train_cfg.get("num_envs", 64))
    if num_envs % world:
        raise ValueError(f"num_envs={num_envs} must divide evenly over {world} ranks")
    local = num_envs // world
    rollout_steps = int(train_cfg.get("rollout_steps", 128))
    roll = DeviceRollout(local, rank * local, num_envs, seed, reward_cfg, rollout_steps, device)
    if main:
        print(f"Created {num_envs} parallel environments" + (f" ({world} shards of {local})" if world > 1 else ""))

    agent_cfg = ppo_config_from(config)
    agent = PPOAgent(agent_cfg, device)
    if train_cfg.get("autocast") in ("bf16", "bfloat16"):
        agent.autocast_dtype = torch.bfloat16
    agent.train()
    broadcast_parameters(agent)
    if main:
        print(f"Created PPO agent with {sum(p.numel() for p in agent.network.parameters()):,} parameters")
    # minibatch per rank: "global" keeps the reference's global minibatch (batch_size // world per rank, so
    # the number of optimizer steps per update grows with the world size); "per_gpu" gives every rank a whole
    # batch_size minibatch of its own shard (per-GPU rollout + per-GPU minibatch 2048; the
    # effective minibatch is world x batch_size, the optimizer steps per update stay those of one GPU)
    scope = str(train_cfg.get("minibatch_scope", "global"))
    if scope not in ("global", "per_gpu"):
        raise ValueError(f"training.minibatch_scope must be 'global' or 'per_gpu', got {scope!r}")
    local_batch = agent_cfg.batch_size if scope == "per_gpu" else max(1, agent_cfg.batch_size // world)
    # data-parallel gradient all-reduce (agents.ppo.DP_OVERLAP_MODES): "graph-segments" (default:
    # the heads + FC bucket's all-reduce overlaps the conv-stack backward), "graph-split" (one exposed
    # all-reduce between two graphs) or "capture" (the collectives inside the step's graph; nccl = RCCL only)
    overlap = str(train_cfg.get("dp_overlap", "graph-segments"))
    if overlap not in DP_OVERLAP_MODES:
        raise ValueError(f"training.dp_overlap must be one of {DP_OVERLAP_MODES}, got {overlap!r}")
    if overlap == "capture" and world > 1 and dist.get_backend() != "nccl":
        raise ValueError("training.dp_overlap 'capture' puts the collectives inside a HIP graph: it needs the nccl "
                         f"(RCCL) backend, this run uses {dist.get_backend()!r}")
    agent.dp_overlap = overlap
    # BASELINE config 5: the rollout step captured in a HIP graph (training.graph_rollout)
    graph_rollout = bool(train_cfg.get("graph_rollout", False)) and device.type == "cuda"

    start_step = 0
    if resume_path and os.path.exists(resume_path):
        if main:
            print(f"Resuming from {resume_path}")
        agent.load(resume_path)
        try:
            start_step = int(Path(resume_path).stem.split("_")[-1])
        except ValueError:
            pass

    total_timesteps = int(train_cfg.get("total_timesteps", 50_000_000))
    log_interval = int(log_cfg.get("log_interval", 100))
    save_interval = int(log_cfg.get("save_interval", 1000))

    roll.reset()
    global_step, num_updates, best_score, n_episodes, max_episode = start_step, 0, 0, 0, None
    if main:
        print(f"\nStarting training for {total_timesteps:,} timesteps...")
        print(f"  Rollout steps: {rollout_steps}")
        print(f"  Batch size: {agent_cfg.batch_size}" + (f" ({scope}: {local_batch} per rank)" if world > 1 else ""))
        print(f"  Learning rate: {agent_cfg.learning_rate}")
        print("-" * 60, flush=True)
    start = time.time()

    def save(path: Path) -> None:
        if main:
            agent.save(str(path))

    try:
        while global_step < total_timesteps:
            roll.collect(agent, graph=graph_rollout)
            global_step += num_envs * rollout_steps
            cnt, smax, scores, moves = roll.episodes(world)
            if cnt:
                n_episodes += cnt
                max_episode = smax if max_episode is None else max(max_episode, smax)
                tracker.extend("episode_score", scores)
                tracker.extend("episode_length", moves)
            last_values = agent.values_device(roll.x)
            update_metrics = agent.update(roll.buffer, last_values, batch_size=local_batch)
            num_updates += 1
            elapsed = time.time() - start
            fps = global_step / elapsed if elapsed > 0 else 0.0  # train.py:214 (includes a resumed start_step)
            if main and num_updates <= 20:
                print(f"Update {num_updates}: step={global_step:,}, FPS={fps:.0f}, "
                      f"policy_loss={update_metrics['policy_loss']:.4f}", flush=True)
            if num_updates % log_interval == 0 or num_updates <= 10:
                avg_score = tracker.get_mean("episode_score")
                metrics = {"step": global_step, "fps": fps, "avg_score": avg_score,
                           "max_score": tracker.get_max("episode_score"), "best_score": best_score,
                           "avg_length": tracker.get_mean("episode_length"), **update_metrics}
                if avg_score > best_score:
                    best_score = avg_score
                    metrics["best_score"] = best_score
                    save(dirs["checkpoint"] / "best.pt")
                logger.log(metrics, global_step)
                logger.print_metrics(metrics)
                sys.stdout.flush()
                tb.log_metrics({"performance/avg_score": avg_score, "performance/max_score": metrics["max_score"],
                                "performance/best_score": best_score, "performance/avg_length": metrics["avg_length"],
                                "performance/fps": fps, **{f"training/{k}": update_metrics[k] for k in
                                                           ("policy_loss", "value_loss", "entropy", "approx_kl",
                                                            "clip_fraction")}}, global_step)
                if progress_callback is not None and main:
                    keep = progress_callback({"total_steps": global_step, "mean_score": avg_score,
                                              "best_score": best_score, "episodes": n_episodes, "fps": fps})
                    if not keep:
                        print("\nTraining stopped by callback")
                        break
            if num_updates % save_interval == 0:
                save(dirs["checkpoint"] / f"checkpoint_{global_step}.pt")
                save(dirs["checkpoint"] / "latest.pt")
                if main:
                    print(f"Saved checkpoint to {dirs['checkpoint'] / f'checkpoint_{global_step}.pt'}")
            if max_updates is not None and num_updates >= max_updates:
                break
    except KeyboardInterrupt:
        if main:
            print("\nTraining interrupted by user")
    finally:
        save(dirs["checkpoint"] / "final.pt")
        logger.save_summary()
        tb.close()
        roll.close()
    elapsed = time.time() - start
    summary = {"total_steps": global_step, "elapsed": elapsed,
               "fps": global_step / elapsed if elapsed > 0 else 0.0,
               "best_score": best_score, "episodes": n_episodes, "max_episode_score": max_episode,
               "updates": num_updates}
    if main:
        print("\n" + "=" * 60)
        print("Training Complete!")
        print(f"  Total steps: {global_step:,}")
        print(f"  Total time: {elapsed / 3600:.2f} hours")
        print(f"  Final FPS: {summary['fps']:.0f}")
        print(f"  Best average score: {best_score:.1f}")
        print(f"  Total episodes: {n_episodes}")
        if max_episode is not None:
            print(f"  Max episode score: {max_episode}")
        print("=" * 60)
    return summary
