#!/usr/bin/env python3
"""BASELINE config 3 (full PPO on one MI355X): rollout + update timing.

One PPO iteration at the reference hyper-parameters is T=128 rollout steps of
N envs, then num_epochs x (T*N / batch) optimizer steps.  At N=65,536 that is
40,960 optimizer steps, so the update is timed over ``--update-steps``
minibatches and extrapolated (stated in the output).  FLOP accounting follows
SURVEY.md §8(d): 113,049,856 FLOP per sample forward, x3 for forward+backward.

Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import torch  # noqa: E402

FWD_FLOP = 113_049_856


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--rollout", type=int, default=128)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--update-steps", type=int, default=100)
    ap.add_argument("--autocast", choices=["none", "bf16"], default="none")
    ap.add_argument("--miopen-find", action="store_true", help="torch.backends.cudnn.benchmark = True")
    ap.add_argument("--layout", choices=["default", "nchw", "channels_last"], default="default",
                    help="conv-stack activation layout (default: the agent's own choice)")
    ap.add_argument("--no-graph", action="store_true", help="issue the update step kernel by kernel")
    ap.add_argument("--copy-inputs", action="store_true",
                    help="gather minibatches into fresh tensors and copy them into the captured step (pre-r02 path)")
    ap.add_argument("--graph-rollout", action="store_true",
                    help="BASELINE config 5: the rollout's T steps captured in one HIP graph and replayed")
    args = ap.parse_args()

    from agents import PPOAgent, PPOConfig
    from training.trainer import DeviceRollout

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if args.miopen_find:
        torch.backends.cudnn.benchmark = True
    agent = PPOAgent(PPOConfig(batch_size=args.batch, num_epochs=args.epochs), device=dev, sample_seed=1)
    if args.autocast == "bf16":
        agent.autocast_dtype = torch.bfloat16
    if args.layout != "default":
        agent.set_channels_last(args.layout == "channels_last")
    agent.use_graphs = not args.no_graph
    agent.train()
    roll = DeviceRollout(args.envs, 0, args.envs, 42, {}, args.rollout, dev)
    roll.reset()
    # warm-up: a short rollout + a few optimizer steps (kernels, MIOpen tuning)
    roll_w = DeviceRollout(min(args.envs, 4096), 0, min(args.envs, 4096), 7, {}, 4, dev)
    roll_w.reset()
    roll_w.collect(agent)
    agent.update(roll_w.buffer, agent.values_device(roll_w.x), batch_size=args.batch)
    roll_w.close()
    agent.values_device(roll.x)
    torch.cuda.synchronize()

    if args.graph_rollout:  # eager warm-up, then capture (+ one replay), all untimed
        roll.collect(agent, graph=True)
        roll.collect(agent, graph=True)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    roll.collect(agent, graph=args.graph_rollout)
    last = agent.values_device(roll.x)
    torch.cuda.synchronize()
    t_roll = time.perf_counter() - t0

    buf = roll.buffer
    buf.compute_returns_and_advantages(last, 0.99, 0.95)
    # as PPOAgent.update: minibatches gathered straight into the captured step's inputs
    batches = buf.get_minibatches(args.batch, out=None if args.copy_inputs else agent.minibatch_inputs)
    done = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for x, m, a, lp, adv, ret in batches:
        agent.train_minibatch(x, m, a, lp, adv, ret)
        done += 1
        if done >= args.update_steps:
            break
    torch.cuda.synchronize()
    t_upd_step = (time.perf_counter() - t0) / done

    samples = args.envs * args.rollout
    n_steps = args.epochs * -(-samples // args.batch)
    t_update = t_upd_step * n_steps
    t_iter = t_roll + t_update
    roll_flops = samples * FWD_FLOP / t_roll
    upd_flops = 3 * FWD_FLOP * args.batch / t_upd_step
    print(json.dumps({
        "workload": "BASELINE config 3: full PPO iteration on 1 MI355X", "envs": args.envs, "rollout_steps": args.rollout,
        "miopen_find": args.miopen_find, "channels_last": agent.channels_last, "graph_rollout": args.graph_rollout,
        "batch": args.batch, "epochs": args.epochs, "compute_dtype": "bf16 autocast" if args.autocast == "bf16" else "fp32",
        "rollout_s": round(t_roll, 4), "rollout_env_steps_per_s": round(samples / t_roll, 1),
        "rollout_cnn_tflops": round(roll_flops / 1e12, 2),
        "update_step_ms": round(t_upd_step * 1e3, 3), "update_steps_timed": done, "update_steps_total": n_steps,
        "update_s_extrapolated": round(t_update, 2), "update_cnn_tflops": round(upd_flops / 1e12, 2),
        "iteration_s": round(t_iter, 2), "ppo_env_steps_per_s": round(samples / t_iter, 1),
    }))
    roll.close()


if __name__ == "__main__":
    main()
