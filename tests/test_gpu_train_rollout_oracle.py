"""The training rollout at BASELINE's sizes, replayed through the C oracle.

``DeviceRollout.collect`` (training/trainer.py, scripts/train.py:173-203 on
the device: packed snapshot, CNN forward, fused masked sample, bb_step with
in-kernel auto-reset, buffer writes, observation expansion) records what every
env saw and did.  The C oracle's envs (same seeds 42 + i) are stepped through
the recorded actions, and every step's pre-step board / hand / 192-bit mask,
f32 reward bits, done flag and -- for the episodes that ended -- final score
and moves (info['final_score'] / info['moves'], scripts/train.py:196-201) must
be identical.

* config 3: 65,536 envs, default.yaml (T = 128), fp32 CNN, eager rollout;
  then one PPO update at the full buffer (8,388,608 samples, minibatch 2048)
  whose metrics must be finite.  The update runs one epoch here (4,096
  optimizer steps, ~30 s); the ten-epoch iteration is timed by
  tools/bench_ppo.py (profiles/).
* config 5 (one GPU's shard): 131,072 envs, long_train.yaml's horizon
  (T = 128), bf16 autocast, the rollout step captured in a HIP graph -- the
  eager warm-up collect, the capture + first replay, and a second replay, each
  checked against the oracle continuing from the previous one; then one bf16
  update epoch over that buffer (16,777,216 samples: 8,192 graph-replayed
  optimizer steps of the per-GPU minibatch 2,048, ppo.py:330-423) whose metrics
  must be finite with a positive entropy; its time is printed.
"""
import time

import numpy as np
import pytest
import torch

from oracle import c_oracle as CO

pytestmark = pytest.mark.gpu


def _check_collect(roll, cpu, label):
    buf = roll.buffer
    torch.cuda.synchronize()
    acts = buf.actions.cpu().numpy().astype(np.int32)
    ref = cpu.replay(acts)
    T, n = acts.shape
    assert np.array_equal(buf.board.cpu().numpy().view(np.uint64), ref["board"]), f"{label}: board snapshots"
    assert np.array_equal(buf.hand.cpu().numpy().view(np.uint32), ref["hand"]), f"{label}: hand snapshots"
    assert np.array_equal(buf.mask_bits.cpu().numpy().view(np.uint64), ref["mask"]), f"{label}: mask snapshots"
    # the sampled actions are legal: the mask bit of every recorded action is set
    bit = (ref["mask"].reshape(T, n, 3)[np.arange(T)[:, None], np.arange(n)[None, :], acts >> 6]
           >> (acts & 63).astype(np.uint64)) & np.uint64(1)
    assert bit.all(), f"{label}: an illegal action was sampled"
    assert np.array_equal(buf.rewards.cpu().numpy().view(np.uint32), ref["reward"].view(np.uint32)), \
        f"{label}: reward bits"
    dones = buf.dones.cpu().numpy()
    assert np.array_equal(dones, ref["terminated"].astype(np.float32)), f"{label}: dones"
    d = dones > 0
    assert d.sum() > 1000, f"{label}: too few episodes ended to check auto-reset ({d.sum()})"
    assert np.array_equal(roll.ep_score.cpu().numpy()[d], ref["ep_score"][d]), f"{label}: final scores"
    assert np.array_equal(roll.ep_moves.cpu().numpy()[d], ref["ep_moves"][d]), f"{label}: episode lengths"
    return int(d.sum())


def _setup(n, cuda, autocast=None):
    from agents import PPOAgent, PPOConfig
    from training.trainer import DeviceRollout

    torch.manual_seed(42)
    agent = PPOAgent(PPOConfig(batch_size=2048, num_epochs=10), device=cuda, sample_seed=7)
    agent.autocast_dtype = autocast
    agent.train()  # scripts/train.py:122: rollouts in train mode
    roll = DeviceRollout(n, 0, n, 42, {}, 128, cuda)
    roll.reset()
    cpu = CO.CVecEnv(np.arange(42, 42 + n, dtype=np.uint64))
    cpu.reset()
    return agent, roll, cpu


def test_config3_training_rollout_matches_c_oracle(cuda):
    agent, roll, cpu = _setup(65536, cuda)
    roll.collect(agent)
    ended = _check_collect(roll, cpu, "config 3")
    print(f"config 3 rollout: 65,536 envs x 128 steps bit-exact, {ended} episodes ended")
    agent.config.num_epochs = 1
    m = agent.update(roll.buffer, agent.values_device(roll.x))
    assert all(np.isfinite(v) for v in m.values()), m
    assert m["entropy"] > 0
    roll.close()
    cpu.close()


def test_config5_graph_rollout_matches_c_oracle(cuda):
    agent, roll, cpu = _setup(131072, cuda, autocast=torch.bfloat16)
    for k, label in enumerate(("eager warm-up", "capture + replay 1", "replay 2")):
        roll.collect(agent, graph=True)
        assert (roll._graph is not None) == (k > 0)
        _check_collect(roll, cpu, f"config 5 {label}")
    agent.config.num_epochs = 1
    last = agent.values_device(roll.x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = agent.update(roll.buffer, last)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert all(np.isfinite(v) for v in m.values()), m
    assert m["entropy"] > 0
    print(f"config 5 shard: one bf16 update epoch over 131,072 x 128 samples (8,192 optimizer steps) in {dt:.2f} s "
          f"({dt / 8192 * 1e3:.3f} ms per step), metrics {m}")
    roll.close()
    cpu.close()
