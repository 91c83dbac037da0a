"""The policy/value network's fp32 forward on the GPU against the oracle's
restatement of the reference network (the rollout's
``_raw`` call, network.py:135-182).

``PPOAgent``'s network in its product configuration (channels_last conv
stack, HIP BatchNorm + ReLU in train mode, the fp32 board convolutions of
csrc/bb_conv32.hip where autograd records nothing and MIOpen's for the input
layer, hipBLASLt GEMMs, fp32) and ``oracle.bb_ppo.ReferenceNetwork`` (the reference's plain
modules on the CPU) share their weights; Dropout is 0 on both sides (its mask
stream cannot be shared).  Inputs: 2,048 states (config 1's minibatch size)
of C-oracle envs (seeds 42 + i) after 24 synthetic-policy steps, so boards,
hands and masks are varied.

Tolerance (written here, checked per element): |logit_gpu - logit_true| <=
1e-5 * max(1, |logit_true|), values alike, where the truth is the same
network in float64 on the CPU -- the fp32 CPU result is held to the same
bound, so the test says the GPU's fp32 is as close to the exact function as
the reference's own fp32 run.  Masked-out actions must be -inf on both sides
at the same positions.  Train mode is the rollout's mode
(scripts/train.py:177 keeps the agent in train(): batch statistics); eval mode
uses the running statistics the train-mode pass left, which are compared too.

Both modes meet the bound on every element.  In train mode the batch-statistics BatchNorms amplify
summation-order differences: with MIOpen's fp32 128-channel convolutions (K = 1,152 products in one
order) the logits ended 1.28e-5 from the truth (round 4, tools/diag_net_fp32.py, profiles/r04/net/);
the product now runs those convolutions on csrc/bb_conv32.hip (16-product fp32 MFMA chains summed in
fp64, rounded once: tests/test_gpu_conv32.py), in every forward autograd does not record (the rollout's
``_raw``).  The train-mode check also runs at a rollout-sized batch of 16,384 C-oracle states (config 3
steps 65,536 boards at once; the batch statistics sum over 8x more terms than at 2,048), against the
same network in float64 on the GPU (the CPU's fp32 is only computed at 2,048).
"""
import copy
import functools

import numpy as np
import pytest
import torch

from oracle import bb_ppo as OP
from oracle import c_oracle as CO

pytestmark = pytest.mark.gpu

B = 2048
B_ROLLOUT = 16384
TOL = 1e-5  # |d| <= TOL * max(1, |truth|)


@functools.lru_cache(maxsize=2)
def _states(n):
    seeds = np.arange(42, 42 + n, dtype=np.uint64)
    env = CO.CVecEnv(seeds)
    env.reset()
    mask = env.state()["mask"]
    for t in range(24):
        mask = env.step(env.random_actions(mask, 0xB10C, t))["mask"]
    st = env.state()
    env.close()
    return OP.expand_packed(st["board"], st["hand"], st["mask"])


@pytest.fixture(scope="module")
def states():
    return _states(B)


def _nets(cuda):
    from agents import PPOAgent, PPOConfig

    torch.manual_seed(0)
    ref = OP.ReferenceNetwork(dropout=0.0)
    agent = PPOAgent(PPOConfig(batch_size=B), device=cuda, sample_seed=1)
    agent.network.load_state_dict(ref.state_dict())
    for mod in agent.network.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return ref, agent


def _check(name, gpu, cpu, truth):
    """Per-element bound against the fp64 truth for the GPU's fp32 (and the CPU's, when given)."""
    scale = np.maximum(1.0, np.abs(truth))
    e_gpu = np.abs(gpu.astype(np.float64) - truth) / scale
    msg = f"{name}: max |d|/max(1,|x|) gpu {e_gpu.max():.2e}"
    if cpu is not None:
        e_cpu = np.abs(cpu.astype(np.float64) - truth) / scale
        msg += f", cpu fp32 {e_cpu.max():.2e}"
    print(msg + f", |x| max {np.abs(truth).max():.2f}")
    if cpu is not None:
        assert e_cpu.max() <= TOL, (name, "the CPU's own fp32 exceeds the bound", e_cpu.max())
    assert e_gpu.max() <= TOL, (name, e_gpu.max(), np.unravel_index(e_gpu.argmax(), e_gpu.shape))


@pytest.mark.parametrize("mode", ["train", "eval"])
def test_network_forward_matches_reference_fp32(cuda, states, mode):
    boards, pieces, masks = states
    ref, agent = _nets(cuda)
    net64 = copy.deepcopy(ref).double()
    tb, tp, tm = torch.from_numpy(boards), torch.from_numpy(pieces), torch.from_numpy(masks)
    if mode == "eval":
        # one train-mode pass on each side first: the running statistics it leaves are the eval-mode input
        agent.train()
        ref.train()
        net64.train()
        with torch.no_grad():
            agent._raw(agent._obs_to_device({"board": boards, "pieces": pieces}))
            ref(tb, tp)
            net64(tb.double(), tp.double())
        sd_gpu = {k: v.detach().double().cpu() for k, v in agent.network.state_dict().items()}
        for k, v in ref.state_dict().items():
            if k.endswith(("running_mean", "running_var")):
                d = float((sd_gpu[k] - v.double()).abs().max())
                assert d <= 1e-5 * max(1.0, float(v.abs().max())), (k, d)
            elif k.endswith("num_batches_tracked"):
                assert int(sd_gpu[k]) == int(v), k
        agent.eval()
        ref.eval()
        net64.eval()
    else:
        agent.train()
        ref.train()
        net64.train()
    with torch.no_grad():
        lg, vg = agent._raw(agent._obs_to_device({"board": boards, "pieces": pieces}))
        mk = tm.to(cuda)
        lg = lg + torch.where(mk.bool(), torch.zeros_like(lg), torch.full_like(lg, float("-inf")))
        lc, vc = ref(tb, tp, tm)
        l64, v64 = net64(tb.double(), tp.double(), tm.double())
    lg, vg = lg.cpu().numpy(), vg.cpu().numpy()
    lc, vc, l64, v64 = lc.numpy(), vc.numpy(), l64.numpy(), v64.numpy()
    assert lg.shape == (B, 192) and vg.shape == (B,)
    inf_gpu, inf_ref = np.isneginf(lg), np.isneginf(l64)
    np.testing.assert_array_equal(inf_gpu, inf_ref)
    np.testing.assert_array_equal(inf_gpu, masks == 0)
    fin = ~inf_ref
    _check(f"{mode} logits", lg[fin], lc[fin], l64[fin])
    _check(f"{mode} values", vg, vc, v64)


def test_network_forward_train_mode_rollout_batch(cuda):
    """Train mode (batch statistics) at a rollout-sized batch: 16,384 C-oracle states in one forward, every
    logit and value within 1e-5 * max(1, |x|) of the same network in float64 (on the GPU)."""
    boards, pieces, masks = _states(B_ROLLOUT)
    ref, agent = _nets(cuda)
    net64 = copy.deepcopy(ref).double().to(cuda).train()
    agent.train()
    tb, tp = torch.from_numpy(boards).to(cuda), torch.from_numpy(pieces).to(cuda)
    with torch.no_grad():
        lg, vg = agent._raw(agent._obs_to_device({"board": boards, "pieces": pieces}))
        l64, v64 = net64(tb.double(), tp.double())
    fin = torch.from_numpy(masks).to(cuda).bool()
    _check(f"train logits B={B_ROLLOUT}", lg[fin].cpu().numpy(), None, l64[fin].cpu().numpy())
    _check(f"train values B={B_ROLLOUT}", vg.cpu().numpy(), None, v64.cpu().numpy())
