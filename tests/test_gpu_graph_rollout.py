"""BASELINE config 5's hipGraph-captured rollout step (DeviceRollout.collect
with graph=True): the T-step rollout loop of scripts/train.py:173-203 --
snapshot, CNN forward, fused masked sample, bb_step, buffer writes,
observation expansion -- captured once and replayed, must fill the packed
buffer exactly like the eager loop with the same sampling counter, and draw
fresh uniforms on every replay (bb_masked_sample_dstep)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

FIELDS = ("board", "hand", "mask_bits", "actions", "log_probs", "values", "rewards", "dones")


def _pair(cuda, n, T, train_mode):
    from agents import PPOAgent, PPOConfig
    from training.trainer import DeviceRollout

    torch.manual_seed(3)
    agents = [PPOAgent(PPOConfig(), cuda, sample_seed=77) for _ in range(2)]
    agents[1].network.load_state_dict(agents[0].network.state_dict())
    for a in agents:
        if train_mode:
            a.train()
            for m in a.network.modules():  # dropout off: its torch RNG stream differs under capture
                if isinstance(m, torch.nn.Dropout):
                    m.p = 0.0
        else:
            a.eval()
    rolls = [DeviceRollout(n, 0, n, 42, {}, T, cuda) for _ in range(2)]
    for r in rolls:
        r.reset()
    return agents, rolls


def _same(ra, rb, what):
    for f in FIELDS:
        x, y = getattr(ra.buffer, f), getattr(rb.buffer, f)
        assert torch.equal(x, y), f"{what}: {f} differs"


@pytest.mark.parametrize("train_mode", [False, True])
def test_graph_rollout_equals_eager(cuda, train_mode):
    n, T = 2048, 16
    (a_eager, a_graph), (r_eager, r_graph) = _pair(cuda, n, T, train_mode)
    prev_actions = None
    for it in range(4):  # warm-up (eager), capture + replay, replay, replay
        r_eager.collect(a_eager)
        r_graph.collect(a_graph, graph=True)
        torch.cuda.synchronize(cuda)
        _same(r_eager, r_graph, f"rollout {it}")
        assert a_eager.sample_step == a_graph.sample_step == (it + 1) * T
        assert r_graph.buffer.ptr == T and r_graph.buffer.full
        if it >= 2:
            assert r_graph._graph is not None
        acts = r_graph.buffer.actions.clone()
        if prev_actions is not None:
            assert not torch.equal(acts, prev_actions)  # fresh states and uniforms each replay
        prev_actions = acts
    # the env state after the rollouts is the same too
    se, sg = r_eager.env.state(), r_graph.env.state()
    for k in se:
        assert (se[k] == sg[k]).all(), k
    for r in (r_eager, r_graph):
        r.close()
