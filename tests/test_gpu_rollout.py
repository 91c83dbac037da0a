"""bb_rollout (T fused steps in one launch) against T chained bb_step calls.

bb_step is itself bit-exact against the CPU oracle (test_gpu_env_parity.py),
so equality of every per-step output (reward, terminated, lines, applied
action, post-step mask), of the final state and of the next policy action
pins the fused kernel to the reference semantics; a small batch is also
checked against the oracle directly.
"""
import numpy as np
import pytest
import torch

from oracle import bb_game as O
from oracle import philox

pytestmark = pytest.mark.gpu

SEED = 0xB10C


def _env(n, offset, cuda, autoreset=True, unseeded=False):
    import ctypes as C

    from runtime.device_env import DeviceEnvBatch

    env = DeviceEnvBatch(n, seeds=[42 + offset + i for i in range(n)], device=cuda, env_offset=offset,
                         autoreset=autoreset)
    if unseeded:  # every other env seed_value None: fixed raw PCG words, stream continues across resets
        seeds = np.array([42 + offset + i for i in range(n)], dtype=np.uint64)
        has = (np.arange(n) % 2 == 0).astype(np.uint8)
        raw = np.random.default_rng(99).integers(0, 2 ** 63, size=(n, 4), dtype=np.int64).astype(np.uint64)
        assert env.lib.bb_seed(env.handle, seeds.ctypes.data_as(C.c_void_p), has.ctypes.data_as(C.c_void_p),
                               raw.ctypes.data_as(C.c_void_p)) == 0
    env.reset()
    mb = torch.zeros((n, 3), dtype=torch.int64, device=cuda)
    env.obs(mask_bits=mb)
    a0 = torch.zeros(n, dtype=torch.int32, device=cuda)
    env.random_actions(mb, a0, seed=SEED, step=0)
    return env, a0


def _chained_steps(n, offset, steps, cuda, step0=0, warm=0, autoreset=True, unseeded=False):
    env, a = _env(n, offset, cuda, autoreset, unseeded)
    nxt = torch.zeros_like(a)
    for t in range(warm):
        env.step(a, next_action=nxt, policy_seed=SEED, policy_step=t + 1)
        a, nxt = nxt, a
    rew, term, lines, acts, masks = [], [], [], [], []
    mb = torch.zeros((n, 3), dtype=torch.int64, device=cuda)
    for t in range(steps):
        acts.append(a.clone())
        env.step(a, next_action=nxt, want_lines=True, policy_seed=SEED, policy_step=step0 + t + 1, mask_out=mb)
        rew.append(env.reward.clone())
        term.append(env.terminated.clone())
        lines.append(env.lines.clone())
        masks.append(mb.clone())
        a, nxt = nxt, a
    torch.cuda.synchronize()
    out = {
        "reward": torch.stack(rew).cpu().numpy(), "terminated": torch.stack(term).cpu().numpy(),
        "lines": torch.stack(lines).cpu().numpy(), "actions": torch.stack(acts).cpu().numpy(),
        "mask": torch.stack(masks).cpu().numpy(), "next_action": a.cpu().numpy(),
    }
    st = env.state()
    env.close()
    return out, st


def _rollout(n, offset, steps, cuda, step0=0, warm=0, splits=(None,), autoreset=True, unseeded=False):
    env, a = _env(n, offset, cuda, autoreset, unseeded)
    nxt = torch.zeros_like(a)
    for t in range(warm):
        env.step(a, next_action=nxt, policy_seed=SEED, policy_step=t + 1)
        a, nxt = nxt, a
    rew = torch.zeros((steps, n), dtype=torch.float32, device=cuda)
    term = torch.zeros((steps, n), dtype=torch.uint8, device=cuda)
    lines = torch.zeros((steps, n), dtype=torch.uint8, device=cuda)
    acts = torch.zeros((steps, n), dtype=torch.int32, device=cuda)
    masks = torch.zeros((steps, n, 3), dtype=torch.int64, device=cuda)
    bounds = [0] + [s for s in splits if s is not None] + [steps]
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        env.rollout(hi - lo, a, rew[lo:hi], term[lo:hi], lines=lines[lo:hi], actions_out=acts[lo:hi],
                    mask_out=masks[lo:hi], next_action=nxt, policy_seed=SEED, policy_step0=step0 + lo)
        a, nxt = nxt, a
    torch.cuda.synchronize()
    out = {
        "reward": rew.cpu().numpy(), "terminated": term.cpu().numpy(), "lines": lines.cpu().numpy(),
        "actions": acts.cpu().numpy(), "mask": masks.cpu().numpy(), "next_action": a.cpu().numpy(),
    }
    st = env.state()
    env.close()
    return out, st


def _assert_same(ref, got):
    (ro, rs), (go, gs) = ref, got
    for k in ro:
        if k == "reward":
            assert np.array_equal(ro[k].view(np.uint32), go[k].view(np.uint32)), k
        else:
            assert np.array_equal(ro[k], go[k]), k
    for k in rs:
        if k == "rng":  # numpy's `uinteger` is meaningful only while has_uint32 (hand bit 22) is set
            assert np.array_equal(rs[k][:, :2], gs[k][:, :2]), "state rng"
            has = ((rs["hand"] >> 22) & 1).astype(bool)
            assert np.array_equal(rs[k][has, 2], gs[k][has, 2]), "state rng uinteger"
        else:
            assert np.array_equal(rs[k], gs[k]), f"state {k}"


@pytest.mark.parametrize("n,steps", [(1, 40), (65, 30), (257, 40), (1000, 60), (4096, 90)])
def test_rollout_equals_chained_steps(cuda, n, steps):
    """Ragged and tiny batches too: one env (a workgroup with 255 dead lanes), 65 (a second env wave of one
    env), 257 (a second workgroup of one env)."""
    _assert_same(_chained_steps(n, 0, steps, cuda), _rollout(n, 0, steps, cuda))


def test_rollout_single_step_segments(cuda):
    """Calls of T = 1 (bb_rollout then runs step_fused_kernel) between async calls continue one trajectory."""
    _assert_same(_chained_steps(777, 5, 40, cuda), _rollout(777, 5, 40, cuda, splits=(1, 2, 9, 10)))


def test_rollout_zero_steps_is_a_no_op(cuda):
    env, a = _env(300, 0, cuda)
    before = env.state()
    rew = torch.full((1, 300), 7.0, device=cuda)
    term = torch.full((1, 300), 9, dtype=torch.uint8, device=cuda)
    nxt = torch.full((300,), -5, dtype=torch.int32, device=cuda)
    env.rollout(0, a, rew, term, next_action=nxt, policy_seed=SEED)
    torch.cuda.synchronize()
    after = env.state()
    for k in before:
        assert np.array_equal(before[k], after[k]), k
    assert bool((rew == 7.0).all()) and bool((term == 9).all()) and bool((nxt == -5).all())
    env.close()


def test_rollout_split_calls_and_offset(cuda):
    """Two rollout calls chained through next_action == one call == steps,
    for a shard with a non-zero global offset, after a warm-up."""
    n, steps, off = 777, 48, 5000
    ref = _chained_steps(n, off, steps, cuda, step0=10, warm=10)
    _assert_same(ref, _rollout(n, off, steps, cuda, step0=10, warm=10))
    _assert_same(ref, _rollout(n, off, steps, cuda, step0=10, warm=10, splits=(17,)))


def test_rollout_without_autoreset(cuda):
    """Single-env semantics: after game over every action is invalid (-10,
    no state change) and the game-over bit stays set."""
    n, steps = 256, 120
    ref = _chained_steps(n, 0, steps, cuda, autoreset=False)
    assert (ref[0]["reward"] == -10.0).any()
    _assert_same(ref, _rollout(n, 0, steps, cuda, autoreset=False))


def test_rollout_unseeded_envs(cuda):
    """seed_value None (half the envs): auto-reset continues the stream
    instead of re-seeding (engine.py:137-138)."""
    n, steps = 512, 150
    ref = _chained_steps(n, 0, steps, cuda, unseeded=True)
    assert ref[0]["terminated"][:, 1::2].any()
    _assert_same(ref, _rollout(n, 0, steps, cuda, unseeded=True))


def test_rollout_full_size(cuda):
    """BASELINE config 2 size: 65,536 envs."""
    n, steps = 65536, 40
    _assert_same(_chained_steps(n, 0, steps, cuda), _rollout(n, 0, steps, cuda))


def test_rollout_matches_oracle(cuda):
    n, steps, off = 40, 60, 777
    out, st = _rollout(n, off, steps, cuda)
    cpu = O.VecEnv(n, seed=42 + off)
    oc, _ = cpu.reset()
    acts = philox.random_policy(oc["action_mask"].astype(bool), SEED, 0, env_offset=off)
    for t in range(steps):
        assert np.array_equal(out["actions"][t], acts), t
        oc, rc, tc, _, _ = cpu.step(acts)
        assert np.array_equal(out["reward"][t].view(np.uint32), rc.view(np.uint32)), t
        assert np.array_equal(out["terminated"][t].astype(bool), tc), t
        acts = philox.random_policy(oc["action_mask"].astype(bool), SEED, t + 1, env_offset=off)
    assert np.array_equal(out["next_action"], acts)
    ps = cpu.packed_state()
    assert np.array_equal(st["board"], ps["board"])
    for key in ("score", "moves", "lines", "combo", "max_combo", "blocks"):
        assert np.array_equal(st[key].astype(np.int64), ps[key].astype(np.int64)), key


def test_rollout_long_horizon(cuda):
    """A long launch: the envs of a wave drift many steps apart while their hand searches are answered by
    the search waves (rollout_async_kernel), and every output still lands at its own [step][env]."""
    n, steps = 2048, 400
    _assert_same(_chained_steps(n, 0, steps, cuda), _rollout(n, 0, steps, cuda))
