"""The shipped rollout kernel's rare paths against the oracle.

bb_rollout with T >= 2 runs rollout_async_kernel (the kernel the bench times): env waves post every hand
that their in-lane quick test leaves open to an LDS record, and search waves claim records by
compare-and-swap, search them together (gen_hands_multi) and hand each env back as soon as its round
decides it.  Random play almost never reaches the rare branches of _generate_new_pieces
(engine.py:155-172): a search that runs all 100 attempts and keeps the last hand, a Lemire-rejected
32-bit draw (pieces.py:350-355, p ~ 1.6e-9 per draw) that shifts the jump-ahead batches back onto the
sequential stream, boards where only SINGLE fits.  These tests start every env on such a board
(tests/_crowded.py, the fixtures test_gpu_solver_stress.py runs through bb_step) and replay the launch's
recorded actions through the oracle: every step's reward bits, termination, lines and post-step mask,
the Philox policy's actions, and the final board, hand, PCG64 state and has_uint32 must be identical.

The iteration caps that keep the kernel from hanging on a lost record must fail loudly: with a
debug-only tiny cap (BB_DEBUG_ASYNC_CAP) the launch raises the handle's status word and the next call
returns BB_ERR_DEVICE until a full reset.
"""
import numpy as np
import pytest
import torch

from _crowded import crowded_setup, mask_bits
from oracle import philox

pytestmark = pytest.mark.gpu

SEED = 0xB10C


def _async_crowded(cuda, fill, pack, monkeypatch, reject_at=None, steps=6, n=512):
    from runtime.device_env import DeviceEnvBatch

    first, nxt = pack.split(",")
    monkeypatch.setenv("BB_PACK_FIRST", first)
    monkeypatch.setenv("BB_PACK_NEXT", nxt)
    dev = DeviceEnvBatch(n, seeds=[5000 + i for i in range(n)], device=cuda)
    state, acts, refs = crowded_setup(fill, n, reject_at)
    dev.set_state(**state)

    rew = torch.zeros((steps, n), dtype=torch.float32, device=cuda)
    term = torch.zeros((steps, n), dtype=torch.uint8, device=cuda)
    lines = torch.zeros((steps, n), dtype=torch.uint8, device=cuda)
    acts_out = torch.zeros((steps, n), dtype=torch.int32, device=cuda)
    masks = torch.zeros((steps, n, 3), dtype=torch.int64, device=cuda)
    nxt_a = torch.zeros(n, dtype=torch.int32, device=cuda)
    dev.rollout(steps, torch.from_numpy(acts).to(cuda), rew, term, lines=lines, actions_out=acts_out,
                mask_out=masks, next_action=nxt_a, policy_seed=SEED, policy_step0=0)
    dev.sync()  # raises if the kernel reported a device-side failure
    rew, term, lines = rew.cpu().numpy(), term.cpu().numpy(), lines.cpu().numpy()
    acts_out, masks = acts_out.cpu().numpy(), masks.cpu().numpy().view(np.uint64)
    st = dev.state()

    attempts = np.zeros(n, np.int64)
    cur = acts.astype(np.int64)
    for t in range(steps):
        assert np.array_equal(acts_out[t], cur), t
        post = np.zeros((n, 192), bool)
        for i, env in enumerate(refs):
            _, r_ref, t_ref, _, inf = env.step(int(cur[i]))
            if t == 0:
                attempts[i] = env.engine.attempts_last
            assert rew[t, i].view(np.uint32) == np.float32(r_ref).view(np.uint32), (t, i)
            assert bool(term[t, i]) == t_ref, (t, i)
            assert int(lines[t, i]) == inf.get("last_move", {}).get("lines_cleared", 0), (t, i)
            if t_ref:  # wrappers.py:97-102: the vec env resets (re-seeded with seed_value)
                env.reset()
            m = env.engine.action_mask()
            assert np.array_equal(masks[t, i], mask_bits(m)), (t, i)
            post[i] = m.reshape(-1)
        cur = philox.random_policy(post, SEED, t + 1).astype(np.int64)
    assert np.array_equal(nxt_a.cpu().numpy(), cur)
    for i, env in enumerate(refs):
        g = env.engine
        h = int(st["hand"][i])
        assert [(h >> (6 * s)) & 63 for s in range(3)] == g.hand, i
        assert [bool((h >> (18 + s)) & 1) for s in range(3)] == [bool(u) for u in g.used], i
        s = g.rng.bit_generator.state
        assert (int(st["rng"][i, 0]) << 64 | int(st["rng"][i, 1])) == s["state"]["state"], i
        assert bool((h >> 22) & 1) == bool(s["has_uint32"]), i
        if s["has_uint32"]:
            assert int(st["rng"][i, 2]) == s["uinteger"], i
        assert int(st["score"][i]) == g.score and int(st["moves"][i]) == g.moves, i
    dev.close()
    return attempts


@pytest.mark.parametrize("fill", [0.45, 0.6, 0.7, 0.8, 0.9, 0.95, -1.0, -2.0])
@pytest.mark.parametrize("pack", ["8,32", "1,0", "3,7"])
def test_async_rollout_crowded_boards(cuda, fill, pack, monkeypatch):
    """Crowded, two-holes-per-line and singles-only boards through the search waves with early hand-back,
    under three attempt schedules of gen_hands_multi."""
    attempts = _async_crowded(cuda, fill, pack, monkeypatch)
    assert attempts.max() > 1  # the boards really exercised rejection sampling
    if fill == -2.0:  # ~6% of the searches run all 100 attempts and keep the last hand (engine.py:159-172)
        assert (attempts == 100).any()


@pytest.mark.parametrize("fill", [0.9, -2.0])
@pytest.mark.parametrize("pack", ["8,32", "1,0"])
def test_async_rollout_lemire_rejection(cuda, fill, pack, monkeypatch):
    """A rejected 32-bit draw at a chosen stream position (attempts 0 .. 39, low and high halves): the
    search waves' jump-ahead batches assume three values per attempt and must fall back to the exact
    sequential stream, while the other envs of the call are handed back early."""
    n = 512
    reject_at = 1 + (np.arange(n) * 37) % 60  # LCG outputs 1 .. 60 = attempts 0 .. 39
    attempts = _async_crowded(cuda, fill, pack, monkeypatch, reject_at=reject_at, n=n)
    reached = attempts > (2 * (reject_at - 1) + (np.arange(n) & 1)) // 3
    assert reached.sum() > (n // 2 if fill == -2.0 else 4)


def test_async_rollout_many_workgroups(cuda, monkeypatch):
    """2,048 singles-only envs (8 workgroups of 256 envs, every record posted at once) over 16 steps."""
    attempts = _async_crowded(cuda, -2.0, "8,32", monkeypatch, steps=16, n=2048)
    assert (attempts == 100).any()


def test_async_iteration_cap_fails_loudly(cuda, monkeypatch):
    """A wave that leaves through its iteration cap raises the status word: bb_sync and every later call
    fail with BB_ERR_DEVICE (-4) until a full reset; a handle without the debug cap is unaffected."""
    from runtime import lib as L
    from runtime.device_env import DeviceEnvBatch

    n, steps = 1024, 32
    monkeypatch.setenv("BB_DEBUG_ASYNC_CAP", "3")
    dev = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=cuda)
    monkeypatch.delenv("BB_DEBUG_ASYNC_CAP")
    ok = DeviceEnvBatch(n, seeds=[42 + i for i in range(n)], device=cuda)
    bufs = [torch.zeros((steps, n), dtype=torch.float32, device=cuda),
            torch.zeros((steps, n), dtype=torch.uint8, device=cuda)]
    a0 = torch.zeros(n, dtype=torch.int32, device=cuda)
    for d in (dev, ok):
        d.reset()
        mb = torch.zeros((n, 3), dtype=torch.int64, device=cuda)
        d.obs(mask_bits=mb)
        d.random_actions(mb, a0, seed=SEED, step=0)
    dev.rollout(steps, a0, *bufs, policy_seed=SEED)
    with pytest.raises(L.BBNativeError, match=r"bb_sync failed \(-4\).*iteration cap"):
        dev.sync()
    with pytest.raises(L.BBNativeError, match=r"bb_rollout failed \(-4\)"):
        dev.rollout(steps, a0, *bufs, policy_seed=SEED)
    with pytest.raises(L.BBNativeError, match=r"\(-4\)"):
        dev.state()
    with pytest.raises(L.BBNativeError, match=r"bb_obs failed \(-4\)"):
        dev.obs(mask_bits=mb)
    with pytest.raises(L.BBNativeError, match=r"bb_snapshot failed \(-4\)"):
        dev.snapshot(torch.zeros(n, dtype=torch.int64, device=cuda), None, None)
    dev.reset()  # a full reset clears the status word
    dev.sync()
    dev.state()
    # a capped launch still queued when the full reset is issued: the reset clears the word in stream
    # order, after that launch has raised it, so the fresh handle's next calls succeed
    dev.rollout(steps, a0, *bufs, policy_seed=SEED)
    dev.reset()
    dev.sync()
    dev.obs(mask_bits=mb)
    dev.state()
    ok.rollout(steps, a0, *bufs, policy_seed=SEED)
    ok.sync()
    dev.close()
    ok.close()
