"""GPU parity of the hand generator on crowded boards.

Random 45-80 % filled boards where the last unused slot holds SINGLE: placing
it triggers _generate_new_pieces (engine.py:155-172) on a crowded board, where
many 3-draw attempts fail (and some envs exhaust all 100 attempts and keep the
last hand).  The device result (hand, pcg state, score, reward, game over)
must equal the oracle's reference DFS exactly; this drives both the per-lane
solver and the wave-cooperative escalation kernel.
"""
import numpy as np
import pytest

from _crowded import crowded_setup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fill", [0.45, 0.6, 0.7, 0.8, 0.9, 0.95, -1.0, -2.0])
@pytest.mark.parametrize("pack", ["1,0", "32,32", "3,7"])
def test_crowded_board_hand_generation(cuda, fill, pack, monkeypatch):
    """pack = escalation schedule (attempts per env in the first round, in
    later rounds; 0 = double the previous round's, capped at 32): every
    schedule must give the same hands."""
    _crowded(cuda, fill, pack, monkeypatch)


@pytest.mark.parametrize("fill", [0.6, 0.8, 0.95, -1.0])
def test_crowded_board_debug_fallback(cuda, fill, monkeypatch):
    """BB_DEBUG_MODE=2 (the solver counters) switches escalate_kernel to the
    one-env-at-a-time wave search (gen_hand_wave, bbvec.h bb_debug_counters):
    that path must stay bit-exact too."""
    monkeypatch.setenv("BB_DEBUG_MODE", "2")
    _crowded(cuda, fill, "8,32", monkeypatch)


def _crowded(cuda, fill, pack, monkeypatch, reject_at=None):
    """reject_at: per env, the LCG output (1-based) whose low or high half is a
    rejected draw (None: the streams of default_rng(seed))."""
    from runtime.device_env import DeviceEnvBatch

    first, nxt = pack.split(",")
    monkeypatch.setenv("BB_PACK_FIRST", first)
    monkeypatch.setenv("BB_PACK_NEXT", nxt)

    n = 512
    dev = DeviceEnvBatch(n, seeds=[5000 + i for i in range(n)], device=cuda)
    state, acts, refs = crowded_setup(fill, n, reject_at)
    dev.set_state(**state)
    import torch

    act_t = torch.from_numpy(acts).to(cuda)
    dev.step(act_t, want_f64=True, want_info=True)
    st = dev.state()
    rew = dev.reward_f64.cpu().numpy()
    term = dev.terminated.cpu().numpy()
    info = dev.info_host()
    attempts = []
    for i, env in enumerate(refs):
        _, r_ref, t_ref, _, inf = env.step(int(acts[i]))
        attempts.append(env.engine.attempts_last)
        assert rew[i] == r_ref, i
        assert bool(term[i]) == t_ref, i
        assert info[i]["score"] == inf["score"]
        if not t_ref:
            h = int(st["hand"][i])
            assert [(h >> (6 * s)) & 63 for s in range(3)] == env.engine.hand, i
            s = env.engine.rng.bit_generator.state
            assert (int(st["rng"][i, 0]) << 64 | int(st["rng"][i, 1])) == s["state"]["state"], i
            assert bool((h >> 22) & 1) == bool(s["has_uint32"]), i
            if s["has_uint32"]:
                assert int(st["rng"][i, 2]) == s["uinteger"], i
        else:  # terminated -> auto-reset happened; the terminal hand is in info
            h = int(info[i]["term_hand"])
            assert [(h >> (6 * s)) & 63 for s in range(3)] == env.engine.hand, i
    attempts = np.array(attempts)
    assert attempts.max() > 1  # the crowded boards really exercised rejection sampling
    dev.close()
    return attempts


@pytest.mark.parametrize("fill", [0.9, -2.0])
@pytest.mark.parametrize("pack", ["8,32", "1,0"])
def test_lemire_rejection_inside_hand_search(cuda, fill, pack, monkeypatch):
    """A rejected 32-bit draw at a chosen stream position (attempt 0 .. 99,
    low and high halves): the jump-ahead batches of the wave and workgroup
    searches assume three values per attempt and must fall back to the exact
    sequential stream from there on."""
    n = 512
    reject_at = 1 + (np.arange(n) * 37) % 60  # LCG outputs 1 .. 60 = attempts 0 .. 39
    attempts = _crowded(cuda, fill, pack, monkeypatch, reject_at=reject_at)
    reached = attempts > (2 * (reject_at - 1) + (np.arange(n) & 1)) // 3
    # searches that got past their rejected draw: ~60% on the singles-only boards, a few at fill 0.9
    assert reached.sum() > (n // 2 if fill == -2.0 else 4)
