"""GPU parity of the fused rollout kernels vs the CPU restatement.

masked sample: log-prob / entropy within 1e-5 (fp32, north_star tolerance) on
every row, actions equal for the same uniforms except on a stated fp32 CDF
rounding boundary (K_ULP); GAE: bit-exact vs the reference loop in
numpy float32 (the kernel follows numpy's op order with no FMA contraction);
gather: exact expansion of packed rollout records.
"""
import numpy as np
import pytest
import torch

from oracle import bb_ppo as OP
from oracle import philox

pytestmark = pytest.mark.gpu


def _masks(rng, n, p_valid):
    m = rng.random((n, 192)) < p_valid
    m[np.arange(n), rng.integers(0, 192, n)] = True  # at least one legal action
    return m


# A sampled index is index work: it must equal the oracle's except where the oracle's target u * sum(P)
# lies on an fp32 rounding boundary of the CDF.  Bound: each probability of Categorical(softmax) is
# exp (<= 1 ulp on each side: ocml's expf, Sleef's u10 on the CPU) then two roundings to nearest (the
# softmax division and Categorical's renormalisation, 0.5 ulp each on each side), so a GPU P_j is within
# 4 ulps (4 * 2^-24 relative) of the oracle's; the common scale factors cancel in cdf_k / total, so the
# position of the target relative to a CDF boundary can move by at most 2 x 4 = 8 units of 2^-24 * sum(P)
# (the fp64 running sums add nothing at this scale).  K_ULP is that 8.
K_ULP = 8


def _check_sampled(logits, mask, u, a, lp, ent, a_ref):
    """Every sampled action legal; every row where it differs from the oracle's for the same uniform sits
    on a CDF boundary (|u * sum(P) - cdf[min(a, a_ref)]| <= K_ULP * 2^-24 * sum(P)); log-prob and entropy
    within 1e-5 of the oracle evaluated at the GPU's action on EVERY row."""
    n = len(a)
    assert mask[np.arange(n), a].all()  # only legal actions
    diff = np.nonzero(a != a_ref)[0]
    if diff.size:
        cdf = OP.categorical_cdf(logits[diff], mask[diff])
        tot = cdf[:, -1]
        lo = np.minimum(a[diff], a_ref[diff])
        dist = np.abs(np.asarray(u, np.float64)[diff] * tot - cdf[np.arange(diff.size), lo]) / (tot * 2.0 ** -24)
        print(f"{diff.size} of {n} sampled actions differ from the oracle; CDF-boundary distance "
              f"max {dist.max():.2f} x 2^-24 sum(P) (bound {K_ULP})")
        assert (dist <= K_ULP).all(), (diff[dist > K_ULP], dist[dist > K_ULP])
    _, lp_at, ent_ref = OP.masked_categorical(logits, mask, action=a)
    np.testing.assert_allclose(lp, lp_at, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ent, ent_ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("p_valid,scale", [(0.05, 1.0), (0.5, 3.0), (1.0, 10.0), (0.02, 30.0)])
def test_masked_sample_matches_torch_reference(cuda, p_valid, scale):
    from runtime import kernels as K

    rng = np.random.default_rng(int(p_valid * 1000))
    n = 4096
    logits = (rng.standard_normal((n, 192)) * scale).astype(np.float32)
    mask = _masks(rng, n, p_valid)
    u = rng.random(n).astype(np.float32)
    a_ref, lp_ref, ent_ref = OP.masked_categorical(logits, mask, uniform=u.astype(np.float64))
    lg = torch.from_numpy(logits).to(cuda)
    mb = K.pack_mask(torch.from_numpy(mask).to(cuda))
    a, lp, ent = K.masked_sample(lg, mb, uniform=torch.from_numpy(u).to(cuda))
    a, lp, ent = a.cpu().numpy(), lp.cpu().numpy(), ent.cpu().numpy()
    _check_sampled(logits, mask, u, a, lp, ent, a_ref)
    np.testing.assert_allclose(ent, ent_ref, rtol=1e-5, atol=1e-5)
    # evaluating given actions (PPO update path) and argmax
    _, lp2, _ = K.masked_sample(lg, mb, action_in=torch.from_numpy(a_ref).to(cuda))
    np.testing.assert_allclose(lp2.cpu().numpy(), lp_ref, rtol=1e-5, atol=1e-5)
    ad, _, _ = K.masked_sample(lg, mb, deterministic=True)
    a_det, _, _ = OP.masked_categorical(logits, mask, deterministic=True)
    assert np.array_equal(ad.cpu().numpy(), a_det)


def test_masked_sample_philox_uniform_and_distribution(cuda):
    from runtime import kernels as K

    rng = np.random.default_rng(3)
    n = 2048
    logits = rng.standard_normal((n, 192)).astype(np.float32)
    mask = _masks(rng, n, 0.3)
    u = philox.sample_uniform(n, seed=77, step=5, env_offset=100)
    a_ref, _, _ = OP.masked_categorical(logits, mask, uniform=u)
    a, lp, ent = K.masked_sample(torch.from_numpy(logits).to(cuda), K.pack_mask(torch.from_numpy(mask).to(cuda)),
                                 seed=77, step=5, env_offset=100)
    _check_sampled(logits, mask, u, a.cpu().numpy(), lp.cpu().numpy(), ent.cpu().numpy(), a_ref)
    # empirical distribution of one row matches the softmax
    row = np.tile(logits[:1], (200000, 1))
    rm = np.tile(mask[:1], (200000, 1))
    a, _, _ = K.masked_sample(torch.from_numpy(row).to(cuda), K.pack_mask(torch.from_numpy(rm).to(cuda)), seed=1)
    counts = np.bincount(a.cpu().numpy(), minlength=192) / 200000.0
    lg = np.where(mask[0], logits[0], -np.inf)
    p = np.exp(lg - lg.max())
    p /= p.sum()
    assert np.abs(counts - p).max() < 0.01


@pytest.mark.parametrize("T,N", [(128, 64), (128, 4096), (7, 3), (128, 65536)])  # (128, 65536): config 3
def test_gae_bit_exact(cuda, T, N):
    from runtime import kernels as K

    rng = np.random.default_rng(T * N)
    r = rng.standard_normal((T, N)).astype(np.float32)
    v = rng.standard_normal((T, N)).astype(np.float32)
    d = (rng.random((T, N)) < 0.05).astype(np.float32)
    last = rng.standard_normal(N).astype(np.float32)
    adv_ref, ret_ref = OP.gae(r, v, d, last, 0.99, 0.95)
    t = lambda a: torch.from_numpy(a).to(cuda)  # noqa: E731
    adv, ret = K.gae(t(r), t(v), t(d), t(last), 0.99, 0.95)
    np.testing.assert_array_equal(adv.cpu().numpy(), adv_ref)
    np.testing.assert_array_equal(ret.cpu().numpy(), ret_ref)


def test_gather_obs_expansion(cuda):
    from runtime import kernels as K
    from environment._host import board_planes, piece_planes

    rng = np.random.default_rng(0)
    n = 3000
    board = rng.integers(0, 2 ** 63, n, dtype=np.int64)
    hand = (rng.integers(0, 37, (n, 3)) * np.array([1, 64, 4096])).sum(1) | (rng.integers(0, 8, n) << 18)
    hand = hand.astype(np.int32)
    mbits = rng.integers(-2 ** 63, 2 ** 63 - 1, (n, 3), dtype=np.int64)
    idx = rng.permutation(n)[:1000]
    x, mf = K.gather_obs(torch.from_numpy(board).to(cuda), torch.from_numpy(hand).to(cuda),
                         torch.from_numpy(mbits).to(cuda), torch.from_numpy(idx).to(cuda))
    exp_board = board_planes(board.view(np.uint64)[idx])
    exp_pieces = piece_planes(hand.view(np.uint32)[idx])
    assert np.array_equal(x.cpu().numpy()[:, 0], exp_board)
    assert np.array_equal(x.cpu().numpy()[:, 1:], exp_pieces)
    bits = ((mbits.view(np.uint64)[idx][:, :, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1))
    assert np.array_equal(mf.cpu().numpy(), bits.reshape(-1, 192).astype(np.float32))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("n,c,nhwc", [(2048, 128, False), (300, 64, False), (7, 4, False),
                                      (2048, 128, True), (300, 64, True), (5, 8, True)])
def test_fused_batchnorm_matches_torch(cuda, dtype, relu, n, c, nhwc):
    """models.network.BatchNorm2d (HIP bb_bn_forward/backward) vs
    nn.BatchNorm2d [+ ReLU] in training mode: output, running statistics,
    num_batches_tracked, dx / dweight / dbias.  fp32 within 1e-4 (reduction
    order), bf16 within bf16 rounding of the output.  NCHW and channels_last
    (NHWC) layouts; the output keeps the input's layout."""
    from models.network import BatchNorm2d
    from runtime.kernels import bn_fusable

    torch.manual_seed(n + c)
    fmt = torch.channels_last if nhwc else torch.contiguous_format
    x0 = (torch.randn(n, c, 8, 8, device=cuda) * 1.7 + 0.3).to(dtype).contiguous(memory_format=fmt)
    if nhwc and c * x0.element_size() % 16 == 0:
        assert bn_fusable(x0)
    ref = torch.nn.BatchNorm2d(c).to(cuda)
    fus = BatchNorm2d(c, relu=relu).to(cuda)
    with torch.no_grad():
        w, b = torch.rand(c, device=cuda) + 0.5, torch.randn(c, device=cuda) * 0.1
        for m in (ref, fus):
            m.weight.copy_(w)
            m.bias.copy_(b)
    g = torch.randn(n, c, 8, 8, device=cuda).to(dtype).contiguous(memory_format=fmt)
    # fused path
    xf = x0.clone().requires_grad_(True)
    yf = fus(xf)
    if nhwc and bn_fusable(x0):
        assert yf.is_contiguous(memory_format=torch.channels_last)
    yf.backward(g)
    # reference (fp32 on the same values); with the ReLU, its backward takes the
    # fused forward's own mask (ties at the kink may round either way)
    xr = x0.float().clone().requires_grad_(True)
    yr = ref(xr)
    gr = g.float() * (yf.detach() > 0).float() if relu else g.float()
    yr.backward(gr)
    if relu:
        yr = torch.relu(yr)
    outs = [(yr.detach().float(), xr.grad.float(), ref.weight.grad, ref.bias.grad),
            (yf.detach().float(), xf.grad.float(), fus.weight.grad, fus.bias.grad)]
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for a, b_, name in zip(outs[0], outs[1], ("y", "dx", "dweight", "dbias")):
        scale = max(1.0, float(a.abs().max()))
        assert torch.allclose(a, b_, rtol=tol, atol=tol * scale), name
    assert torch.allclose(ref.running_mean, fus.running_mean, rtol=1e-4, atol=1e-5)
    assert torch.allclose(ref.running_var, fus.running_var, rtol=1e-4, atol=1e-5)
    assert int(ref.num_batches_tracked) == int(fus.num_batches_tracked) == 1
    fus.eval()
    ref.eval()
    xe = x0.float()[:5]
    ye = fus(xe)
    assert torch.allclose(torch.relu(ref(xe)) if relu else ref(xe), ye, atol=1e-5)


@pytest.mark.parametrize("channels_last", [False, True])
def test_network_fused_conv_bias_batchnorm_matches_torch(cuda, channels_last):
    """BlockBlastNetwork in training mode with the HIP BatchNorm (conv bias
    folded into it, NCHW or channels_last) vs the same weights on torch's own
    conv(+bias) -> nn.BatchNorm2d -> ReLU (use_fused off), fp32: logits,
    values, every parameter gradient and the BN running statistics.  The conv
    biases feed a BatchNorm, so their true gradient is 0: both sides must be
    at rounding level against the weight gradients."""
    from models.network import BatchNorm2d, BlockBlastNetwork

    torch.manual_seed(11)
    net = BlockBlastNetwork().to(cuda).train()
    ref = BlockBlastNetwork().to(cuda).train()
    ref.load_state_dict(net.state_dict())
    for n in (net, ref):
        for m in n.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
    if channels_last:
        net.to(memory_format=torch.channels_last)
    x = (torch.rand((512, 4, 8, 8), device=cuda) < 0.4).float()
    xin = x.contiguous(memory_format=torch.channels_last) if channels_last else x
    BatchNorm2d.use_fused = True
    lf, vf = net.raw(xin)
    BatchNorm2d.use_fused = False
    try:
        lr_, vr = ref.raw(x)
    finally:
        BatchNorm2d.use_fused = True
    assert torch.allclose(lf, lr_, rtol=1e-4, atol=1e-4 * float(lr_.detach().abs().max()))
    assert torch.allclose(vf, vr, rtol=1e-4, atol=1e-4 * float(vr.detach().abs().max()))
    w = torch.randn_like(lr_)
    ((lf * w).sum() + vf.sum()).backward()
    ((lr_ * w).sum() + vr.sum()).backward()
    named_ref = dict(ref.named_parameters())
    for name, p in net.named_parameters():
        g, gr = p.grad, named_ref[name].grad
        if name.endswith(".bias") and named_ref[name[:-5] + ".weight"].dim() == 4:  # a conv bias
            wscale = float(named_ref[name.replace(".bias", ".weight")].grad.abs().max())
            assert float(g.abs().max()) <= 1e-3 * wscale and float(gr.abs().max()) <= 1e-3 * wscale, name
            continue
        # relative L2 error: single elements of these long reductions (sum over
        # batch x 64 positions) differ more between conv algorithms (MIOpen picks
        # winograd or implicit GEMM per layout) than the norm
        rel = float((g - gr).norm() / gr.norm().clamp_min(1e-30))
        assert rel < 5e-3, (name, rel)
    for (name, b), br in zip(net.named_buffers(), ref.buffers()):
        assert torch.allclose(b.float(), br.float(), rtol=1e-4, atol=1e-5), name


@pytest.mark.parametrize("density", [0.02, 0.3, 1.0])
def test_fused_ppo_loss_matches_torch(cuda, density):
    """bb_ppo_loss_forward/backward (PPOLossFunction) vs the torch ops of
    ppo.py:362-392 (agents.ppo.ppo_loss_torch), fp32: the loss, the six update
    metrics, d/dlogits and d/dvalues.  Rows include single-legal-action masks
    (P = 1: the log-prob clamps and passes no gradient), ratios inside and
    outside the clip range, ratio-1 rows and zero advantages."""
    from agents.ppo import PPOConfig, ppo_loss_torch
    from runtime.kernels import PPOLossFunction

    torch.manual_seed(int(density * 100))
    B = 2048
    cfg = PPOConfig()
    logits = (torch.randn(B, 192, device=cuda) * 3).requires_grad_(True)
    values = torch.randn(B, device=cuda).requires_grad_(True)
    mask = (torch.rand(B, 192, device=cuda) < density).float()
    mask[torch.arange(B, device=cuda), torch.randint(0, 192, (B,), device=cuda)] = 1.0
    mask[:16] = 0.0
    mask[:16, 5] = 1.0
    actions = torch.multinomial(mask, 1).squeeze(1)
    with torch.no_grad():
        lp = torch.log_softmax(logits.masked_fill(mask == 0, float("-inf")), -1).gather(1, actions[:, None])[:, 0]
    old = lp + torch.randn(B, device=cuda) * 0.3
    old[16:32] = lp[16:32]
    adv = torch.randn(B, device=cuda)
    adv[32:40] = 0.0
    ret = torch.randn(B, device=cuda)
    lf, sf = PPOLossFunction.apply(logits, values, mask, actions, old, adv, ret, cfg.clip_epsilon, cfg.value_coef,
                                   cfg.entropy_coef)
    gl_f, gv_f = torch.autograd.grad(lf, [logits, values])
    lr, sr = ppo_loss_torch(logits, values, mask, actions, old, adv, ret, cfg)
    gl_r, gv_r = torch.autograd.grad(lr, [logits, values])
    torch.testing.assert_close(lf, lr.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(sf[:5], sr[:5], rtol=1e-5, atol=1e-6)
    assert abs(float(sf[5] - sr[5])) <= 2.0 / B  # a ratio on the clip boundary may round either way
    torch.testing.assert_close(gv_f, gv_r, rtol=1e-5, atol=1e-9)
    scale = float(gl_r.abs().max())
    torch.testing.assert_close(gl_f, gl_r, rtol=1e-4, atol=1e-5 * scale)
    assert float(gl_f[:16].abs().max()) <= 1e-5 * scale  # clamped log-prob + one-point entropy: no gradient


@pytest.mark.parametrize("density", [0.02, 0.3])
def test_fused_ppo_loss_bf16_inputs_equal_cast_path(cuda, density):
    """bb_ppo_loss_*_bf16 (bf16 logits / values, as the autocast network outputs them) == the fp32 loss on the same
    values widened, then its gradients cast to bf16 (autograd's casts around the fp32 loss): the loss and the
    metrics bit for bit, d/dlogits and d/dvalues bit for bit."""
    from agents.ppo import PPOConfig
    from runtime.kernels import PPOLossFunction

    torch.manual_seed(7 + int(density * 100))
    B = 2048
    cfg = PPOConfig()
    lb = (torch.randn(B, 192, device=cuda) * 3).to(torch.bfloat16)
    vb = torch.randn(B, device=cuda).to(torch.bfloat16)
    mask = (torch.rand(B, 192, device=cuda) < density).float()
    mask[torch.arange(B, device=cuda), torch.randint(0, 192, (B,), device=cuda)] = 1.0
    actions = torch.multinomial(mask, 1).squeeze(1)
    old = -torch.rand(B, device=cuda) * 4
    adv, ret = torch.randn(B, device=cuda), torch.randn(B, device=cuda)
    res = []
    for bf16 in (True, False):
        lg = lb.clone().requires_grad_(True)
        vg = vb.clone().requires_grad_(True)
        x, v = (lg, vg) if bf16 else (lg.float(), vg.float())  # the cast path: autograd casts the gradients back
        loss, stats = PPOLossFunction.apply(x, v, mask, actions, old, adv, ret, cfg.clip_epsilon, cfg.value_coef,
                                            cfg.entropy_coef)
        loss.backward()
        assert lg.grad.dtype == torch.bfloat16 and vg.grad.dtype == torch.bfloat16
        res.append((loss.detach(), stats, lg.grad, vg.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("bf16", [False, True])
def test_fused_ppo_loss_one_launch_equals_two(cuda, bf16):
    """bb_ppo_loss_fused (forward and backward in one launch, the loss gradient given up front as the seed that
    PPOAgent backpropagates with) == bb_ppo_loss_forward + bb_ppo_loss_backward, bit for bit: loss, metrics and
    both gradients; a seed of 0.5 halves the gradients exactly; a backward with another gradient tensor than the
    seed runs the backward kernel; odd batch sizes (the in-kernel finalisation's last block)."""
    from agents.ppo import PPOConfig
    from runtime.kernels import PPOLossFunction

    cfg = PPOConfig()
    for B in (2048, 37, 1):
        torch.manual_seed(B)
        dt = torch.bfloat16 if bf16 else torch.float32
        lb = (torch.randn(B, 192, device=cuda) * 3).to(dt)
        vb = torch.randn(B, device=cuda).to(dt)
        mask = (torch.rand(B, 192, device=cuda) < 0.3).float()
        mask[torch.arange(B, device=cuda), torch.randint(0, 192, (B,), device=cuda)] = 1.0
        actions = torch.multinomial(mask, 1).squeeze(1)
        old = -torch.rand(B, device=cuda) * 4
        adv, ret = torch.randn(B, device=cuda), torch.randn(B, device=cuda)
        args = (mask, actions, old, adv, ret, cfg.clip_epsilon, cfg.value_coef, cfg.entropy_coef)
        out = {}
        for mode in ("two", "fused", "half", "other"):
            lg, vg = lb.clone().requires_grad_(True), vb.clone().requires_grad_(True)
            seed = torch.full((), 0.5 if mode == "half" else 1.0, device=cuda)
            loss, stats = PPOLossFunction.apply(lg, vg, *args, None if mode == "two" else seed)
            loss.backward(torch.ones((), device=cuda) if mode == "other" else (seed if mode != "two" else None))
            out[mode] = (loss.detach(), stats.clone(), lg.grad.clone(), vg.grad.clone())
        for m in ("fused", "other"):
            for a, b in zip(out["two"], out[m]):
                assert torch.equal(a, b), (B, m)
        assert torch.equal(out["half"][2].float(), (out["two"][2].float() * 0.5).to(dt).float())
        assert torch.equal(out["half"][3].float(), (out["two"][3].float() * 0.5).to(dt).float())
