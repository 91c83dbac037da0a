"""GPU parity of the bf16 Linear tails (csrc/bb_optim.hip: bb_dropout_forward, bb_linear_bgrad), through the
C-ABI.

bb_linear_bgrad: g bit-exact against torch's masked scale -> threshold_backward chain (network.py:89-117's
nn.Dropout after nn.ReLU; autograd rounds each to bf16), the bias gradient within one bf16 rounding of the
fp64 column sum (f32 sums in a fixed order: run-to-run identical).  bb_dropout_forward: kept elements exactly
bf16(y * 1/(1-p)), the drop rate within 5 sigma of p, a new mask per launch and per graph replay, the same mask
for the same generator word.  The network's bf16 training step with the fused tails: equal to torch's tails
with dropout at 0 (forward bit-exact), and graph replays equal to eager steps with dropout at 0.1 (the same
generator words).  Dropout masks are not torch's stream (neither side can reproduce the other's RNG); parity of
the mask is its distribution.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.parametrize("rows,cols,masked,scale", [(2048, 512, True, 1 / 0.9), (2048, 256, True, 1.0),
                                                    (2048, 192, False, 1.0), (2048, 1, False, 1.0),
                                                    (37, 24, True, 1.25), (1000, 100, True, 1 / 0.9),
                                                    (5, 7, False, 1.0)])
def test_linear_bgrad_matches_torch(cuda, rows, cols, masked, scale):
    from runtime import kernels as K

    g0 = torch.Generator(device=cuda).manual_seed(rows * 131 + cols)
    gy = _bf(torch.randn((rows, cols), device=cuda, generator=g0))
    yd = _bf(torch.randn((rows, cols), device=cuda, generator=g0)).clamp_min(0) if masked else None
    if masked:
        yd[::7] = 0.0  # whole rows dropped / below the ReLU
        yd[:, ::5] = -0.0
    g, db = K.linear_bgrad(gy, yd, scale)
    if masked:
        ref = torch.where(yd > 0, _bf(gy.float() * scale), torch.zeros_like(gy))
        assert torch.equal(g, ref)
    else:
        ref = gy
        assert g.data_ptr() == gy.data_ptr()
    exact = ref.double().sum(0)
    tol = 2.0 ** -8 * exact.abs() + 1e-5 * ref.double().abs().sum(0) + 1e-30
    assert bool(((db.double() - exact).abs() <= tol).all())
    assert db.dtype == torch.bfloat16 and db.shape == (cols,)
    g2, db2 = K.linear_bgrad(gy, yd, scale)
    assert torch.equal(db, db2) and torch.equal(g, g2)
    # torch's own bf16 reduction agrees but for the last bit of a few columns
    assert float((db == ref.sum(0)).float().mean()) > 0.9


def _bf16_near(out, ref, what):
    """bf16 out within one bf16 rounding of the fp64 reference (plus f32 summation noise)."""
    err = (out.double() - ref).abs()
    tol = 2.0 ** -8 * ref.abs() + 1e-5 * float(ref.abs().max())
    assert bool((err <= tol).all()), (what, float((err - tol).max()))


@pytest.mark.parametrize("rows,n,k", [(2048, 128, 256), (2048, 192, 256), (2048, 256, 512), (2048, 512, 512),
                                      (37, 32, 64), (1000, 64, 96), (5, 32, 32)])
def test_linear_wgrad_matches_fp64(cuda, rows, n, k):
    """bb_linear_wgrad: g^T x within one bf16 rounding of fp64, deterministic; rows not a multiple of 64."""
    from runtime import kernels as K

    g0 = torch.Generator(device=cuda).manual_seed(rows + n + k)
    g = _bf(torch.randn((rows, n), device=cuda, generator=g0))
    x = _bf(torch.randn((rows, k), device=cuda, generator=g0)).clamp_min(0)
    dw = K.linear_wgrad(g, x)
    assert dw.shape == (n, k) and dw.dtype == torch.bfloat16
    _bf16_near(dw, g.double().t().mm(x.double()), "linear_wgrad")
    assert torch.equal(dw, K.linear_wgrad(g, x))


@pytest.mark.parametrize("rows,k,bias", [(2048, 128, True), (37, 128, True), (1000, 64, False), (3, 8, True)])
def test_linear_n1_matches_fp64(cuda, rows, k, bias):
    """bb_linear_n1_forward / _backward (the value head's Linear(128, 1)): y, dW, db within one bf16 rounding of
    fp64; dx bit-exact (the K = 1 product rounded once, as the GEMM)."""
    from runtime import kernels as K

    g0 = torch.Generator(device=cuda).manual_seed(rows + k)
    x0 = _bf(torch.randn((rows, k), device=cuda, generator=g0)).clamp_min(0)
    w0 = _bf(torch.randn((1, k), device=cuda, generator=g0) * 0.1)
    b0 = _bf(torch.randn(1, device=cuda, generator=g0)) if bias else None
    gy = _bf(torch.randn((rows, 1), device=cuda, generator=g0))
    assert K.linear_n1_ok(x0, w0)
    x, w = x0.clone().requires_grad_(True), w0.clone().requires_grad_(True)
    b = b0.clone().requires_grad_(True) if bias else None
    y = K.LinearN1Function.apply(x, w, b)
    ref = x0.double().mm(w0.double().t()) + (b0.double() if bias else 0.0)
    _bf16_near(y, ref, "y")
    y.backward(gy)
    assert torch.equal(x.grad, _bf(gy.float() * w0.float()))
    _bf16_near(w.grad, gy.double().t().mm(x0.double()), "dW")
    if bias:
        _bf16_near(b.grad, gy.double().sum(0), "db")


def _dropout(y, p, rng):
    from runtime import kernels as K
    from runtime import lib as L

    L.check(L.load().bb_dropout_forward(K._p(y), y.numel(), float(p), K._p(rng), K._s(y.device)), "dropout")


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_dropout_forward_statistics(cuda, p):
    import struct

    g0 = torch.Generator(device=cuda).manual_seed(5)
    y0 = _bf(torch.rand((2048, 512), device=cuda, generator=g0) + 0.25)  # all > 0: a 0 is a drop
    rng = torch.tensor([12345, 0, 0, 0], dtype=torch.int64, device=cuda)
    scale = 1.0 / struct.unpack("f", struct.pack("f", 1.0 - p))[0]
    masks = []
    for k in range(3):
        y = y0.clone()
        _dropout(y, p, rng)
        kept = y != 0
        assert torch.equal(y[kept], _bf(y0.float() * scale)[kept])
        frac = 1.0 - float(kept.float().mean())
        sigma = (p * (1 - p) / y.numel()) ** 0.5
        assert abs(frac - p) < 5 * sigma, (k, frac)
        masks.append(kept)
        assert rng.tolist() == [12345, k + 1, 0, 0]
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])
    # columns and rows carry no pattern: per-column drop rates within 6 sigma
    col = 1.0 - masks[0].float().mean(0)
    assert float((col - p).abs().max()) < 6 * (p * (1 - p) / 2048) ** 0.5
    # the same generator word draws the same mask
    rng.copy_(torch.tensor([12345, 0, 0, 0]))
    y = y0.clone()
    _dropout(y, p, rng)
    assert torch.equal(y != 0, masks[0])


def test_dropout_graph_replays_draw_new_masks(cuda):
    y0 = _bf(torch.rand((256, 256), device=cuda) + 0.25)
    rng = torch.tensor([7, 0, 0, 0], dtype=torch.int64, device=cuda)
    y = y0.clone()
    side = torch.cuda.Stream(cuda)
    side.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(side):
        _dropout(y, 0.1, rng)  # warm-up launch (offset 0 -> 1)
    torch.cuda.current_stream(cuda).wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side):
        _dropout(y, 0.1, rng)
    masks = []
    for _ in range(3):
        y.copy_(y0)
        graph.replay()
        masks.append(y != 0)
    torch.cuda.synchronize()
    assert rng.tolist() == [7, 4, 0, 0]
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])


def test_linear_relu_dropout_function(cuda):
    """LinearReLUFunction with dropout: the output is the epilogue-ReLU GEMM's, scaled where kept; the
    gradients are the GEMMs of torch's masked-scale + threshold gradient (dx, dw bit-exact)."""
    import struct

    from runtime import kernels as K

    g0 = torch.Generator(device=cuda).manual_seed(8)
    x0 = _bf(torch.randn((2048, 512), device=cuda, generator=g0))
    w0 = _bf(torch.randn((256, 512), device=cuda, generator=g0) * 0.05)
    b0 = _bf(torch.randn(256, device=cuda, generator=g0) * 0.1)
    gy = _bf(torch.randn((2048, 256), device=cuda, generator=g0))
    rng = torch.tensor([99, 0, 0, 0], dtype=torch.int64, device=cuda)
    x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
    y = K.LinearReLUFunction.apply(x, w, b, 0.1, rng)
    y.backward(gy)
    scale = 1.0 / struct.unpack("f", struct.pack("f", 0.9))[0]
    yr = torch._addmm_activation(b0, x0, w0.t())
    kept = y != 0
    assert torch.equal(y[kept], _bf(yr.float() * scale)[kept])
    assert bool((yr[~kept] == 0).sum() + (yr[~kept] > 0).sum() == (~kept).sum())
    live = yr > 0
    frac = float((~kept & live).sum()) / float(live.sum())
    assert abs(frac - 0.1) < 0.01, frac
    g = torch.where(y > 0, _bf(gy.float() * scale), torch.zeros_like(gy))
    assert torch.equal(x.grad, g.mm(w0))
    _bf16_near(w.grad, g.double().t().mm(x0.double()), "dw")
    exact = g.double().sum(0)
    assert bool(((b.grad.double() - exact).abs() <= 2.0 ** -8 * exact.abs() + 1e-5 * g.double().abs().sum(0)).all())


def test_network_linear_tail_equals_torch_tails(cuda, monkeypatch):
    """bf16 raw() forward + backward with dropout at 0: the fused tails (bb_linear_bgrad, LinearBiasFunction)
    give torch's logits and values bit for bit and its Linear gradients within bf16 rounding."""
    import models.network as N
    from runtime import kernels as K

    torch.manual_seed(0)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    x = (torch.rand((512, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    res = {}
    monkeypatch.setattr(N, "HEADS_FUSED", False)  # the joint heads GEMM is test_heads_function_*'s
    for tail in (True, False):
        monkeypatch.setattr(K, "LINEAR_TAIL", tail)
        net.load_state_dict(state0)
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            lo, va = net.raw(x)
        (lo.float().square().mean() + va.float().sum()).backward()
        res[tail] = (lo.detach().float(), va.detach().float(), {n: p.grad.clone() for n, p in net.named_parameters()})
    assert torch.equal(res[True][0], res[False][0])
    # the value head's one-output layer sums in another order (bb_linear_n1_forward): one bf16 rounding apart
    assert torch.allclose(res[True][1], res[False][1], rtol=2.0 ** -7, atol=1e-6)
    for n, gr in res[True][2].items():
        ref = res[False][2][n]
        rel = float((gr - ref).norm() / ref.norm().clamp_min(1e-30))
        assert rel < 1e-2, (n, rel)


def _heads_params(cuda, k, seed):
    """bf16 head weights with wp0 / wv0 and bp0 / bv0 back to back (as the network's shadow buffer)."""
    g0 = torch.Generator(device=cuda).manual_seed(seed)
    w_cat = _bf(torch.randn((384, k), device=cuda, generator=g0) * 0.05)
    b_cat = _bf(torch.randn(384, device=cuda, generator=g0) * 0.1)
    wp2 = _bf(torch.randn((192, 256), device=cuda, generator=g0) * 0.05)
    bp2 = _bf(torch.randn(192, device=cuda, generator=g0) * 0.1)
    wv2 = _bf(torch.randn((1, 128), device=cuda, generator=g0) * 0.1)
    bv2 = _bf(torch.randn(1, device=cuda, generator=g0))
    return w_cat, b_cat, wp2, bp2, wv2, bv2


@pytest.mark.parametrize("rows,k", [(2048, 512), (1000, 256), (37, 64)])
def test_heads_function_matches_fp64(cuda, rows, k):
    """HeadsFunction (both heads' first layers as one GEMM + ReLU epilogue, the policy's last layer on a column
    slice, the value's on bb_linear_n1_forward; backward through bb_linear_bgrad2 and one dh GEMM): every
    stage within one bf16 rounding of fp64 on the same bf16 operands, the ReLU-masked hidden gradient exact."""
    from runtime import kernels as K

    w_cat, b_cat, wp2, bp2, wv2, bv2 = _heads_params(cuda, k, rows + k)
    g0 = torch.Generator(device=cuda).manual_seed(k)
    h0 = _bf(torch.randn((rows, k), device=cuda, generator=g0)).clamp_min(0)
    glog = _bf(torch.randn((rows, 192), device=cuda, generator=g0))
    gval = _bf(torch.randn((rows, 1), device=cuda, generator=g0))
    leaves = [t.clone().requires_grad_(True) for t in (h0, w_cat, b_cat, wp2, bp2, wv2, bv2)]
    h, wc, bc, p2, pb2, v2, vb2 = leaves
    wp0, wv0, bp0, bv0 = wc[:256], wc[256:], bc[:256], bc[256:]
    assert K.heads_ok(h0, wp0.detach(), bp0.detach(), wv0.detach(), bv0.detach(), wp2, bp2, wv2, bv2)
    logits, value = K.HeadsFunction.apply(h, wp0, bp0, wv0, bv0, p2, pb2, v2, vb2)
    torch.autograd.backward([logits, value], [glog, gval])
    y = torch._addmm_activation(b_cat, h0, w_cat.t())
    _bf16_near(y, (h0.double().mm(w_cat.double().t()) + b_cat.double()).clamp_min(0), "y")
    _bf16_near(logits, y[:, :256].double().mm(wp2.double().t()) + bp2.double(), "logits")
    _bf16_near(value, y[:, 256:].double().mm(wv2.double().t()) + bv2.double(), "value")
    dyp = glog.mm(wp2)
    dyv = _bf(gval.float() * wv2.float())
    g = torch.where(y > 0, torch.cat([dyp, dyv], 1), torch.zeros_like(y))
    _bf16_near(h.grad, g.double().mm(w_cat.double()), "dh")
    _bf16_near(wc.grad, g.double().t().mm(h0.double()), "dW first layers")
    _bf16_near(bc.grad, g.double().sum(0), "db first layers")
    _bf16_near(p2.grad, glog.double().t().mm(y[:, :256].double()), "dW policy")
    _bf16_near(pb2.grad, glog.double().sum(0), "db policy")
    _bf16_near(v2.grad, gval.double().t().mm(y[:, 256:].double()), "dW value")
    _bf16_near(vb2.grad, gval.double().sum(0), "db value")


def test_network_heads_fused_equals_separate(cuda, monkeypatch):
    """bf16 raw() forward + backward with the heads as one HeadsFunction == the heads layer by layer: logits
    and values within a bf16 rounding, every parameter gradient within 1% (relative norm); the Linear
    shadows lie in one buffer with the heads' first layers adjacent."""
    import models.network as N

    torch.manual_seed(0)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    x = (torch.rand((512, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(N, "HEADS_FUSED", fused)
        net.load_state_dict(state0)
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            if fused:
                h, sh = net._trunk(x)
                wp0, wv0 = sh[net.policy_head[0]][0], sh[net.value_head[0]][0]
                assert wv0.data_ptr() == wp0.data_ptr() + 2 * wp0.numel()
            lo, va = net.raw(x)
        (lo.float().square().mean() + va.float().sum()).backward()
        res[fused] = (lo.detach().float(), va.detach().float(), {n: p.grad.clone() for n, p in net.named_parameters()})
    assert torch.allclose(res[True][0], res[False][0], rtol=2.0 ** -7, atol=1e-3)
    assert torch.allclose(res[True][1], res[False][1], rtol=2.0 ** -7, atol=1e-3)
    conv_bias = {n + ".bias" for n, m in net.named_modules() if isinstance(m, torch.nn.Conv2d)}
    for n, gr in res[True][2].items():
        if n in conv_bias:
            continue  # a bias before training-mode BatchNorm: its gradient is 0 up to rounding noise
        ref = res[False][2][n]
        rel = float((gr - ref).norm() / ref.norm().clamp_min(1e-30))
        assert rel < 1e-2, (n, rel)


def test_graphed_step_with_dropout_matches_eager(cuda):
    """bf16 train_minibatch with dropout 0.1 replayed from a HIP graph == the eager steps: the capture
    restores the dropout generator word, so replay k draws eager step k's masks."""
    from agents import PPOAgent, PPOConfig

    def make():
        torch.manual_seed(3)
        a = PPOAgent(PPOConfig(batch_size=256), device=cuda, sample_seed=1)
        a.autocast_dtype = torch.bfloat16
        a.train()
        return a

    g = torch.Generator(device=cuda).manual_seed(9)
    B = 256
    eager, graphed = make(), make()
    eager.use_graphs = False
    assert graphed.use_graphs
    for k in range(3):
        x = (torch.rand((B, 4, 8, 8), device=cuda, generator=g) < 0.4).float()
        m = (torch.rand((B, 192), device=cuda, generator=g) < 0.3).float()
        m[:, 0] = 1.0
        a = torch.multinomial(m, 1, generator=g).squeeze(1)
        lp = -torch.rand(B, device=cuda, generator=g) * 4
        adv = torch.randn(B, device=cuda, generator=g)
        ret = torch.randn(B, device=cuda, generator=g)
        s_e = eager.train_minibatch(x, m, a, lp, adv, ret).clone()
        s_g = graphed.train_minibatch(x, m, a, lp, adv, ret).clone()
        tol = 2e-2 if k == 0 else 1.5e-1
        assert torch.allclose(s_e, s_g, rtol=tol, atol=tol), (k, s_e, s_g)
    re = eager.network._dropout_rng(cuda)
    rg = graphed.network._dropout_rng(cuda)
    torch.cuda.synchronize()
    assert re.tolist() == rg.tolist() and re.tolist()[1] == 6  # two dropout layers, three steps
