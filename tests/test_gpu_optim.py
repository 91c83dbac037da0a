"""GPU parity of the minibatch-step fusions (csrc/bb_optim.hip, bb_bn_forward_res), through the C-ABI.

bb_adam_clip_step vs torch's own nn.utils.clip_grad_norm_ + torch.optim.Adam
(fp32, the reference's ppo.py:400-401): parameters, moments and clipped
gradients within 2e-6 relative or 2e-7 of the largest element (the norm is summed in fp64 here, per tensor in
fp32 by torch), step counts equal, run-to-run bit-identical.
bb_cast_multi: bit-exact against torch's .to(bfloat16) / .float() casts,
permuted and not.  The network's bf16 forward / backward with the multi-tensor
casts == autocast's per-tensor casts, bit for bit.  The ResidualBlock tail fused
into the BatchNorm pass == BatchNorm -> add -> relu, bit for bit.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(512, 8192), (512,), (7,), (1,), (2049,), (64, 4, 3, 3), (128, 128, 3, 3), (192, 256), (3, 5)]


def _tensors(cuda, seed, shapes=SHAPES, channels_last=True):
    g = torch.Generator(device=cuda).manual_seed(seed)
    ps = []
    for s in shapes:
        p = torch.randn(s, device=cuda, generator=g)
        if channels_last and len(s) == 4:
            p = p.contiguous(memory_format=torch.channels_last)
        ps.append(p)
    return ps


@pytest.mark.parametrize("max_norm", [0.5, 1e9])
def test_adam_clip_matches_torch(cuda, max_norm):
    from runtime import kernels as K

    ref = [torch.nn.Parameter(p) for p in _tensors(cuda, 1)]
    mine = [p.detach().clone() for p in ref]
    opt = torch.optim.Adam(ref, lr=3e-4, eps=1e-5, fused=True)  # the agent's optimizer (ppo.py PPOAgent)
    m = [torch.zeros_like(p) for p in mine]
    v = [torch.zeros_like(p) for p in mine]
    steps = [torch.zeros((), device=cuda) for _ in mine]
    ws = K.adam_clip_workspace([p.numel() for p in mine], cuda)
    norm = torch.zeros((), device=cuda)

    def close(a, b):  # 2e-6 relative, or 2e-7 of the tensor's largest element
        return torch.allclose(a, b, rtol=2e-6, atol=2e-7 * float(b.abs().max()))

    for k in range(4):
        grads = _tensors(cuda, 100 + k)
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        tn = torch.nn.utils.clip_grad_norm_(ref, max_norm)
        opt.step()
        gm = [gr.clone() for gr in grads]
        K.adam_clip_step(mine, gm, m, v, steps, 3e-4, 0.9, 0.999, 1e-5, max_norm, ws, norm)
        assert torch.allclose(norm, tn, rtol=1e-6), (norm, tn)
        for i, p in enumerate(ref):
            st = opt.state[p]
            assert close(gm[i], p.grad), i
            assert close(m[i], st["exp_avg"]), i
            assert close(v[i], st["exp_avg_sq"]), i
            assert close(mine[i], p.detach()), i
            assert float(steps[i]) == float(st["step"]) == k + 1
            assert mine[i].stride() == p.stride()


def test_adam_clip_deterministic(cuda):
    from runtime import kernels as K

    runs = []
    for _ in range(2):
        ps = _tensors(cuda, 5)
        m = [torch.zeros_like(p) for p in ps]
        v = [torch.zeros_like(p) for p in ps]
        steps = [torch.zeros((), device=cuda) for _ in ps]
        ws = K.adam_clip_workspace([p.numel() for p in ps], cuda)
        for k in range(3):
            K.adam_clip_step(ps, _tensors(cuda, 50 + k), m, v, steps, 1e-3, 0.9, 0.999, 1e-5, 0.5, ws)
        runs.append(ps + m + v)
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_adam_clip_rejects_bad_tables(cuda):
    from runtime import kernels as K
    from runtime import lib as L

    ps = _tensors(cuda, 2, shapes=[(4,)] * 49)
    with pytest.raises(L.BBNativeError):
        K.adam_clip_step(ps, ps, ps, ps, [torch.zeros((), device=cuda)] * 49, 1e-3, 0.9, 0.999, 1e-5, 0.5,
                         torch.empty(8, dtype=torch.float64, device=cuda))
    assert L.load().bb_adam_clip_workspace_bytes(0, None) < 0


@pytest.mark.parametrize("bad", [float("nan"), 3e9])
def test_adam_clip_guard_names_the_chunk(cuda, bad):
    """A non-finite or huge gradient-norm operand (the round-5 one-off: a clip norm ~1e10x too large) is
    flagged on the device and raised by the host check with the tensor and element range; a clean step after
    the check leaves the word clear."""
    from runtime import kernels as K
    from runtime import lib as L

    ps = _tensors(cuda, 3)
    gs = _tensors(cuda, 4)
    m = [torch.zeros_like(p) for p in ps]
    v = [torch.zeros_like(p) for p in ps]
    steps = [torch.zeros((), device=cuda) for _ in ps]
    numels = [p.numel() for p in ps]
    names = [f"p{i}" for i in range(len(ps))]
    ws = K.adam_clip_workspace(numels, cuda)
    K.adam_clip_step(ps, gs, m, v, steps, 1e-3, 0.9, 0.999, 1e-5, 0.5, ws)
    K.adam_guard_check(ws, numels, names)  # clean
    gs[0].view(-1)[5000] = bad  # (512, 8192): its chunk 2 holds element 5000
    K.adam_clip_step(ps, gs, m, v, steps, 1e-3, 0.9, 0.999, 1e-5, 0.5, ws)
    with pytest.raises(L.BBNativeError, match=r"p0 elements \[4096, 6144\)"):
        K.adam_guard_check(ws, numels, names)
    gs = _tensors(cuda, 5)
    K.adam_clip_step(ps, gs, m, v, steps, 1e-3, 0.9, 0.999, 1e-5, 0.5, ws)
    K.adam_guard_check(ws, numels, names)  # cleared by the check


def test_counters_rearmed_after_update(cuda):
    """Every hand-off counter block (stream-keyed and capture-owned) is back to zero after bf16 and fp32
    graph-replayed optimizer steps: no launch left a counter armed."""
    from agents import PPOAgent, PPOConfig
    from runtime import kernels as K

    for bf16 in (False, True):
        torch.manual_seed(0)
        agent = PPOAgent(PPOConfig(batch_size=256), device=cuda, sample_seed=1)
        if bf16:
            agent.autocast_dtype = torch.bfloat16
        agent.train()
        g = torch.Generator().manual_seed(1)
        x = (torch.rand((256, 4, 8, 8), generator=g) < 0.4).float().to(cuda)
        masks = (torch.rand((256, 192), generator=g) < 0.3).float()
        masks[:, 0] = 1.0
        act = torch.multinomial(masks, 1, generator=g).squeeze(1).to(cuda)
        ins = (x, masks.to(cuda), act, -torch.rand(256).to(cuda), torch.randn(256).to(cuda), torch.randn(256).to(cuda))
        for _ in range(5):
            agent.train_minibatch(*ins)
        torch.cuda.synchronize()
        blocks = K.counter_blocks()
        assert blocks and all(int(b.abs().sum()) == 0 for b in blocks)
        agent.check_optimizer_guard()
        ent = next(iter(agent._graphs.values()))
        assert getattr(ent[0][0], "bb_counters", None) is not None  # the capture's own block, kept with it


def test_cast_multi_exact(cuda):
    from runtime import kernels as K

    src = _tensors(cuda, 7, shapes=[(512, 8192), (512,), (3,), (2051,), (192, 256), (4, 64), (3, 60)],
                   channels_last=False)
    src[0] *= 1e-3
    src[1][:4] = torch.tensor([float("inf"), float("-inf"), float("nan"), 1.0 + 2 ** -8], device=cuda)
    perms = [(128, 64), (0, 0), (0, 0), (0, 0), (0, 0), (16, 4), (12, 5)]  # (12, 5): the scalar permute
    out = [torch.empty(s.shape, dtype=torch.bfloat16, device=cuda) for s in src]
    K.cast_multi(0, src, out, perms)

    def permuted(t, pc, ph):
        if pc == 0:
            return t
        o = t.shape[0]
        return t.reshape(o, pc, ph).permute(0, 2, 1).reshape(t.shape)

    for s, o, (pc, ph) in zip(src, out, perms):
        want = permuted(s, pc, ph).to(torch.bfloat16)
        assert torch.equal(o.view(torch.int16), want.view(torch.int16)) or torch.equal(
            o.float().nan_to_num(7.0), want.float().nan_to_num(7.0))
    back = [torch.empty(s.shape, dtype=torch.float32, device=cuda) for s in src]
    K.cast_multi(1, out, back, perms)
    for s, b, (pc, ph) in zip(src, back, perms):
        assert torch.equal(b.nan_to_num(7.0), s.to(torch.bfloat16).float().nan_to_num(7.0))


def test_network_fused_casts_equal_autocast(cuda, monkeypatch):
    """bf16 raw() forward + backward: the multi-tensor Linear casts give the
    same logits, values and parameter gradients as autocast's own casts."""
    import models.network as N

    from runtime import kernels as K

    monkeypatch.setattr(N, "LINEAR_RELU", False)  # the casts alone (the epilogue ReLU has its own test,
    monkeypatch.setattr(K, "LINEAR_TAIL", False)  # the fused Linear tails theirs: tests/test_gpu_linear_tail.py)
    torch.manual_seed(0)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    x = (torch.rand((64, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(N, "FUSED_CASTS", fused)
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            lo, va = net.raw(x)
        (lo.float().square().mean() + va.float().sum()).backward()
        res[fused] = (lo.detach().float(), va.detach().float(),
                      {n: p.grad.clone() for n, p in net.named_parameters()})
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    for n, gr in res[True][2].items():
        # Linear gradients are identical; the conv stack sees the same bf16 values (its
        # MIOpen / split-K paths may still differ in the last bits between two backward runs)
        if n.startswith(("fc_encoder", "policy_head", "value_head")):
            assert torch.equal(gr, res[False][2][n]), n
        else:
            assert torch.allclose(gr, res[False][2][n], rtol=1e-2, atol=1e-4), n


@pytest.mark.parametrize("res_mask", [False, True])
@pytest.mark.parametrize("dtype,nhwc", [(torch.float32, False), (torch.float32, True), (torch.bfloat16, True)])
def test_bn_add_relu_equals_composite(cuda, dtype, nhwc, res_mask, monkeypatch):
    """BatchNormAddReLUFunction == BatchNormReLUFunction(relu=False) -> + res ->
    relu, forward, running statistics and every gradient, bit for bit; the backward both ways
    (threshold_backward + bb_bn_backward, and bb_bn_backward_res with the mask inside the passes)."""
    from runtime import kernels as K

    monkeypatch.setattr(K, "RES_MASK", res_mask)

    g = torch.Generator(device=cuda).manual_seed(11)
    fmt = torch.channels_last if nhwc else torch.contiguous_format
    n, c = 96, 128
    x0 = (torch.randn((n, c, 8, 8), device=cuda, generator=g) * 2 + 0.5).to(dtype).contiguous(memory_format=fmt)
    r0 = torch.randn((n, c, 8, 8), device=cuda, generator=g).to(dtype).contiguous(memory_format=fmt)
    pb0 = torch.randn(c, device=cuda, generator=g) * 0.1
    w0 = torch.rand(c, device=cuda, generator=g) + 0.5
    b0 = torch.randn(c, device=cuda, generator=g) * 0.1
    dy = torch.randn((n, c, 8, 8), device=cuda, generator=g).to(dtype).contiguous(memory_format=fmt)
    outs = []
    for fused in (True, False):
        x, r, pb, w, b = (t.clone().requires_grad_(True) for t in (x0, r0, pb0, w0, b0))
        rm, rv = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
        nbt = torch.zeros((), dtype=torch.long, device=cuda)
        if fused:
            y = K.BatchNormAddReLUFunction.apply(x, pb, r, w, b, rm, rv, 0.1, 1e-5, nbt)
        else:
            y = torch.relu(K.BatchNormReLUFunction.apply(x, pb, w, b, rm, rv, 0.1, 1e-5, False, nbt) + r)
        y.backward(dy)
        outs.append([y.detach(), rm, rv, nbt, x.grad, r.grad, pb.grad, w.grad, b.grad])
    for i, (a, bb) in enumerate(zip(*outs)):
        assert torch.equal(a, bb), i


def test_network_res_fused_equals_unfused(cuda, monkeypatch):
    """bf16 training forward + backward of the whole CNN with the ResidualBlock
    tail fused and not: logits, values, BatchNorm statistics and gradients."""
    import models.network as N

    torch.manual_seed(1)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    x = (torch.rand((128, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    res = {}
    from runtime import kernels as K

    # the BatchNorm sums from the convolutions' store passes follow the block's wiring (bn1's backward takes
    # them from conv2 only in the fused block): off here, compared on their own in test_gpu_conv.py
    monkeypatch.setattr(K, "CONV_STATS", False)
    for fused in (True, False):
        monkeypatch.setattr(N, "RES_FUSED", fused)
        net.load_state_dict(state0)
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            lo, va = net.raw(x)
        (lo.float().square().mean() + va.float().sum()).backward()
        res[fused] = (lo.detach().float(), va.detach().float(),
                      {n: p.grad.clone() for n, p in net.named_parameters()},
                      {k: v.clone() for k, v in net.state_dict().items()})
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    for k, v in res[True][3].items():
        assert torch.equal(v, res[False][3][k]), k
    for n, gr in res[True][2].items():
        if n.startswith("conv_encoder.0."):  # MIOpen's first-layer weight gradient may differ in the last bits
            assert torch.allclose(gr, res[False][2][n], rtol=1e-2, atol=1e-4), n
        else:
            assert torch.equal(gr, res[False][2][n]), n


def test_linear_relu_epilogue(cuda):
    """LinearReLUFunction (ReLU in the GEMM epilogue) vs relu(F.linear) in bf16:
    outputs within one bf16 rounding, gradients within bf16 accumulation noise."""
    from runtime import kernels as K

    g = torch.Generator(device=cuda).manual_seed(4)
    x0 = torch.randn((2048, 512), device=cuda, generator=g).to(torch.bfloat16)
    w0 = (torch.randn((256, 512), device=cuda, generator=g) * 0.05).to(torch.bfloat16)
    b0 = (torch.randn(256, device=cuda, generator=g) * 0.1).to(torch.bfloat16)
    gy = torch.randn((2048, 256), device=cuda, generator=g).to(torch.bfloat16)
    outs = []
    for fused in (True, False):
        x, w, b = (t.clone().requires_grad_(True) for t in (x0, w0, b0))
        y = K.LinearReLUFunction.apply(x, w, b) if fused else torch.relu(torch.nn.functional.linear(x, w, b))
        y.backward(gy)
        outs.append((y.detach().float(), x.grad.float(), w.grad.float(), b.grad.float()))
    (y1, *g1), (y2, *g2) = outs
    assert torch.allclose(y1, y2, rtol=8e-3, atol=1e-3)
    assert ((y1 > 0) == (y2 > 0)).float().mean() > 0.999
    for a, bb in zip(g1, g2):
        assert float((a - bb).norm() / bb.norm()) < 1e-2


def test_network_prep_multi_equals_per_layer(cuda, monkeypatch):
    """The HIP convolutions' bf16 weight images from one bb_conv3x3_prep_multi
    launch == one bb_conv3x3_prep per layer: the bf16 training forward and
    backward are bit-identical."""
    import models.network as N
    from runtime import kernels as K

    torch.manual_seed(2)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    convs = [m for m in net.conv_encoder.modules() if isinstance(m, torch.nn.Conv2d) and m.in_channels >= 64]
    for c, (wf, wd) in zip(convs, K.conv3x3_prep_multi([c.weight for c in convs])):
        n = c.weight.shape[0] * c.weight.shape[1] * 9
        wf1, wd1 = (torch.empty(n, dtype=torch.bfloat16, device=cuda) for _ in range(2))
        assert K.L.load().bb_conv3x3_prep(K._p(c.weight), c.in_channels, c.out_channels, K._w_layout(c.weight),
                                          K._p(wf1), K._p(wd1), K._s(cuda)) == 0
        assert torch.equal(wf.view(torch.int16), wf1.view(torch.int16))
        assert torch.equal(wd.view(torch.int16), wd1.view(torch.int16))
    x = (torch.rand((64, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    res = {}
    for multi in (True, False):
        monkeypatch.setattr(N, "PREP_MULTI", multi)
        net.load_state_dict(state0)
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            lo, va = net.raw(x)
        (lo.float().square().mean() + va.float().sum()).backward()
        res[multi] = (lo.detach().float(), va.detach().float(),
                      {n: p.grad.clone() for n, p in net.named_parameters()})
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
    for n, gr in res[True][2].items():
        if n.startswith("conv_encoder.0."):  # MIOpen's first-layer weight gradient may differ in the last bits
            assert torch.allclose(gr, res[False][2][n], rtol=1e-2, atol=1e-4), n
        else:
            assert torch.equal(gr, res[False][2][n]), n


def test_update_direct_gather_equals_copies(cuda, monkeypatch):
    """PPOAgent.update gathering packed minibatches straight into the captured
    step's inputs == gathering into fresh tensors and copying them in."""
    from agents import PPOAgent, PPOConfig
    from training.trainer import DeviceRollout

    results = []
    for direct in (True, False):
        torch.manual_seed(5)
        agent = PPOAgent(PPOConfig(batch_size=256, num_epochs=2), device=cuda, sample_seed=3)
        agent.autocast_dtype = torch.bfloat16
        agent.train()
        if not direct:
            monkeypatch.setattr(agent, "minibatch_inputs", lambda b: None)
        roll = DeviceRollout(1024, 0, 1024, 42, {}, 4, cuda)
        roll.reset()
        roll.collect(agent)
        torch.manual_seed(6)
        stats = agent.update(roll.buffer, agent.values_device(roll.x), batch_size=256)
        results.append((stats, [p.detach().clone() for p in agent.network.parameters()]))
        roll.close()
    # MIOpen's first-layer weight gradient (split-K with atomics) differs in the last bits from run to
    # run, so the two agents drift by rounding only
    for k, v in results[0][0].items():
        assert abs(v - results[1][0][k]) <= 1e-3 * max(1.0, abs(v)), k
    for a, b in zip(results[0][1], results[1][1]):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-5)


def test_network_res_grad_fused_equals_unfused(cuda, monkeypatch):
    """The identity path's input gradient added in conv1's data-gradient store
    pass (bb_conv3x3_forward_add) == autograd's separate add, bit for bit, for
    the whole bf16 CNN (its other convolutions on the HIP kernels too)."""
    import models.network as N

    torch.manual_seed(8)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    x = (torch.rand((256, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(N, "RES_GRAD_FUSED", fused)
        net.load_state_dict(state0)
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            lo, va = net.raw(x)
        (lo.float().square().mean() + va.float().sum()).backward()
        res[fused] = {n: p.grad.clone() for n, p in net.named_parameters()}
    for n, gr in res[True].items():
        if n.startswith("conv_encoder.0."):  # MIOpen's first-layer weight gradient may differ in the last bits
            assert torch.allclose(gr, res[False][n], rtol=1e-2, atol=1e-4), n
        else:
            assert torch.equal(gr, res[False][n]), n


def test_conv3x3_forward_add(cuda):
    """bb_conv3x3_forward_add == bf16(conv) + add, rounded once more."""
    from runtime import kernels as K

    g = torch.Generator(device=cuda).manual_seed(12)
    n = 33
    x = torch.randn((n, 128, 8, 8), device=cuda, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn((128, 128, 3, 3), device=cuda, generator=g) * 0.04
    a = torch.randn((n, 128, 8, 8), device=cuda, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    y0 = K.Conv3x3Function.apply(x, w)
    wf, wd = K.conv3x3_prep_multi([w])[0]
    y1 = torch.empty_like(y0)
    lib = K.L.load()
    assert lib.bb_conv3x3_forward_add(K._p(x), K._p(wf), n, 128, 128, K._p(a), K._p(y1), K._s(cuda)) == 0
    assert torch.equal(y1.view(torch.int16), (y0 + a).view(torch.int16))


@pytest.mark.parametrize("graphs", [False, True])
def test_deferred_wgrad_equals_inline(cuda, monkeypatch, graphs):
    """The opt-in side-stream weight gradients (runtime.kernels.deferred_wgrad, BB_ASYNC_WGRAD=1): the bf16
    optimizer step with the board convolutions' weight gradients on a side stream, joined before clip + Adam,
    eager and graph-captured, equals the step with them inline (the same kernels and values; the weights after three
    steps agree up to the run-to-run rounding of MIOpen's first-layer weight gradient, which uses atomics)."""
    import runtime.kernels as K
    from agents import PPOAgent, PPOConfig

    g = torch.Generator().manual_seed(3)
    b = 512
    x = (torch.rand(b, 4, 8, 8, generator=g) < 0.4).float().to(cuda)
    mask = (torch.rand(b, 192, generator=g) < 0.3).float()
    mask[:, 0] = 1.0
    act = torch.multinomial(mask, 1, generator=g).squeeze(1).to(cuda)
    mask = mask.to(cuda)
    old = (-3.0 * torch.rand(b, generator=g)).to(cuda)
    adv, ret = torch.randn(b, generator=g).to(cuda), torch.randn(b, generator=g).to(cuda)
    res = {}
    for on in (False, True):
        monkeypatch.setattr(K, "ASYNC_WGRAD", on)
        torch.manual_seed(0)
        agent = PPOAgent(PPOConfig(batch_size=b), device=cuda, sample_seed=1)
        agent.autocast_dtype = torch.bfloat16
        agent.use_graphs = graphs
        agent.train()
        for m in agent.network.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
        for _ in range(3):
            agent.train_minibatch(x, mask, act, old, adv, ret)
        torch.cuda.synchronize()
        res[on] = {n: p.detach().clone() for n, p in agent.network.named_parameters()}
    for n, p in res[True].items():
        if n.startswith("conv_encoder.0."):
            assert torch.allclose(p, res[False][n], rtol=1e-3, atol=1e-5), n
        else:
            assert torch.allclose(p, res[False][n], rtol=1e-4, atol=1e-6), n
