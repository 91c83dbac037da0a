"""The CNN's 3x3 / pad-1 convolutions on bf16 MFMA (csrc/bb_conv.hip) against
torch's f32 convolution of the same bf16 values (network.py:75-117 layers,
nn.Conv2d under bf16 autocast).

Tolerances: forward and data gradient are f32 accumulations rounded to bf16,
so each element equals the f32 reference rounded to bf16 or a neighbour one
bf16 step away (different summation order); the weight gradient is f32 and
within 1e-4 of the largest element (sums over N x 64 pixels in a different
order)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [(64, 64), (64, 128), (128, 64), (128, 128)]


def _bf16_close(out: torch.Tensor, ref: torch.Tensor, what: str):
    """out (bf16) vs the f32 reference: within one bf16 step of round(ref)."""
    o = out.float()
    r = ref.float()
    step = (r.abs() * 2.0 ** -7).clamp_min(1e-30)  # one bf16 ulp is 2^-7 relative at worst
    bad = (o - r).abs() > step + 1e-6 * float(r.abs().max())
    assert int(bad.sum()) == 0, f"{what}: {int(bad.sum())} elements off by more than one bf16 step"
    exact = (o == r.bfloat16().float()).float().mean()
    assert float(exact) > 0.97, f"{what}: only {float(exact):.3f} equal to the rounded reference"


def _inputs(cuda, n, cin, cout, seed, layout):
    g = torch.Generator(device=cuda).manual_seed(seed)
    x = torch.randn((n, cin, 8, 8), device=cuda, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn((cout, cin, 3, 3), device=cuda, generator=g) * (2.0 / (9 * cin)) ** 0.5
    if layout == 1:
        w = w.contiguous(memory_format=torch.channels_last)
    dy = torch.randn((n, cout, 8, 8), device=cuda, generator=g).bfloat16().contiguous(
        memory_format=torch.channels_last)
    return x, w, dy


@pytest.mark.parametrize("cin,cout", SHAPES)
@pytest.mark.parametrize("n", [1, 3, 6, 257, 1000, 2048])
def test_conv3x3_forward_and_data_grad(cuda, lib, cin, cout, n):
    from runtime.kernels import Conv3x3Function

    x, w, dy = _inputs(cuda, n, cin, cout, 100 + n + cin + cout, layout=n % 2)
    wb = w.bfloat16().float()
    y = Conv3x3Function.apply(x, w)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    _bf16_close(y, F.conv2d(x.float(), wb, padding=1), "forward")
    xg = x.clone().requires_grad_(True)
    yg = Conv3x3Function.apply(xg, w)
    yg.backward(dy)
    ref_dx = torch.nn.grad.conv2d_input(x.shape, wb, dy.float(), padding=1)
    _bf16_close(xg.grad, ref_dx, "data gradient")


@pytest.mark.parametrize("cin,cout", SHAPES)
@pytest.mark.parametrize("n,layout", [(1, 0), (5, 1), (64, 0), (2048, 1)])
def test_conv3x3_weight_grad(cuda, lib, cin, cout, n, layout):
    from runtime.kernels import Conv3x3Function

    x, w, dy = _inputs(cuda, n, cin, cout, 7 * n + cin - cout, layout)
    wp = w.clone().requires_grad_(True)
    y = Conv3x3Function.apply(x, wp)
    y.backward(dy)
    ref = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), padding=1)
    g = wp.grad
    assert g.dtype == torch.float32 and g.shape == w.shape
    if layout == 1:
        assert g.is_contiguous(memory_format=torch.channels_last)
    err = float((g - ref).abs().max())
    assert err <= 1e-4 * float(ref.abs().max()), err
    # deterministic: the same call again is bit-identical
    wp2 = w.clone().requires_grad_(True)
    Conv3x3Function.apply(x, wp2).backward(dy)
    assert torch.equal(wp2.grad, g)


def test_conv3x3_taps_and_board_edges(cuda, lib):
    """One-hot inputs and weights: every (tap, pixel) pair lands where conv2d
    puts it, including the zero padding at all four board edges."""
    from runtime.kernels import Conv3x3Function

    n, c = 64, 64
    x = torch.zeros((n, c, 8, 8), device=cuda)
    for b in range(n):
        x[b, b % c, b // 8, b % 8] = 1.0 + b / 64  # one pixel per board, every position once
    x = x.bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.zeros((c, c, 3, 3), device=cuda)
    for t in range(9):
        w[(5 * t) % c, :, t // 3, t % 3] = 1.0 + t  # output channel 5t sees tap t only
    y = Conv3x3Function.apply(x, w)
    ref = F.conv2d(x.float(), w, padding=1)
    assert torch.equal(y.float(), ref.bfloat16().float())


def test_network_bf16_hip_conv_matches_miopen(cuda, lib):
    """BlockBlastNetwork training forward + backward under bf16 autocast with
    the HIP convolutions, and the same network on torch's (MIOpen) bf16
    convolutions, both against the f32 network: the HIP path is as close to
    f32 as MIOpen's bf16 path (logits, values, every parameter gradient,
    relative L2)."""
    import models.network as NW
    from models.network import BlockBlastNetwork

    torch.manual_seed(5)
    nets = [BlockBlastNetwork().to(cuda).train().to(memory_format=torch.channels_last) for _ in range(3)]
    for m in nets[1:]:
        m.load_state_dict(nets[0].state_dict())
    for net in nets:
        for m in net.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
    x = (torch.rand((512, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    wgt = None
    outs = []
    for model, mode in zip(nets, ("hip", "miopen", "f32")):
        NW.HIP_CONV = mode == "hip"
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False, enabled=mode != "f32"):
                lo, va = model.raw(x)
        finally:
            NW.HIP_CONV = True
        lo, va = lo.float(), va.float()
        if wgt is None:
            wgt = torch.randn_like(lo)
        ((lo * wgt).sum() + va.sum()).backward()
        outs.append((lo.detach(), va.detach(), {k: p.grad for k, p in model.named_parameters()}))

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    (lh, vh, gh), (lm, vm, gm), (l32, v32, g32) = outs
    rows = [("logits", rel(lh, l32), rel(lm, l32)), ("values", rel(vh, v32), rel(vm, v32))]
    for name, p in nets[2].named_parameters():
        if name.endswith(".bias") and p.dim() == 1 and dict(nets[2].named_parameters())[name[:-5] + ".weight"].dim() == 4:
            continue  # conv biases feed a BatchNorm: true gradient 0
        rows.append((name, rel(gh[name], g32[name]), rel(gm[name], g32[name])))
    table = "\n".join(f"{n:40s} hip {a:.4f} miopen {b:.4f}" for n, a, b in rows)
    for name, a, b in rows:
        assert a <= 1.5 * b + 2e-3, f"{name}: HIP bf16 error {a:.4f} vs MIOpen bf16 {b:.4f}\n{table}"
    print(table)


def test_network_routes_bf16_convs_to_hip(cuda, lib, monkeypatch):
    """Under bf16 autocast the six 64/128-channel 3x3 layers of the conv stack
    run on Conv3x3Function (no silent MIOpen fallback); the 4->64 input layer
    and f32 runs stay on torch's convolution."""
    import runtime.kernels as K
    from models.network import BlockBlastNetwork

    calls = []
    orig = K.Conv3x3Function.apply

    def counting(x, w, *rest):
        calls.append((x.shape[1], w.shape[0]))
        return orig(x, w, *rest)

    monkeypatch.setattr(K.Conv3x3Function, "apply", counting)
    net = BlockBlastNetwork().to(cuda).train().to(memory_format=torch.channels_last)
    x = (torch.rand((64, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        lo, va = net.raw(x)
    (lo.float().sum() + va.float().sum()).backward()
    assert sorted(calls) == sorted([(64, 128)] + [(128, 128)] * 5), calls
    calls.clear()
    net.raw(x)  # f32: torch's convolutions
    assert calls == []


@pytest.mark.parametrize("autocast", [False, True])
def test_nhwc_flatten_matches_reference_flatten(cuda, lib, autocast):
    """The channels_last trunk flattens in (h, w, c) order against the first FC
    weight permuted the same way (models/network.py NHWC_FLATTEN): same
    features and the same parameter gradients as the reference's (c, h, w)
    flatten (network.py:163), f32 and bf16."""
    import models.network as NW
    from models.network import BlockBlastNetwork

    torch.manual_seed(9)
    net = BlockBlastNetwork().to(cuda).train().to(memory_format=torch.channels_last)
    for m in net.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    x = (torch.rand((256, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    outs = []
    for flat in (True, False):
        NW.NHWC_FLATTEN = flat
        net.zero_grad(set_to_none=True)
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False, enabled=autocast):
                f = net.trunk(x)
        finally:
            NW.NHWC_FLATTEN = True
        f.float().square().sum().backward()
        outs.append((f.detach().float(), {k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None}))
    (fa, ga), (fb, gb) = outs
    # f32: MIOpen's weight-gradient algorithms accumulate in varying order (split-K with atomics),
    # so the first layers' gradients move by ~1e-3 between any two runs (see test_gpu_ppo_kernels)
    tol = 2e-2 if autocast else 5e-3
    assert float((fa - fb).norm() / fb.norm()) < tol
    params = dict(net.named_parameters())
    for k in gb:
        if k.endswith(".bias") and params[k[:-5] + ".weight"].dim() == 4:
            continue  # conv biases feed a BatchNorm: true gradient 0, both sides rounding noise
        assert float((ga[k] - gb[k]).norm() / gb[k].norm()) < tol, k


@pytest.mark.parametrize("cin,cout", SHAPES)
@pytest.mark.parametrize("n", [1, 3, 257, 2048])
def test_conv3x3_forward_stats(cuda, lib, cin, cout, n):
    """bb_conv3x3_forward_stats: the same y as bb_conv3x3_forward, and per channel the fp64 sums of
    u = y + pre_bias and u^2 over every pixel (BatchNorm's forward statistics) equal to a float64
    reduction of the stored values; bit-identical on a second call."""
    from runtime.kernels import _p, _s

    x, w, _ = _inputs(cuda, n, cin, cout, 300 + n + cin + cout, layout=0)
    wf = torch.empty(9 * cout * cin, dtype=torch.bfloat16, device=cuda)
    wd = torch.empty_like(wf)
    assert lib.bb_conv3x3_prep(_p(w), cin, cout, 0, _p(wf), _p(wd), _s(cuda)) == 0
    pb = torch.randn(cout, device=cuda)
    y0 = torch.empty((n, cout, 8, 8), dtype=torch.bfloat16, device=cuda, memory_format=torch.channels_last)
    assert lib.bb_conv3x3_forward(_p(x), _p(wf), n, cin, cout, _p(y0), _s(cuda)) == 0
    nparts = lib.bb_conv3x3_stats_parts(n, cout)
    assert nparts >= 1
    outs = []
    for _ in range(2):
        y = torch.empty_like(y0)
        part = torch.full((nparts, cout, 3), float("nan"), dtype=torch.float64, device=cuda)
        assert lib.bb_conv3x3_forward_stats(_p(x), _p(wf), n, cin, cout, _p(y), _p(pb), _p(part), _s(cuda)) == 0
        outs.append((y, part))
    torch.cuda.synchronize()
    (y, part), (y2, part2) = outs
    assert torch.equal(y, y0) and torch.equal(y2, y0)
    assert torch.equal(part, part2)
    u = (y.float() + pb.view(1, -1, 1, 1)).double()
    s_ref = u.sum(dim=(0, 2, 3))
    q_ref = (u * u).sum(dim=(0, 2, 3))
    s = part[:, :, 0].sum(0)
    q = part[:, :, 1].sum(0)
    assert torch.allclose(s, s_ref, rtol=1e-12, atol=1e-9 * float(s_ref.abs().max()))
    assert torch.allclose(q, q_ref, rtol=1e-12, atol=0)
    assert bool((part[:, :, 2] == 0).all())


@pytest.mark.parametrize("relu,res", [(True, False), (False, True)])
def test_bn_forward_from_conv_stats(cuda, lib, relu, res):
    """bb_bn_forward_parts (statistics from the convolution's epilogue) against bb_bn_forward[_res]
    (its own reduction pass) on the same convolution output: mean / inverse std / running statistics
    within f32 rounding, the output within one bf16 step, num_batches_tracked incremented."""
    from runtime.kernels import BatchNormAddReLUFunction, BatchNormReLUFunction, Conv3x3Function

    n, c = 2048, 128
    x, w, _ = _inputs(cuda, n, 64, c, 7, layout=0)
    pb = torch.randn(c, device=cuda) * 0.1
    parts = torch.empty((lib.bb_conv3x3_stats_parts(n, c), c, 3), dtype=torch.float64, device=cuda)
    z = Conv3x3Function.apply(x, w, None, None, (pb, parts))
    r = torch.randn_like(z) if res else None
    outs = []
    for use in (None, parts):
        bn = torch.nn.BatchNorm2d(c).to(cuda)
        with torch.no_grad():  # the same affine parameters for both
            bn.weight.copy_(torch.linspace(0.5, 1.5, c, device=cuda))
            bn.bias.copy_(torch.linspace(-0.2, 0.2, c, device=cuda))
        if res:
            y = BatchNormAddReLUFunction.apply(z, pb, r, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                                               0.1, 1e-5, bn.num_batches_tracked, None, use)
        else:
            y = BatchNormReLUFunction.apply(z, pb, bn.weight, bn.bias, bn.running_mean, bn.running_var, 0.1, 1e-5,
                                            relu, bn.num_batches_tracked, use)
        outs.append((y, bn))
    (y0, bn0), (y1, bn1) = outs
    assert int(bn1.num_batches_tracked) == 1
    assert torch.allclose(bn1.running_mean, bn0.running_mean, rtol=1e-5, atol=1e-7)
    assert torch.allclose(bn1.running_var, bn0.running_var, rtol=1e-5, atol=1e-7)
    if not res:
        _bf16_close(y1.detach(), y0.detach().float(), "BatchNorm output from the conv statistics")
    else:  # relu(round(bn) + res), rounded again: one bf16 step of the BatchNorm value before the add and one
        # of the sum after it
        a, b = y1.detach().float(), y0.detach().float()
        bad = (a - b).abs() > 2.0 ** -7 * (2 * b.abs() + r.float().abs()) + 1e-6
        assert int(bad.sum()) == 0, f"{int(bad.sum())} residual-path elements off by more than one bf16 step"
        assert float((a == b).float().mean()) > 0.97


def test_network_bf16_conv_stats_matches_reduction(cuda, lib, monkeypatch):
    """The whole CNN's bf16 training forward + backward with the BatchNorm statistics from the
    convolution epilogues (BB_CONV_BN_STATS=1) and with the BatchNorm's own reduction passes,
    both against the f32 network: the fused path is as close to f32 as the unfused one (logits, values,
    every parameter gradient, relative L2 <= 1.5x + 2e-3 -- the first convolution's gradient is a
    difference of near-equal terms behind a BatchNorm and MIOpen's weight gradient is not deterministic,
    so a direct comparison of the two bf16 runs is not meaningful there), running statistics within 1e-5."""
    import models.network as NW
    from models.network import BlockBlastNetwork

    torch.manual_seed(6)
    nets = [BlockBlastNetwork().to(cuda).train().to(memory_format=torch.channels_last) for _ in range(3)]
    for m in nets[1:]:
        m.load_state_dict(nets[0].state_dict())
    for net in nets:
        for m in net.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
    x = (torch.rand((1024, 4, 8, 8), device=cuda) < 0.4).float().contiguous(memory_format=torch.channels_last)
    wgt = None
    outs = []
    for net, mode in zip(nets, ("stats", "reduce", "f32")):
        monkeypatch.setattr(NW, "CONV_BN_STATS", mode == "stats")
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False, enabled=mode != "f32"):
            lo, va = net.raw(x)
        lo, va = lo.float(), va.float()
        if wgt is None:
            wgt = torch.randn_like(lo)
        ((lo * wgt).sum() + va.sum()).backward()
        outs.append((lo.detach(), va.detach(), {k: p.grad for k, p in net.named_parameters()},
                     {k: b for k, b in net.named_buffers()}))

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    (l1, v1, g1, b1), (l0, v0, g0, b0), (l32, v32, g32, _) = outs
    rows = [("logits", rel(l1, l32), rel(l0, l32)), ("values", rel(v1, v32), rel(v0, v32))]
    params = dict(nets[2].named_parameters())
    for k in g32:
        if k.endswith(".bias") and params[k].dim() == 1 and params[k[:-5] + ".weight"].dim() == 4:
            continue  # conv biases feed a BatchNorm: true gradient 0
        rows.append((k, rel(g1[k], g32[k]), rel(g0[k], g32[k])))
    table = "\n".join(f"{n:40s} stats {a:.4f} reduce {b:.4f}" for n, a, b in rows)
    for name, a, b in rows:
        assert a <= 1.5 * b + 2e-3, f"{name}: conv-statistics error {a:.4f} vs reduction {b:.4f}\n{table}"
    for k in b0:
        if b0[k].dtype.is_floating_point:
            assert torch.allclose(b1[k], b0[k], rtol=1e-5, atol=1e-6), k
        else:
            assert torch.equal(b1[k], b0[k]), k
