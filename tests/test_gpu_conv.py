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


@pytest.mark.parametrize("n,x_nhwc,w_layout", [(1, 0, 0), (3, 1, 1), (7, 0, 1), (1000, 1, 0), (2048, 0, 0),
                                               (4099, 1, 1)])
def test_conv_in_forward_and_weight_grad(cuda, lib, n, x_nhwc, w_layout):
    """The 4 -> 64 input layer (bb_conv_in_forward / _wgrad) against torch's f32 convolution of the same bf16
    values: the stacked board planes (0/1) and random inputs, both memory formats."""
    from runtime.kernels import ConvInFunction

    g = torch.Generator(device=cuda).manual_seed(7 + n)
    x = torch.randn((n, 4, 8, 8), device=cuda, generator=g)
    x[: n // 2] = (x[: n // 2] > 0.3).float()  # board / piece planes
    if x_nhwc:
        x = x.contiguous(memory_format=torch.channels_last)
    w = torch.randn((64, 4, 3, 3), device=cuda, generator=g) * (2.0 / 36) ** 0.5
    if w_layout:
        w = w.contiguous(memory_format=torch.channels_last)
    dy = torch.randn((n, 64, 8, 8), device=cuda, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    xb, wb = x.bfloat16().double(), w.bfloat16().double()
    wp = w.clone().requires_grad_(True)
    y = ConvInFunction.apply(x, wp)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    _bf16_close(y, F.conv2d(xb, wb, padding=1), "input-layer forward")
    y.backward(dy)
    ref = torch.nn.grad.conv2d_weight(xb, w.shape, dy.double(), padding=1)
    assert wp.grad.dtype == torch.float32 and wp.grad.stride() == w.stride()
    err = float((wp.grad.double() - ref).abs().max())
    assert err <= 1e-5 * float(ref.abs().max()) + 1e-6, err
    # deterministic: a second backward gives the same bits
    wp2 = w.clone().requires_grad_(True)
    ConvInFunction.apply(x, wp2).backward(dy)
    assert torch.equal(wp.grad, wp2.grad)


def test_network_conv_in_equals_miopen(cuda, monkeypatch):
    """bf16 training forward + backward of the CNN with the input layer on bb_conv_in_* and on MIOpen: logits
    and values within bf16 rounding; the first layer's weight gradient against the fp64 weight gradient of the
    same bf16 input and the same output gradient (captured at the BatchNorm's input), each path on its own."""
    import models.network as N
    from runtime import kernels as K

    torch.manual_seed(3)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    x = (torch.rand((512, 4, 8, 8), device=cuda) < 0.4).float()
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    conv0, bn0 = net.conv_encoder[0], net.conv_encoder[1]
    grabbed = {}

    def pre_hook(mod, args):
        z = args[0]
        if z.requires_grad:
            z.register_hook(lambda gz: grabbed.__setitem__("dz", gz.detach().clone()))

    h = bn0.register_forward_pre_hook(pre_hook)
    res = {}
    try:
        for on in (True, False):
            monkeypatch.setattr(K, "CONV_IN", on)
            net.load_state_dict(state0)
            net.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                lo, va = net.raw(x.contiguous(memory_format=torch.channels_last) if not on else x)
            (lo.float().square().mean() + va.float().sum()).backward()
            truth = torch.nn.grad.conv2d_weight(x.double(), conv0.weight.shape, grabbed["dz"].double(), padding=1)
            res[on] = (lo.detach().float(), va.detach().float(),
                       {n: p.grad.clone() for n, p in net.named_parameters()}, truth)
    finally:
        h.remove()
    for a, b in ((res[True][0], res[False][0]), (res[True][1], res[False][1])):
        assert float((a - b).norm() / b.norm()) < 2e-2
    for on in (True, False):
        g0, truth = res[on][2]["conv_encoder.0.weight"].double(), res[on][3]
        rel = float((g0 - truth).norm() / truth.norm())
        print(f"input-layer weight gradient vs fp64 ({'bb_conv_in' if on else 'MIOpen'}): {rel:.2e} rel L2")
        if on:
            assert rel < 1e-4, rel
    # the rest of the network sees the input layer's output rounded to bf16 from two different f32 sums, and
    # every later layer rounds to bf16 again: the BatchNorm parameter gradients (sums with heavy cancellation)
    # move by up to ~20% per tensor (measured), so the check is on the whole gradient and a loose per-tensor
    # bound that a layout or indexing error (>= 100%) would still break
    names = [n for n in res[True][2] if not n.startswith("conv_encoder.0.")]
    a = torch.cat([res[True][2][n].flatten() for n in names])
    b = torch.cat([res[False][2][n].flatten() for n in names])
    cos = float(torch.nn.functional.cosine_similarity(a, b, dim=0))
    rel = float((a - b).norm() / b.norm())
    print(f"network gradient, bb_conv_in vs MIOpen input layer: cosine {cos:.5f}, rel L2 {rel:.2e}")
    assert cos > 0.995 and rel < 0.1, (cos, rel)
    for name in names:
        gr, ref = res[True][2][name], res[False][2][name]
        if name.endswith(".bias") and res[True][2][name[:-5] + ".weight"].dim() == 4:
            continue  # a conv bias before BatchNorm: zero up to noise
        assert float((gr - ref).norm() / ref.norm().clamp_min(1e-30)) < 0.5, name


def test_wgrad_piggyback_equals_plain(cuda, monkeypatch):
    """The board convolutions' weight-gradient reductions carried by the next BatchNorm backward's finalisation
    launch (wgrad_piggyback, bb_bn_backward_red) == the plain two-launch weight gradient, bit for bit: the whole
    bf16 CNN's parameter gradients and the BatchNorm outputs; a pending reduction with no BatchNorm after it is
    flushed when the block closes."""
    import models.network as N
    from runtime import kernels as K

    torch.manual_seed(5)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    x = (torch.rand((256, 4, 8, 8), device=cuda) < 0.4).float()
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    res = {}
    for on in (True, False):
        net.load_state_dict(state0)
        for p in net.parameters():
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            lo, va = net.raw(x)
        with K.wgrad_piggyback(cuda, enabled=on):
            (lo.float().square().mean() + va.float().sum()).backward()
        res[on] = {n: p.grad.clone() for n, p in net.named_parameters()}
    for n, g in res[True].items():
        if n.startswith("conv_encoder.0."):  # the input layer's own reduction is not carried; MIOpen-free either way
            assert torch.equal(g, res[False][n]), n
            continue
        assert torch.equal(g, res[False][n]), n
    # a lone convolution: its pending reduction is flushed at the block's exit
    conv = [m for m in net.conv_encoder.modules() if isinstance(m, torch.nn.Conv2d) and m.in_channels == 128][0]
    xb = torch.randn((64, 128, 8, 8), device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn((64, 128, 8, 8), device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for on in (True, False):
        w = conv.weight.detach().clone().requires_grad_(True)
        with K.wgrad_piggyback(cuda, enabled=on):
            K.Conv3x3Function.apply(xb, w).backward(dy)
        outs.append(w.grad)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("cin,cout", SHAPES)
@pytest.mark.parametrize("n", [1, 3, 257, 2048])
def test_conv3x3_forward_stats(cuda, lib, cin, cout, n):
    """bb_conv3x3_forward_stats: the same output as bb_conv3x3_forward (bit for bit) and, per workgroup and
    channel, the sum and sum of squares of the stored bf16 outputs: their total within f32 summation noise of
    the fp64 sums, the third slot 0."""
    from runtime import kernels as K

    x, w, _ = _inputs(cuda, n, cin, cout, 300 + n + cin + cout, layout=0)
    y0 = K.Conv3x3Function.apply(x, w)
    slot = K.StatsSlot()
    y = K.Conv3x3Function.apply(x, w, None, None, slot)
    assert torch.equal(y, y0)
    assert slot.ptr == y.data_ptr() and slot.nb == lib.bb_conv3x3_stats_blocks(n, cout) == (n + 1) // 2
    part = slot.part.view(slot.nb, cout, 3)
    yd = y.double().permute(0, 2, 3, 1).reshape(-1, cout)
    for m, ref in ((0, yd.sum(0)), (1, yd.square().sum(0))):
        tot = part[:, :, m].sum(0)
        scale = (yd.abs().sum(0) if m == 0 else yd.square().sum(0)).clamp_min(1e-30)
        assert float(((tot - ref).abs() / scale).max()) < 1e-6, m
    assert bool((part[:, :, 2] == 0).all())


@pytest.mark.parametrize("res", [False, True])
def test_bn_forward_from_conv_stats(cuda, lib, res):
    """BatchNorm forward from the convolution's partials (bb_bn_forward_part) == its own reduction
    (bb_bn_forward / _res): saved mean and inverse std within f64-vs-f32 summation noise, outputs within one
    bf16 step (an element may round the other way), running statistics and num_batches_tracked alike."""
    from runtime import kernels as K

    n, c = 2048, 128
    x, w, _ = _inputs(cuda, n, c, c, 77, layout=0)
    slot = K.StatsSlot()
    z = K.Conv3x3Function.apply(x, w, None, None, slot)
    g = torch.Generator(device=cuda).manual_seed(3)
    pre_b, wt, bs = (torch.randn(c, device=cuda, generator=g) * 0.1 for _ in range(3))
    wt = wt + 1.0
    r = torch.randn_like(z.float()).bfloat16().contiguous(memory_format=torch.channels_last)
    outs = []
    for use in (slot, None):
        rm, rv = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
        nbt = torch.zeros((), dtype=torch.int64, device=cuda)
        if res:
            y = K.BatchNormAddReLUFunction.apply(z, pre_b, r, wt, bs, rm, rv, 0.1, 1e-5, nbt, None, use)
        else:
            y = K.BatchNormReLUFunction.apply(z, pre_b, wt, bs, rm, rv, 0.1, 1e-5, True, nbt, use)
        outs.append((y, rm, rv, int(nbt)))
    (y1, rm1, rv1, n1), (y2, rm2, rv2, n2) = outs
    assert n1 == n2 == 1
    assert torch.allclose(rm1, rm2, rtol=1e-5, atol=1e-6) and torch.allclose(rv1, rv2, rtol=1e-5, atol=1e-6)
    step = (y2.float().abs() * 2.0 ** -7).clamp_min(2.0 ** -126)
    assert bool(((y1.float() - y2.float()).abs() <= step).all())
    assert float((y1 == y2).float().mean()) > 0.999


@pytest.mark.parametrize("bstats", [False, True])
def test_network_conv_stats_equals_own_reduction(cuda, monkeypatch, bstats):
    """bf16 raw() forward + backward with the BatchNorm statistics (and, bstats, bn1's backward sums) from the
    convolutions' store passes == with the BatchNorms' own reduction passes: outputs within bf16 rounding,
    parameter gradients within 1%."""
    import models.network as N
    from runtime import kernels as K

    monkeypatch.setattr(K, "CONV_BSTATS", bstats)

    torch.manual_seed(11)
    net = N.BlockBlastNetwork().to(cuda).to(memory_format=torch.channels_last)
    for mod in net.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    net.train()
    x = (torch.rand((512, 4, 8, 8), device=cuda) < 0.4).float()
    state0 = {k: v.clone() for k, v in net.state_dict().items()}
    res = {}
    for on in (True, False):
        monkeypatch.setattr(K, "CONV_STATS", on)
        net.load_state_dict(state0)
        net.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            lo, va = net.raw(x)
        (lo.float().square().mean() + va.float().sum()).backward()
        res[on] = (lo.detach().float(), va.detach().float(), {k: p.grad.clone() for k, p in net.named_parameters()},
                   {k: b.clone() for k, b in net.named_buffers()})
    assert torch.allclose(res[True][0], res[False][0], rtol=2.0 ** -6, atol=2e-3)
    assert torch.allclose(res[True][1], res[False][1], rtol=2.0 ** -6, atol=2e-3)
    for k, gr in res[True][2].items():
        if k.endswith(".bias") and gr.dim() == 1 and res[True][2][k[:-5] + ".weight"].dim() == 4:
            continue  # a conv bias before BatchNorm: zero up to noise
        ref = res[False][2][k]
        assert float((gr - ref).norm() / ref.norm().clamp_min(1e-30)) < 1e-2, k
    for k, b in res[True][3].items():
        assert torch.allclose(b.float(), res[False][3][k].float(), rtol=1e-4, atol=1e-6), k


@pytest.mark.parametrize("c,n,relu", [(128, 2048, 1), (64, 257, 1), (128, 3, 0)])
def test_conv3x3_forward_bstats(cuda, lib, c, n, relu):
    """bb_conv3x3_forward_bstats: the data gradient bit-identical to bb_conv3x3_forward, and per workgroup and
    channel the BatchNorm backward sums {sum g, sum g xhat, sum xhat} of the stored bf16 gradient, g masked
    where the forward's ReLU was off (the same f32 operations), within f32 summation noise of fp64."""
    from runtime import kernels as K

    x, w, dy = _inputs(cuda, n, c, c, 500 + n + c, layout=0)
    g0 = torch.Generator(device=cuda).manual_seed(n)
    bx = torch.randn((n, c, 8, 8), device=cuda, generator=g0).bfloat16().contiguous(memory_format=torch.channels_last)
    mean = torch.randn(c, device=cuda, generator=g0) * 0.1
    invstd = torch.rand(c, device=cuda, generator=g0) + 0.5
    bw = torch.randn(c, device=cuda, generator=g0) * 0.2 + 1.0
    bb = torch.randn(c, device=cuda, generator=g0) * 0.1
    wf = torch.empty(9 * c * c, dtype=torch.bfloat16, device=cuda)
    wd = torch.empty_like(wf)
    L_ = K.L
    L_.check(lib.bb_conv3x3_prep(K._p(w), c, c, 0, K._p(wf), K._p(wd), K._s(cuda)), "prep")
    y0 = torch.empty_like(x)
    y = torch.empty_like(x)
    L_.check(lib.bb_conv3x3_forward(K._p(dy), K._p(wd), n, c, c, K._p(y0), K._s(cuda)), "fwd")
    nbp = lib.bb_conv3x3_stats_blocks(n, c)
    part = torch.empty(nbp * c * 3, dtype=torch.float64, device=cuda)
    L_.check(lib.bb_conv3x3_forward_bstats(K._p(dy), K._p(wd), n, c, c, K._p(y), K._p(bx), K._p(mean), K._p(invstd),
                                           K._p(bw), K._p(bb), relu, K._p(part), K._s(cuda)), "bstats")
    assert torch.equal(y, y0)
    u = bx.float().permute(0, 2, 3, 1).reshape(-1, c)
    gy = y.float().permute(0, 2, 3, 1).reshape(-1, c)
    sc = invstd * bw
    off = ((u - mean) * sc + bb) <= 0 if relu else torch.zeros_like(u, dtype=torch.bool)
    g = torch.where(off, torch.zeros_like(gy), gy).double()
    xh = ((u - mean) * invstd).double()
    tot = part.view(nbp, c, 3).sum(0)
    for m, ref, scale in ((0, g.sum(0), g.abs().sum(0)), (1, (g * xh).sum(0), (g * xh).abs().sum(0)),
                          (2, xh.sum(0), xh.abs().sum(0))):
        assert float(((tot[:, m] - ref).abs() / scale.clamp_min(1e-30)).max()) < 1e-5, m
