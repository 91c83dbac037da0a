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
