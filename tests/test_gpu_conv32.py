"""The fp32 board convolutions (csrc/bb_conv32.hip, runtime.kernels.Conv3x3F32Function) against float64.

Forward and data gradient: every output within the rigorous error bound of the kernel's summation against
the float64 convolution of the same f32 values: |y - y64| <= 2^-24 |y64| + gamma_16 sum|x w| (the final
rounding, plus gamma_16 = 16 * 2^-24 for one 16-product fp32 chain per block; the fp64 adds of the blocks
are ~1e-14), where one 1,152-product chain (MIOpen's kind of order) is only bounded by gamma_1152, 72x
looser.  The measured typical error (RMS of |y - y64| / sum|x w|) is printed beside MIOpen's on the same
inputs and must not exceed it.  At 1, 3, 257 and 2,048 boards for each supported (cin, cout) and both
weight layouts; zeros outside the board (one-hot inputs at every edge and tap, exact); bit-identical on a
second call.  The weight gradient (aten's) within 1e-5 relative L2 of float64.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

PAIRS = [(128, 128), (64, 128), (128, 64)]


def _data(n, cin, cout, dev, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, cin, 8, 8, generator=g).relu() * 1.3  # post-ReLU activations, like the network's
    w = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cin)) ** 0.5
    return x.to(dev).contiguous(memory_format=torch.channels_last), w.to(dev)


def _run(x, w, wl):
    from runtime import kernels as K
    from runtime import lib as L

    n, cin, cout = x.shape[0], x.shape[1], w.shape[0]
    w = w.contiguous(memory_format=torch.channels_last) if wl else w.contiguous()
    wf = torch.empty(9 * cin * cout, device=x.device)
    wd = torch.empty(9 * cin * cout, device=x.device)
    lib = L.load()
    L.check(lib.bb_conv3x3_f32_prep(K._p(w), cin, cout, wl, K._p(wf), K._p(wd), K._s(x.device)), "prep")
    y = torch.empty((n, cout, 8, 8), device=x.device, memory_format=torch.channels_last)
    L.check(lib.bb_conv3x3_f32_forward(K._p(x), K._p(wf), n, cin, cout, K._p(y), K._s(x.device)), "forward")
    return y, wd


def _bound(y, y64, absum):
    err = (y.double() - y64).abs()
    lim = 2.0 ** -24 * y64.abs() + 16 * 2.0 ** -24 * absum
    return err, lim


def _rms_rel(y, y64, absum):
    return float((((y.double() - y64).abs() / absum.clamp_min(1e-30)) ** 2).mean().sqrt())


@pytest.mark.parametrize("cin,cout", PAIRS)
@pytest.mark.parametrize("n", [1, 3, 257, 2048])
@pytest.mark.parametrize("wl", [0, 1])
def test_conv32_forward_within_error_bound_of_float64(cuda, cin, cout, n, wl):
    if n == 257 and wl == 1:
        pytest.skip("layouts are covered at the other sizes")
    x, w = _data(n, cin, cout, cuda, n * 7 + cin + cout + wl)
    y, _ = _run(x, w, wl)
    y64 = F.conv2d(x.double(), w.double(), padding=1)
    absum = F.conv2d(x.double().abs(), w.double().abs(), padding=1)
    err, lim = _bound(y, y64, absum)
    ym = F.conv2d(x, w, padding=1)  # MIOpen fp32 on the same inputs
    ours, miopen = _rms_rel(y, y64, absum), _rms_rel(ym, y64, absum)
    print(f"{n}x{cin}->{cout} wl{wl}: max err / bound {float((err / lim).max()):.3f}; RMS |err|/sum|xw| "
          f"ours {ours:.2e}, MIOpen {miopen:.2e}; max |err| ours {float(err.max()):.2e}, "
          f"MIOpen {float((ym.double() - y64).abs().max()):.2e}")
    assert bool((err <= lim).all()), float((err / lim).max())
    if n >= 257:
        assert ours <= miopen, (ours, miopen)
    y2, _ = _run(x, w, wl)
    assert torch.equal(y, y2)  # deterministic


@pytest.mark.parametrize("cin,cout", [(128, 128), (64, 128)])
def test_conv32_data_gradient_within_error_bound(cuda, cin, cout):
    from runtime import kernels as K
    from runtime import lib as L

    n = 300
    x, w = _data(n, cin, cout, cuda, 99 + cin)
    dy = torch.randn(n, cout, 8, 8, device=cuda).contiguous(memory_format=torch.channels_last)
    _, wd = _run(x, w, 0)
    dx = torch.empty_like(x)
    L.check(L.load().bb_conv3x3_f32_forward(K._p(dy), K._p(wd), n, cout, cin, K._p(dx), K._s(cuda)), "dgrad")
    x64 = x.double().requires_grad_(True)
    F.conv2d(x64, w.double(), padding=1).backward(dy.double())
    absum = torch.nn.grad.conv2d_input(x.shape, w.double().abs(), dy.double().abs(), padding=1)
    err, lim = _bound(dx, x64.grad, absum)
    assert bool((err <= lim).all()), float((err / lim).max())


def test_conv32_one_hot_edges_exact(cuda):
    """One-hot inputs and weights at every board position and tap: each output is a single product (exact),
    so y must equal the float64 convolution bit for bit -- taps leaving the board read zeros."""
    cin = cout = 128
    n = 64
    x = torch.zeros(n, cin, 8, 8, device=cuda)
    for b in range(n):
        x[b, b % cin, b // 8, b % 8] = 1.0 + b
    x = x.contiguous(memory_format=torch.channels_last)
    w = torch.zeros(cout, cin, 3, 3, device=cuda)
    for t in range(9):
        for c in range(cin):
            w[(c + t) % cout, c, t // 3, t % 3] = 0.5 + t
    y, _ = _run(x, w, 0)
    y64 = F.conv2d(x.double(), w.double(), padding=1)
    assert torch.equal(y.double(), y64)


def test_conv32_function_autograd(cuda):
    """Conv3x3F32Function: forward as above, backward = (data gradient on the kernel, aten weight gradient)
    against float64 autograd."""
    from runtime.kernels import Conv3x3F32Function

    n, cin, cout = 200, 64, 128
    x, w = _data(n, cin, cout, cuda, 5)
    xg = x.clone().requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    y = Conv3x3F32Function.apply(xg, wg)
    dy = torch.randn_like(y)
    y.backward(dy)
    x64 = x.double().requires_grad_(True)
    w64 = w.double().requires_grad_(True)
    y64 = F.conv2d(x64, w64, padding=1)
    y64.backward(dy.double())
    assert float((y.double() - y64).abs().max()) <= 1e-5 * float(y64.abs().max())
    for got, want in ((xg.grad, x64.grad), (wg.grad, w64.grad)):
        rel = float((got.double() - want).norm() / want.norm())
        assert rel < 1e-5, rel


# the last two take the 128-row tile (>= 1,024 workgroups), ragged in M
@pytest.mark.parametrize("m,n,k", [(1, 128, 32), (77, 512, 8192), (2048, 512, 8192), (300, 256, 512), (64, 128, 256),
                                   (32700, 512, 512), (16385, 1024, 256)])
def test_linear_f32_within_error_bound(cuda, m, n, k):
    """bb_linear_f32 (nn.Linear forward) against float64: |y - y64| <= 2^-24 |y64| + gamma_16 sum|x w| (+ the
    bias, added in fp64 before the one rounding); ragged M; its RMS error not above hipBLASLt's fp32 at K >= 512."""
    from runtime.kernels import linear_f32

    g = torch.Generator().manual_seed(m + n + k)
    x = (torch.randn(m, k, generator=g).relu() * 1.7).to(cuda)
    w = (torch.randn(n, k, generator=g) * (2.0 / k) ** 0.5).to(cuda)
    b = (torch.randn(n, generator=g) * 0.1).to(cuda)
    y = linear_f32(x, w, b)
    y64 = x.double() @ w.double().t() + b.double()
    absum = x.double().abs() @ w.double().abs().t()
    err = (y.double() - y64).abs()
    lim = 2.0 ** -24 * y64.abs() + 16 * 2.0 ** -24 * absum
    assert bool((err <= lim).all()), float((err / lim).max())
    yb = torch.nn.functional.linear(x, w, b)
    ours, blas = _rms_rel(y, y64, absum), _rms_rel(yb, y64, absum)
    print(f"linear {m}x{k}->{n}: max err / bound {float((err / lim).max()):.3f}; RMS ours {ours:.2e}, hipBLASLt {blas:.2e}")
    if k >= 512 and m >= 64:
        assert ours <= blas, (ours, blas)
    assert torch.equal(y, linear_f32(x, w, b))
