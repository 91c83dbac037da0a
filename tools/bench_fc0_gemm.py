"""Diagnostics: the first FC layer's bf16 GEMMs (2,048 x 8,192 -> 512) under the operand layouts hipBLASLt can be
handed -- weight [512][8192] (the parameter's) or its transpose [8192][512] -- timed with HIP events."""
import torch

dev = torch.device("cuda", 0)
torch.manual_seed(0)
M, K, N = 2048, 8192, 512
x = torch.randn(M, K, device=dev).bfloat16()
w = (torch.randn(N, K, device=dev) * 0.01).bfloat16()
wt = w.t().contiguous()
b = torch.randn(N, device=dev).bfloat16()
g = torch.randn(M, N, device=dev).bfloat16()


def t(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


cases = {
    "fwd addmm_act(b, x, w.t())  [w NK]": lambda: torch._addmm_activation(b, x, w.t()),
    "fwd addmm_act(b, x, wt)     [w KN]": lambda: torch._addmm_activation(b, x, wt),
    "fwd mm(w, x.t()) -> yT": lambda: torch.mm(w, x.t()),
    "dgrad g.mm(w)               [w NK]": lambda: g.mm(w),
    "dgrad g.mm(wt.t())          [w KN]": lambda: g.mm(wt.t()),
    "wgrad g.t().mm(x)  -> dW NK": lambda: g.t().mm(x),
    "wgrad x.t().mm(g)  -> dW KN": lambda: x.t().mm(g),
}
y0 = torch._addmm_activation(b, x, w.t())
y1 = torch._addmm_activation(b, x, wt)
print("fwd equal:", bool(torch.equal(y0, y1)))
for k, fn in cases.items():
    print(f"{k:40s} {t(fn):7.1f} us")
