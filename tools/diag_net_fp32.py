"""Diagnostics (not product): where the fp32 network forward on the GPU departs
from the float64 truth -- per module, the GPU's and the CPU fp32's max
|d| / max(1, |x|) against the same network in float64 on the CPU, on the inputs
of tests/test_gpu_network_oracle.py (train mode, dropout 0)."""
import copy
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "block-blast-ai---reinforcement-learning-agent_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import bb_ppo as OP  # noqa: E402
from oracle import c_oracle as CO  # noqa: E402


def main():
    if os.environ.get("BB_DIAG_NO_TF32") == "1":
        torch.backends.cudnn.allow_tf32 = False
        torch.backends.cuda.matmul.allow_tf32 = False
    print("cudnn.allow_tf32", torch.backends.cudnn.allow_tf32, "matmul.allow_tf32",
          torch.backends.cuda.matmul.allow_tf32, "fp32 precision", torch.get_float32_matmul_precision())
    B = 2048
    env = CO.CVecEnv(np.arange(42, 42 + B, dtype=np.uint64))
    env.reset()
    mask = env.state()["mask"]
    for t in range(24):
        mask = env.step(env.random_actions(mask, 0xB10C, t))["mask"]
    st = env.state()
    env.close()
    boards, pieces, _ = OP.expand_packed(st["board"], st["hand"], st["mask"])
    from agents import PPOAgent, PPOConfig

    torch.manual_seed(0)
    ref = OP.ReferenceNetwork(dropout=0.0)
    net64 = copy.deepcopy(ref).double()
    agent = PPOAgent(PPOConfig(batch_size=B), device=torch.device("cuda", 0), sample_seed=1)
    agent.network.load_state_dict(ref.state_dict())
    for m in agent.network.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    if os.environ.get("BB_DIAG_NCHW") == "1":
        agent.set_channels_last(False)
    agent.train()
    ref.train()
    net64.train()
    outs = {}

    def hook(tag):
        def f(mod, inp, out):
            outs.setdefault(tag, {})[id(mod)] = out[0] if isinstance(out, tuple) else out
        return f

    names = {}
    for tag, net in (("gpu", agent.network), ("cpu", ref), ("f64", net64)):
        for name, m in net.named_modules():
            if name and name.count(".") <= 2 and not isinstance(m, torch.nn.Sequential):
                m.register_forward_hook(hook(tag))
                names.setdefault(tag, []).append((name, id(m)))
    with torch.no_grad():
        agent._raw(agent._obs_to_device({"board": boards, "pieces": pieces}))
        ref(torch.from_numpy(boards), torch.from_numpy(pieces))
        net64(torch.from_numpy(boards).double(), torch.from_numpy(pieces).double())
    g = dict(names["gpu"])
    c = dict(names["cpu"])
    for name, i64 in names["f64"]:
        if name not in g or name not in c or g[name] not in outs["gpu"]:
            continue
        t = outs["f64"][i64].double()
        xg = outs["gpu"][g[name]].double().cpu().contiguous()
        xc = outs["cpu"][c[name]].double()
        if xg.shape != t.shape:
            continue
        sc = t.abs().clamp(min=1.0)
        print(f"{name:28s} gpu {float(((xg - t).abs() / sc).max()):.2e}  cpu {float(((xc - t).abs() / sc).max()):.2e}"
              f"  |x|max {float(t.abs().max()):.2f}")


if __name__ == "__main__":
    main()
