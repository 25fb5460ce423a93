"""Time one PPO mini-batch forward+backward (actor+critic MLPs, 24576 rows): nn.Linear vs SplitKLinear."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
from rsl_rl.modules import splitk_linear as skl  # noqa: E402
from rsl_rl.modules import mfma_mlp  # noqa: E402


def net(lin):
    L = [lin(48, 512), nn.ELU(), lin(512, 256), nn.ELU(), lin(256, 128), nn.ELU(), lin(128, 12)]
    return nn.Sequential(*L).cuda()


x = torch.randn(24576, 48, device="cuda")
for name, lin in (("nn.Linear", nn.Linear), ("SplitKLinear", skl.SplitKLinear)):
    for chunk in ((1024,) if name == "nn.Linear" else (512, 1024, 2048, 4096)):
        skl.CHUNK = chunk
        a, c = net(lin), net(lin)
        for _ in range(3):
            (a(x).square().mean() + c(x).square().mean()).backward()
        torch.cuda.synchronize()
        t0 = time.time()
        for _ in range(20):
            (a(x).square().mean() + c(x).square().mean()).backward()
        torch.cuda.synchronize()
        print(f"{name:14s} chunk {chunk:5d}: {(time.time() - t0) / 20 * 1e3:.3f} ms per actor+critic fwd+bwd", flush=True)

skl.CHUNK = 4096
a, c = net(skl.SplitKLinear), net(skl.SplitKLinear)
for mode in ("mfma",):
    f = lambda n: mfma_mlp.mlp_apply(n, x)  # noqa: E731
    for _ in range(3):
        (f(a).square().mean() + f(c).square().mean()).backward()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(20):
        (f(a).square().mean() + f(c).square().mean()).backward()
    torch.cuda.synchronize()
    print(f"{'mfma bf16':14s}           : {(time.time() - t0) / 20 * 1e3:.3f} ms per actor+critic fwd+bwd", flush=True)
    with torch.inference_mode():
        xi = torch.randn(4096, 48, device="cuda")
        for _ in range(3):
            mfma_mlp.mlp_apply(a, xi); mfma_mlp.mlp_apply(c, xi)
        torch.cuda.synchronize(); t0 = time.time()
        for _ in range(50):
            mfma_mlp.mlp_apply(a, xi); mfma_mlp.mlp_apply(c, xi)
        torch.cuda.synchronize()
        t1 = (time.time() - t0) / 50 * 1e3
        for _ in range(3):
            a(xi); c(xi)
        torch.cuda.synchronize(); t0 = time.time()
        for _ in range(50):
            a(xi); c(xi)
        torch.cuda.synchronize()
        print(f"rollout inference 4096 rows actor+critic: mfma {t1:.3f} ms, torch fp32 {(time.time() - t0) / 50 * 1e3:.3f} ms", flush=True)

# ---- graph-captured fwd+bwd (how PPO runs it): GPU time without Python dispatch
for name, fn in (("splitK fp32", lambda n: n(x)), ("mfma bf16", lambda n: mfma_mlp.mlp_apply(n, x))):
    a, c = net(skl.SplitKLinear), net(skl.SplitKLinear)
    for p in list(a.parameters()) + list(c.parameters()):
        p.grad = torch.zeros_like(p)

    def body():
        for p in list(a.parameters()) + list(c.parameters()):
            p.grad.zero_()
        (fn(a).square().mean() + fn(c).square().mean()).backward()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            body()
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(50):
        g.replay()
    torch.cuda.synchronize()
    print(f"graphed {name:12s}: {(time.time() - t0) / 50 * 1e3:.3f} ms per actor+critic fwd+bwd", flush=True)
