"""Probe: bf16-autocast MLP forward (+backward +Adam) captured in a HIP graph vs eager.
Finds whether replays see live weights (forward) and produce eager-equal updates."""
import copy
import torch
import torch.nn as nn

torch.manual_seed(0)
dev = "cuda"


def mlp():
    return nn.Sequential(nn.Linear(48, 512), nn.ELU(), nn.Linear(512, 256), nn.ELU(), nn.Linear(256, 128), nn.ELU(),
                         nn.Linear(128, 12)).to(dev)


def run(net, x):
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        y = net(x)
    return y.float()


# ---- 1. forward only: replay after changing weights
net = mlp()
x = torch.randn(4096, 48, device=dev)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    run(net, x)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        y_static = run(net, x)
torch.cuda.current_stream().wait_stream(side)
for k in range(3):
    with torch.no_grad():
        for p in net.parameters():
            p.add_(0.05 * torch.randn_like(p))
        x.copy_(torch.randn_like(x))
    g.replay()
    torch.cuda.synchronize()
    ref = run(net, x)
    print(f"forward replay {k}: max |graph - eager| = {float((y_static - ref).abs().max()):.3e} "
          f"(|y| {float(ref.abs().max()):.2f})", flush=True)

# ---- 2. forward+backward+Adam step
for mp in (True, False):
    net = mlp()
    twin = copy.deepcopy(net)
    opt = torch.optim.Adam(net.parameters(), lr=torch.tensor(1e-3, device=dev), fused=True, capturable=True)
    opt2 = torch.optim.Adam(twin.parameters(), lr=torch.tensor(1e-3, device=dev), fused=True, capturable=True)
    x = torch.randn(4096, 48, device=dev)
    t = torch.randn(4096, 12, device=dev)

    def body(n, o):
        y = run(n, x) if mp else n(x)
        loss = ((y - t) ** 2).mean()
        o.zero_grad(set_to_none=False)
        loss.backward()
        o.step()
        return loss

    body(net, opt)  # eager first step creates state/grads
    body(twin, opt2)
    snap = [p.detach().clone() for p in net.parameters()]
    snap_o = [{k: v.clone() for k, v in opt.state[p].items()} for p in net.parameters()]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body(net, opt)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            body(net, opt)
    torch.cuda.current_stream().wait_stream(side)
    with torch.no_grad():
        for p, v, o in zip(net.parameters(), snap, snap_o):
            p.copy_(v)
            for k2, v2 in o.items():
                opt.state[p][k2].copy_(v2)
    for k in range(4):
        with torch.no_grad():
            x.copy_(torch.randn_like(x))
            t.copy_(torch.randn_like(t))
        g.replay()
        body(twin, opt2)
        torch.cuda.synchronize()
        d = max(float((a - b).abs().max()) for a, b in zip(net.parameters(), twin.parameters()))
        print(f"mp={mp} train replay {k}: max |param graph - eager| = {d:.3e}", flush=True)
