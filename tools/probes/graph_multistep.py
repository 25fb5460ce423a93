"""Probe: K optimizer steps inside ONE captured graph vs the same K steps eager.
Variants: autocast bf16 on/off x Adam fused/foreach."""
import copy
import sys
import torch
import torch.nn as nn

dev = "cuda"
K = int(sys.argv[1]) if len(sys.argv) > 1 else 2


def mlp():
    return nn.Sequential(nn.Linear(48, 512), nn.ELU(), nn.Linear(512, 256), nn.ELU(), nn.Linear(256, 128), nn.ELU(),
                         nn.Linear(128, 12)).to(dev)


def trial(mp, impl):
    torch.manual_seed(0)
    net = mlp()
    twin = copy.deepcopy(net)
    kw = dict(fused=True) if impl == "fused" else dict(foreach=True)
    opt = torch.optim.Adam(net.parameters(), lr=torch.tensor(1e-3, device=dev), capturable=True, **kw)
    opt2 = torch.optim.Adam(twin.parameters(), lr=torch.tensor(1e-3, device=dev), capturable=True, **kw)
    x = torch.randn(4096, 48, device=dev)
    t = torch.randn(4096, 12, device=dev)

    def step(n, o):
        if mp:
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                y = n(x)
            y = y.float()
        else:
            y = n(x)
        loss = ((y - t) ** 2).mean()
        o.zero_grad(set_to_none=False)
        loss.backward()
        o.step()

    def body(n, o):
        for _ in range(K):
            step(n, o)

    step(net, opt)
    step(twin, opt2)
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
    out = []
    for k in range(3):
        g.replay()
        body(twin, opt2)
        torch.cuda.synchronize()
        out.append(max(float((a - b).abs().max()) for a, b in zip(net.parameters(), twin.parameters())))
    print(f"K={K} mp={mp} adam={impl}: max |param graph - eager| per replay {['%.2e' % d for d in out]}", flush=True)


for mp in (True, False):
    for impl in ("fused", "foreach"):
        trial(mp, impl)
