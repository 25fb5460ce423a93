"""Probe: PPO-shaped update (K steps in one graph) vs eager, features switchable.
flags: perm (index_select mini-batches), dist (actor+critic+Normal log-prob), clip (grad-norm clipping)."""
import copy
import os
import itertools
import torch
import torch.nn as nn
from torch.distributions import Normal

dev = "cuda"
replay_stream = torch.cuda.Stream()


def mlp(o):
    return nn.Sequential(nn.Linear(48, 512), nn.ELU(), nn.Linear(512, 256), nn.ELU(), nn.Linear(256, 128), nn.ELU(),
                         nn.Linear(128, o)).to(dev)


class AC(nn.Module):
    def __init__(self):
        super().__init__()
        self.actor, self.critic = mlp(12), mlp(1)
        self.std = nn.Parameter(torch.ones(12, device=dev))


def run(net, x):
    with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
        y = net(x)
    return y.float()


def trial(perm_on, dist_on, clip_on, rows, K=8, mb=4):
    torch.manual_seed(0)
    ac = AC()
    twin = copy.deepcopy(ac)
    mk = lambda m: torch.optim.Adam(m.parameters(), lr=torch.tensor(1e-3, device=dev), capturable=True, fused=True)  # noqa
    opt, opt2 = mk(ac), mk(twin)
    N = rows * mb
    obs = torch.randn(N, 48, device=dev)
    act = torch.randn(N, 12, device=dev)
    adv = torch.randn(N, device=dev)
    ret = torch.randn(N, 1, device=dev)
    oldlp = torch.randn(N, device=dev) - 15.0
    perm = torch.randperm(N, device=dev)
    accs = {}

    def step(m, o, i, acc):
        if perm_on:
            idx = perm[i * rows:(i + 1) * rows]
            ob, ab, av, rb, lb = (t.index_select(0, idx) for t in (obs, act, adv, ret, oldlp))
        else:
            s = slice(i * rows, (i + 1) * rows)
            ob, ab, av, rb, lb = obs[s], act[s], adv[s], ret[s], oldlp[s]
        if dist_on:
            mean = run(m.actor, ob)
            d = Normal(mean, mean * 0.0 + m.std, validate_args=False)
            if os.environ.get("KEEP"):
                m.distribution = d  # survives the step (and the capture), as ActorCritic does
            lp = d.log_prob(ab).sum(dim=-1)
            ratio = torch.exp(lp - lb)
            surr = torch.max(-av * ratio, -av * torch.clamp(ratio, 0.8, 1.2)).mean()
            v = run(m.critic, ob)
            loss = surr + (rb - v).pow(2).mean()
        else:
            y = run(m.actor, ob)
            loss = (y - ab).pow(2).mean()
        o.zero_grad(set_to_none=False)
        loss.backward()
        if clip_on:
            nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        o.step()
        with torch.no_grad():
            acc += loss.detach()

    def body(m, o, acc):
        acc.zero_()
        for k in range(K):
            step(m, o, k % mb, acc)

    a1, a2 = torch.zeros((), device=dev), torch.zeros((), device=dev)
    step(ac, opt, 0, a1)
    step(twin, opt2, 0, a2)
    snap = [p.detach().clone() for p in ac.parameters()]
    snap_o = [{k: v.clone() for k, v in opt.state[p].items()} for p in ac.parameters()]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        body(ac, opt, a1)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            body(ac, opt, a1)
    torch.cuda.current_stream().wait_stream(side)
    with torch.no_grad():
        for p, v, o in zip(ac.parameters(), snap, snap_o):
            p.copy_(v)
            for k2, v2 in o.items():
                opt.state[p][k2].copy_(v2)
    R = int(os.environ.get("REPS", 2))
    gen = torch.Generator(device=dev).manual_seed(5)
    bad_at = None
    for r in range(R):
        if os.environ.get("NEWDATA"):
            with torch.no_grad():
                obs.copy_(torch.randn(obs.shape, device=dev, generator=gen))
                act.copy_(torch.randn(act.shape, device=dev, generator=gen))
                adv.copy_(torch.randn(adv.shape, device=dev, generator=gen))
                ret.copy_(torch.randn(ret.shape, device=dev, generator=gen))
                perm.copy_(torch.randperm(N, device=dev, generator=gen))
        mode = os.environ.get("MODE", "plain")
        if mode == "sync":
            torch.cuda.synchronize()
            g.replay()
        elif mode == "stream":
            rs = replay_stream
            rs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(rs):
                g.replay()
            torch.cuda.current_stream().wait_stream(rs)
        else:
            g.replay()
        body(twin, opt2, a2)
        torch.cuda.synchronize()
        dp = max(float((x - y).abs().max()) for x, y in zip(ac.parameters(), twin.parameters()))
        if dp != 0.0 and bad_at is None:
            bad_at = (r, dp)
    dp = max(float((x - y).abs().max()) for x, y in zip(ac.parameters(), twin.parameters()))
    print(f"perm={perm_on:d} dist={dist_on:d} clip={clip_on:d} rows={rows} K={K} reps={R}: first diff {bad_at} dparam {dp:.1e} "
          f"finite {all(bool(torch.isfinite(p).all()) for p in ac.parameters())}", flush=True)


trial(1, 1, 1, 24576, K=1)
trial(1, 1, 1, 24576, K=20)
trial(0, 0, 0, 4096, K=1)
trial(1, 1, 1, 4096, K=1)
