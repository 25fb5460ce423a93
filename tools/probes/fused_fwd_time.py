"""Time pmlp_mlp_forward (the fused 4-layer forward of both Go2 nets, 24,576 gathered rows) and
variants that drop one piece of its work, to place its time: no hidden-output stores (y), no
row gather, one net only, and the rollout's 4096-row shape.  HIP events around 200 launches.

usage: python tools/probes/fused_fwd_time.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic, mfma_mlp  # noqa: E402

N, T, O, A = 4096, 24, 48, 12
torch.manual_seed(0)
alg = PPO(ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda(), num_learning_epochs=1,
          num_mini_batches=4, device="cuda")
alg.init_storage(N, T, [O], [None], [A])
f = alg._fused
f.ensure_weights()
x = torch.randn(T * N, O, device="cuda")
M = T * N // 4
idx = torch.randperm(T * N, device="cuda")[:M]


x2 = x.clone()  # the same rows in another tensor: the kernel cannot reuse job 0's staged input


def jobs(M, rows, ys, nets=(0, 1), frag=True, share=True):
    y = [[torch.empty((M, lin.out_features), dtype=torch.bfloat16, device="cuda") for lin in ls[:-1]]
         for ls in f.lins]
    out = [torch.empty((M, ls[-1].out_features), device="cuda") for ls in f.lins]
    xa = torch.empty((M, f.k0p[0]), dtype=torch.bfloat16, device="cuda")
    return [dict(x=x if (n == 0 or share) else x2, kx=O, rows=rows, xa=xa if (n == 0 and ys) else None,
                 K0=f.k0p[n], W=f.wb[n], Wf=f.wf[n] if (f.wf and frag) else None,
                 b=[lin.bias.detach() for lin in f.lins[n]], N=[lin.out_features for lin in f.lins[n]],
                 y=y[n] if ys else None, out=out[n]) for n in nets]


def time_it(js, M, R=200):
    for _ in range(5):
        mfma_mlp.mlp_forward(js, M)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(R):
        mfma_mlp.mlp_forward(js, M)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / R * 1e3


cases = [("update: both nets, gather, y stores", jobs(M, idx, True), M),
         ("update: .. critic input gathered again", jobs(M, idx, True, share=False), M),
         ("update: .. row-major weights", jobs(M, idx, True, frag=False), M),
         ("update: .. row-major, gathered again", jobs(M, idx, True, frag=False, share=False), M),
         ("update: no y stores", jobs(M, idx, False), M),
         ("update: no gather", jobs(M, None, True), M),
         ("update: actor only", jobs(M, idx, True, (0,)), M),
         ("rollout: 4096 rows, no y", jobs(N, None, False), N)]
for rnd in range(2):
    for name, js, m in cases:
        print(f"round {rnd}  {name:42s} {time_it(js, m):7.1f} us", flush=True)
