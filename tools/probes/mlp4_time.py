"""Time the register-chained policy forward (pmlp_mlp4_forward) against the
convert + per-layer GEMM path, actor + critic on N rows."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "unitree-rl-gym_amd"))
import torch  # noqa: E402
from rsl_rl.algorithms import PPO, fused_step  # noqa: E402
from rsl_rl.modules import ActorCritic, mfma_mlp  # noqa: E402

for N in (4096, 24576):
    torch.manual_seed(0)
    alg = PPO(ActorCritic(48, 48, 12, [512, 256, 128], [512, 256, 128]).cuda(), device="cuda")
    alg.init_storage(N, 24, [48], [None], [12])
    ro = alg._rollout
    obs = torch.randn(N, 48, device="cuda")
    res = {}
    for regs in (True, False):
        ro.regs = regs and mfma_mlp.mlp4_supported([alg.actor_critic.actor, alg.actor_critic.critic])
        for _ in range(5):
            ro.forward(obs, obs)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            ro.forward(obs, obs)
        e1.record()
        torch.cuda.synchronize()
        res[regs] = (e0.elapsed_time(e1) / 50 * 1e3, [o.clone() for o in ro.out])
    d = max(float((a - b).abs().max() / b.abs().max()) for a, b in zip(res[True][1], res[False][1]))
    print(f"N={N}: regs {res[True][0]:.1f} us, gemm path {res[False][0]:.1f} us, rel diff {d:.2e}", flush=True)
