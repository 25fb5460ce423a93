"""Probe: the real rsl_rl PPO (graphed update) on synthetic rollouts, many updates; NaN / divergence check.
usage: python ppo_graph_stress.py [updates] [graph 0/1] [mp 0/1]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic  # noqa: E402

U = int(sys.argv[1]) if len(sys.argv) > 1 else 30
use_graph = (sys.argv[2] if len(sys.argv) > 2 else "1") == "1"
mp = (sys.argv[3] if len(sys.argv) > 3 else "1") == "1"
dev = "cuda"
torch.manual_seed(0)
N, T, O, A = 4096, 24, 48, 12
ac = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128], mixed_precision=mp).to(dev)
alg = PPO(ac, num_learning_epochs=5, num_mini_batches=4, learning_rate=1e-3, schedule="adaptive", desired_kl=0.01,
          entropy_coef=0.01, device=dev)
alg.use_graph = use_graph
if os.environ.get("FIXED"):
    alg.schedule = "fixed"
if os.environ.get("NOENT"):
    alg.entropy_coef = 0.0
if os.environ.get("NOVCLIP"):
    alg.use_clipped_value_loss = False
if os.environ.get("FOREACH"):
    alg.optimizer = torch.optim.Adam(ac.parameters(), lr=alg._lr, foreach=True, capturable=True)
if os.environ.get("NOCLIP"):
    alg.max_grad_norm = 1e9
alg.init_storage(N, T, [O], [None], [A])
g = torch.Generator(device=dev).manual_seed(1)
times = []
for u in range(U):
    if os.environ.get("FP32ROLL"):
        ac.mixed_precision = False
    with torch.inference_mode():
        obs = torch.randn(N, O, device=dev, generator=g)
        for t in range(T):
            alg.act(obs, obs)
            obs = torch.randn(N, O, device=dev, generator=g)
            rew = 0.1 * torch.randn(N, device=dev, generator=g)
            dones = (torch.rand(N, device=dev, generator=g) < 0.02)
            alg.process_env_step(rew, dones, {})
        alg.compute_returns(obs)
    ac.mixed_precision = mp
    torch.cuda.synchronize()
    import time as _t
    t0 = _t.time()
    vl, sl = alg.update()
    torch.cuda.synchronize()
    if u >= 3:
        times.append(_t.time() - t0)
    fin = all(bool(torch.isfinite(p).all()) for p in ac.parameters())
    if u % 5 == 0 or not fin:
        print(f"update {u}: value {vl:.4f} surr {sl:.4f} lr {float(alg._lr):.2e} std {float(ac.std.mean()):.4f} finite {fin}",
              flush=True)
    if not fin:
        break
print(f"graph={use_graph} mp={mp}: update median {sorted(times)[len(times)//2]*1e3:.2f} ms over {len(times)}", flush=True)
