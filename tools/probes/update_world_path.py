"""The world > 1 optimizer step's kernel structure, timed on one GPU ("the
world > 1 optimizer step is 11 launches plus the collective ... untimed").  Captured Go2 PPO
update (4096 envs x 24 steps, 5 x 4 mini-batches), interleaved rounds in one process:
  w1      the shipped world-size-1 step (7 launches: the norm partials and the step / LR
          bookkeeping folded into the slab-reduce launch);
  w1nf    world size 1 with that fold off (8 launches: k_opt_prepare after the reduce) --
          the world > 1 step without its collective;
  w2path  the world > 1 code path (PPO.world_size forced to 2 after construction) on a
          one-rank RCCL group: the 8 launches plus the captured all-reduce of the one
          bucket (1.52 MB), which on one rank is RCCL's local copy -- the xGMI transfer
          itself is only measured by a multi-GPU run.
usage: python tools/probes/update_world_path.py"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic  # noqa: E402

N, T, O, A = 4096, 24, 48, 12


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def build(variant):
    torch.manual_seed(0)
    ac = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda()
    alg = PPO(ac, num_learning_epochs=5, num_mini_batches=4, device="cuda")
    if variant == "w2path":
        alg.world_size = 2
    alg.init_storage(N, T, [O], [None], [A])
    if variant == "w1nf":
        alg._fused.fold_opt = False
    st = alg.storage
    g = torch.Generator(device="cuda").manual_seed(1)
    for k in ("observations", "actions", "values", "returns", "advantages", "mu"):
        getattr(st, k).copy_(torch.randn(getattr(st, k).shape, device="cuda", generator=g))
    st.sigma.fill_(1.0)
    st.actions_log_prob.copy_(-12.0 + torch.randn(st.actions_log_prob.shape, device="cuda", generator=g))
    for _ in range(3):  # eager, then capture + replay
        st.step = T
        alg.update()
    assert alg._fgraph is not None, variant
    return alg


def main():
    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    algs = {v: build(v) for v in ("w1", "w1nf", "w2path")}
    times = {v: [] for v in algs}
    for rnd in range(7):
        for v, alg in algs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                alg._fgraph.replay()
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 5)
    base = sorted(times["w1"])[3]
    for v, ts in times.items():
        ts.sort()
        print(f"{v:7s} update {ts[3]:.3f} ms median ({ts[0]:.3f} min), {ts[3] - base:+.3f} ms vs w1, "
              f"{(ts[3] - base) / 20 * 1e3:+.1f} us per optimizer step", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
