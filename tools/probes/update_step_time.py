"""Per-launch-group timing of one fused PPO optimizer step (Go2 MLPs, 24,576-row
mini-batch): every pmlp_gemm / convert / loss / reduce / optimizer call bracketed by
HIP events on torch's current stream (the stream the library launches on)."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402

from rsl_rl.algorithms import PPO  # noqa: E402
from rsl_rl.modules import ActorCritic, mfma_mlp as mm  # noqa: E402

N, T, O, A = 4096, 24, 48, 12
torch.manual_seed(0)
ac = ActorCritic(O, O, A, [512, 256, 128], [512, 256, 128]).cuda()
alg = PPO(ac, num_learning_epochs=5, num_mini_batches=4, device="cuda")
alg.init_storage(N, T, [O], [None], [A])
st = alg.storage
g = torch.Generator(device="cuda").manual_seed(1)
for k in ("observations", "actions", "values", "returns", "advantages", "mu"):
    getattr(st, k).copy_(torch.randn(getattr(st, k).shape, device="cuda", generator=g))
st.sigma.fill_(1.0)
st.actions_log_prob.copy_(-12.0 + torch.randn(st.actions_log_prob.shape, device="cuda", generator=g))
f = alg._fused
mb = f.M
src = (st.observations.flatten(0, 1), st.observations.flatten(0, 1), st.actions.flatten(0, 1),
       st.values.flatten(0, 1), st.advantages.flatten(0, 1), st.returns.flatten(0, 1),
       st.actions_log_prob.flatten(0, 1), st.mu.flatten(0, 1), st.sigma.flatten(0, 1))
acc = torch.zeros(2, device="cuda")
perm = torch.randperm(4 * mb, device="cuda")

times = collections.defaultdict(list)
record = [False]
stream = torch.cuda.current_stream()


def wrap(name, fn, keyf):
    def w(*a, **k):
        if not record[0]:
            return fn(*a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r = fn(*a, **k)
        e1.record(stream)
        times[keyf(*a, **k)].append((e0, e1))
        return r
    return w


EPI = {mm.EPI_FWD_HIDDEN: "FWD", mm.EPI_FWD_OUT: "FWD_OUT", mm.EPI_PARTIAL: "PARTIAL", mm.EPI_BWD_DX: "BWD_DX",
       mm.EPI_PARTIAL_TN: "PART_TN"}
mm._gemm = wrap("gemm", mm._gemm, lambda epi, jobs, ksplit=0: f"gemm {EPI.get(epi, epi):8s} M={jobs[0]['M']:6d} "
                f"N={jobs[0]['N']:4d} K={jobs[0]['K']:6d} x{len(jobs)}")
mm._convert = wrap("convert", mm._convert, lambda jobs: "convert")
mm._reduce = wrap("reduce", mm._reduce, lambda jobs: "reduce slabs")
mm.mlp_forward = wrap("mlp_forward", mm.mlp_forward, lambda nets, M: f"mlp_forward (fused, both nets) M={M}")

for i in range(3):
    f.run(perm[(i % 4) * mb:((i % 4) + 1) * mb], src, acc)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
R = 20
record[0] = True
e0.record(stream)
for i in range(R):
    f.run(perm[(i % 4) * mb:((i % 4) + 1) * mb], src, acc)
e1.record(stream)
torch.cuda.synchronize()
tot = e0.elapsed_time(e1) / R * 1e3
acc_us = 0.0
for k, v in times.items():
    us = sum(a.elapsed_time(b) for a, b in v) / R * 1e3
    acc_us += us
    print(f"{us:8.1f} us/step  {k}")
print(f"{tot:8.1f} us/step  TOTAL eager step (sum of timed groups {acc_us:.1f}; rest = loss/optimizer/launch gaps)")
