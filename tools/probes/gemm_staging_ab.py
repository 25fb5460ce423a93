"""A/B of the GEMM k-loop operand staging (pmlp_set_gemm_staging: 0 = register staging,
1 = LDS-DMA, one barrier per k-tile) on one fused PPO optimizer step (Go2 MLPs, 24,576-row
mini-batch): (1) bitwise equality of the parameters after one step from the same state;
(2) per-GEMM-group and whole-step times, interleaved rounds in one process."""
import collections
import ctypes as C
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
lib = mm.load()
lib.pmlp_set_gemm_staging.argtypes = [C.c_int32]
lib.pmlp_set_gemm_staging.restype = C.c_int32

# (1) bitwise: one step from the same state under each staging
f.ensure_weights()
snap = [t.clone() for t in (f.flat, f.exp_avg, f.exp_avg_sq, f.step_t, alg._lr)] + [w.clone() for ws in f.wb for w in ws]
outs = {}
for s in (0, 1, 2):
    for t, v in zip([f.flat, f.exp_avg, f.exp_avg_sq, f.step_t, alg._lr] + [w for ws in f.wb for w in ws], snap):
        t.copy_(v)
    lib.pmlp_set_gemm_staging(s)
    f.run(perm[:mb], src, acc)
    torch.cuda.synchronize()
    outs[s] = (f.flat.clone(), f.grad.clone(), [x.clone() for xs in f.y for x in xs], [o.clone() for o in f.out])
same = all(torch.equal(outs[0][0], outs[q][0]) and torch.equal(outs[0][1], outs[q][1]) for q in (1, 2)) and \
    all(torch.equal(a, b) for a, b in zip(outs[0][2], outs[1][2])) and all(torch.equal(a, b) for a, b in zip(outs[0][3], outs[1][3]))
print(f"bitwise equal (params, grad, activations, outputs): {same}")
if not same:
    print("  grad max|d|", float((outs[0][1] - outs[1][1]).abs().max()),
          " y max|d|", [float((a.float() - b.float()).abs().max()) for a, b in zip(outs[0][2], outs[1][2])],
          " out max|d|", [float((a - b).abs().max()) for a, b in zip(outs[0][3], outs[1][3])])

# (2) timing
times = collections.defaultdict(list)
record = [None]
stream = torch.cuda.current_stream()


def wrap(fn, keyf):
    def w(*a, **k):
        if record[0] is None:
            return fn(*a, **k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        r = fn(*a, **k)
        e1.record(stream)
        times[(record[0], keyf(*a, **k))].append((e0, e1))
        return r
    return w


EPI = {mm.EPI_FWD_HIDDEN: "FWD", mm.EPI_FWD_OUT: "FWD_OUT", mm.EPI_PARTIAL: "PARTIAL", mm.EPI_BWD_DX: "BWD_DX",
       mm.EPI_PARTIAL_TN: "PART_TN"}
mm._gemm = wrap(mm._gemm, lambda epi, jobs, ksplit=0: f"gemm {EPI.get(epi, epi):8s} M={jobs[0]['M']:6d} "
                f"N={jobs[0]['N']:4d} K={jobs[0]['K']:6d} x{len(jobs)}")
R = 20
tot = collections.defaultdict(list)
for rnd in range(3):
    for s in (0, 1, 2):
        lib.pmlp_set_gemm_staging(s)
        for i in range(3):
            f.run(perm[(i % 4) * mb:((i % 4) + 1) * mb], src, acc)
        torch.cuda.synchronize()
        record[0] = s
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(R):
            f.run(perm[(i % 4) * mb:((i % 4) + 1) * mb], src, acc)
        e1.record(stream)
        torch.cuda.synchronize()
        record[0] = None
        tot[s].append(e0.elapsed_time(e1) / R * 1e3)
keys = sorted({k for (_, k) in times})
print(f"{'group':48s} {'reg us':>8s} {'glds us':>8s} {'ring us':>8s}")
for k in keys:
    v = [sum(a.elapsed_time(b) for a, b in times[(s, k)]) / (3 * R) * 1e3 for s in (0, 1, 2)]
    print(f"{k:48s} {v[0]:8.1f} {v[1]:8.1f} {v[2]:8.1f}")
print(f"{'TOTAL eager optimizer step (min over rounds)':48s} {min(tot[0]):8.1f} {min(tot[1]):8.1f} {min(tot[2]):8.1f}")

# (3) the rollout's policy forward (4,096 rows, FusedRollout.forward: 4 GEMM launches)
ro = alg._rollout
obs = torch.randn(N, O, device="cuda")
rt = collections.defaultdict(list)
record[0] = None
for rnd in range(3):
    for s in (0, 1, 2):
        lib.pmlp_set_gemm_staging(s)
        for _ in range(5):
            ro.forward(obs, obs)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(50):
            ro.forward(obs, obs)
        e1.record(stream)
        torch.cuda.synchronize()
        rt[s].append(e0.elapsed_time(e1) / 50 * 1e3)
print(f"{'rollout forward 4096 rows (4 launches, min)':48s} {min(rt[0]):8.1f} {min(rt[1]):8.1f} {min(rt[2]):8.1f}")
