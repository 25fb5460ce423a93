"""Run-to-run stability of the fused LSTM backward (pmlp_lstm_bwd_dw_mfma_jobs, both memories, the
H1 update's mini-batch: T = 24, B = 2048, I = 41 / 44): one forward, then the backward N times on
the same inputs, counting the launches whose weight-gradient slabs differ from the first launch's
(the kernel has no atomics: any difference is a race).  With the libppomlp.so named by PPOMLP_LIB.
usage: [PPOMLP_LIB=...] python tools/probes/lstm_bwd_race.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
from rsl_rl.modules import lstm_seq as ls  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
T, B, H = 24, 2048, 64
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
L = ls._lib()
reset = (torch.rand(T, B, device=dev, generator=g) < 0.02).to(torch.uint8)
keep, jobs = [], []
P = lambda t: t.data_ptr()  # noqa: E731
for I in (41, 44):
    R = lambda *s: 0.3 * torch.randn(*s, device=dev, generator=g)  # noqa: E731
    x, wih, bih, bhh, whh = R(T, B, I), R(4 * H, I), R(4 * H), R(4 * H), R(4 * H, H)
    h0, c0 = R(B, H), R(B, H)
    hout, cout, gact = (torch.empty(T, B, n, device=dev) for n in (H, H, 4 * H))
    xh = torch.empty(T, B, I + H + 1, device=dev)
    dh = R(T, B, H)
    slab = torch.empty(L.pmlp_lstm_bwd_dw_blocks(B), 4 * H * (I + H + 1), device=dev)
    keep.append((x, wih, bih, bhh, whh, h0, c0, hout, cout, gact, xh, dh, slab))
    jobs.append(ls.LstmJob(I, P(x), P(wih), P(bih), P(bhh), P(whh), P(h0), P(c0), P(hout), P(cout), P(gact),
                           P(xh), P(dh), P(slab), None, None))
arr = (ls.LstmJob * 2)(*jobs)
st = torch.cuda.current_stream().cuda_stream
ls._ok(L.pmlp_lstm_fwd_mfma_jobs(2, arr, T, B, H, P(reset), st), "fwd")
ls._ok(L.pmlp_lstm_bwd_dw_mfma_jobs(2, arr, T, B, H, P(reset), st), "bwd")
ref = [k[-1].clone() for k in keep]
bad = torch.zeros((), dtype=torch.int64, device=dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(N):
    ls._ok(L.pmlp_lstm_bwd_dw_mfma_jobs(2, arr, T, B, H, P(reset), st), "bwd")
    bad += sum((k[-1] != r).any().to(torch.int64) for k, r in zip(keep, ref))
    if i % 2000 == 1999:
        torch.cuda.synchronize()
        print(f"  {i + 1} launches, {int(bad)} differing slabs", flush=True)
e1.record()
torch.cuda.synchronize()
print(f"{os.path.basename(os.environ.get('PPOMLP_LIB', 'libppomlp.so'))}: {N} backward launches, "
      f"{int(bad)} with slabs differing from the first ({e0.elapsed_time(e1) / N * 1e3:.0f} us per launch "
      f"and check)", flush=True)
