"""Times the recurrent heads kernels on the update's shape (pmlp_heads_forward / _backward, both
nets, M = 49,152 rows of H = 64: an H1 / H1_2 8192-env mini-batch) with the libppomlp.so named
by PPOMLP_LIB, and digests their outputs (for a bitwise comparison of two builds).
usage: [PPOMLP_LIB=...] python tools/probes/heads_time.py [M]"""
import ctypes as C
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
from rsl_rl.modules import mfma_mlp as mm  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 49152
H, N0 = 64, 32
g = torch.Generator(device="cuda").manual_seed(0)
dev = "cuda"
lib = mm.load()
bufs, jobs = [], []
for N1 in (10, 1):
    h = torch.randn(M, H, device=dev, generator=g)
    W0, b0 = 0.2 * torch.randn(N0, H, device=dev, generator=g), 0.1 * torch.randn(N0, device=dev, generator=g)
    W1, b1 = 0.2 * torch.randn(N1, N0, device=dev, generator=g), 0.1 * torch.randn(N1, device=dev, generator=g)
    y0, out = torch.empty(M, N0, device=dev), torch.empty(M, N1, device=dev)
    dout = torch.randn(M, N1, device=dev, generator=g)
    dh = torch.empty(M, H, device=dev)
    nb = lib.pmlp_heads_blocks(M)
    slab = torch.empty(nb, N0 * H + N0 + N1 * N0 + N1, device=dev)
    bufs.append((h, W0, b0, W1, b1, y0, out, dout, dh, slab))
    P = lambda t: t.data_ptr()  # noqa: E731
    jobs.append(mm.HeadJob(P(h), P(W0), P(b0), P(W1), P(b1), P(y0), P(out), P(dout), P(dh), P(slab), N0, N1))
arr = (mm.HeadJob * 2)(*jobs)
st = torch.cuda.current_stream().cuda_stream


def run(fn):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


tf = run(lambda: mm._ok(lib.pmlp_heads_forward(2, arr, M, H, st), "fwd"))
tb = run(lambda: mm._ok(lib.pmlp_heads_backward(2, arr, M, H, st), "bwd"))
torch.cuda.synchronize()
dig = hashlib.sha256()
for b in bufs:
    for t in (b[5], b[6], b[8], b[9]):
        dig.update(t.cpu().numpy().tobytes())
print(f"{os.path.basename(os.environ.get('PPOMLP_LIB', 'libppomlp.so'))}: heads fwd {tf:.1f} us, bwd {tb:.1f} us "
      f"(M = {M}); outputs {dig.hexdigest()[:16]}", flush=True)
