"""Phase clocks of pmlp_mlp_forward (Go2 update shape: both nets, 24,576 gathered rows, hidden
outputs stored) from the diagnostic build (make build/libppomlp_fstamps.so, -DPMLP_FMLP_STAMPS):
per workgroup s_memtime at job start, after input staging, after each layer and each hidden-
output store; prints the median and max over workgroups of each phase.

usage: PPOMLP_LIB=unitree-rl-gym_amd/csrc/build/libppomlp_fstamps.so python tools/probes/fused_fwd_stamps.py
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools", "probes"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import fused_fwd_time as F  # noqa: E402  (builds the PPO, the jobs and times the cases)

lib = F.mfma_mlp.load()
lib.pmlp_diag_fmlp_stamps.argtypes = [C.c_void_p, C.c_int]
NS = 20
js = F.jobs(F.M, F.idx, True)
for _ in range(3):
    F.mfma_mlp.mlp_forward(js, F.M)
torch.cuda.synchronize()
F.mfma_mlp.mlp_forward(js, F.M)
torch.cuda.synchronize()
nb = (F.M + 95) // 96
buf = np.zeros(4096 * NS, dtype=np.uint64)
assert lib.pmlp_diag_fmlp_stamps(buf.ctypes.data, buf.size) == 0
st = buf.reshape(4096, NS)[:nb, :18].astype(np.int64)
names = ["stage x", "layer0", "sync+store y0", "layer1", "sync+store y1", "layer2", "sync+store y2",
         "layer3+sync"]
t0 = st[:, 0].min()
print(f"workgroups {nb}; span {(st[:, 17].max() - t0)} clocks; start skew {st[:, 0].max() - t0}")
for j in range(2):
    for k, nm in enumerate(names):
        d = st[:, 9 * j + k + 1] - st[:, 9 * j + k]
        print(f"job {j} {nm:14s} median {int(np.median(d)):7d}  max {int(d.max()):7d}")
    if j == 0:
        d = st[:, 9] - st[:, 8]
        print(f"between jobs   median {int(np.median(d)):7d}")
print("per workgroup total median", int(np.median(st[:, 17] - st[:, 0])))
