"""rocprof target: 10 x (actor+critic fwd+bwd) on the MFMA kernels, 24576 rows."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
from rsl_rl.modules import mfma_mlp  # noqa: E402
from rsl_rl.modules.actor_critic import mlp, get_activation  # noqa: E402
a = mlp(48, [512, 256, 128], 12, get_activation("elu")).cuda()
c = mlp(48, [512, 256, 128], 1, get_activation("elu")).cuda()
x = torch.randn(24576, 48, device="cuda")
for _ in range(10):
    (mfma_mlp.mlp_apply(a, x).square().mean() + mfma_mlp.mlp_apply(c, x).square().mean()).backward()
torch.cuda.synchronize()
print("done")
