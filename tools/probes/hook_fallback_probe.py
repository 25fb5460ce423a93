"""Diagnostic: which state differs between a runner whose collection capture failed (and fell
back to eager) and one that never tried, and whether two never-tried runners agree at all.
usage: python tools/probes/hook_fallback_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "unitree-rl-gym_amd"), os.path.join(ROOT, "tests")]
import isaacgym  # noqa: F401,E402
import test_gpu_step_hooks as T  # noqa: E402


def run(name, graph, iters):
    env, r = T._runner(name, T.H1HostSyncHook, rollout_graph=graph)
    r.learn(iters)
    torch.cuda.synchronize()
    return env, r


def cmp(tag, a, b):
    (ea, ra), (eb, rb) = a, b
    bad = [i for i, (p, q) in enumerate(zip(ra.alg.actor_critic.parameters(), rb.alg.actor_critic.parameters()))
           if not torch.equal(p, q)]
    st = [k for k in ("observations", "rewards", "actions", "values", "dones", "actions_log_prob")
          if not torch.equal(getattr(ra.alg.storage, k), getattr(rb.alg.storage, k))]
    print(f"{tag}: params differ {bad}; storage differs {st}; counters {ea.common_step_counter} {eb.common_step_counter}",
          flush=True)


for iters in (1, 2, 3):
    b1 = run(f"e1_{iters}", False, iters)
    b2 = run(f"e2_{iters}", False, iters)
    cmp(f"eager vs eager, {iters} it", b1, b2)
    a = run(f"t_{iters}", True, iters)
    cmp(f"try vs eager, {iters} it", a, b1)
