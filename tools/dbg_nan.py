"""Debug: find where non-finite values first appear in the bench flow (env leg, rollouts, PPO)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "unitree-rl-gym_amd"))
import torch  # noqa: E402
import isaacgym  # noqa: F401,E402
from legged_gym.envs import task_registry  # noqa: E402
from legged_gym.utils import get_args  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402
from rsl_rl.runners import OnPolicyRunner  # noqa: E402


def bad(t):
    return int((~torch.isfinite(t)).reshape(t.shape[0], -1).any(dim=1).sum()) if t is not None else 0


def report(env, tag):
    r = {k: bad(v) for k, v in (("root", env.root_states), ("dofs", env.dof_state.view(env.num_envs, -1)),
                                 ("obs", env.obs_buf), ("rew", env.rew_buf.view(-1, 1)),
                                 ("cf", env._contact_forces.view(env.num_envs, -1)))}
    big = int((env.root_states[:, 7:13].abs() > 1e3).any(dim=1).sum())
    print(tag, r, "huge-vel envs", big, "max |v|", float(env.root_states[:, 7:13].abs().max()), flush=True)
    return sum(r.values())


def main(n=4096):
    dev = "cuda:0"
    gargs = get_args(["--task", "go2", "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name="go2", args=gargs)
    _, train_cfg = task_registry.get_cfgs("go2")
    runner = OnPolicyRunner(env, class_to_dict(train_cfg), log_dir=None, device=dev)
    runner.alg.use_graph = os.environ.get("PPO_GRAPH", "1") == "1"
    print("use_graph", runner.alg.use_graph, flush=True)
    alg = runner.alg
    orig_update = alg.update

    def nf(t):
        return int((~torch.isfinite(t)).sum())

    def upd():
        st = alg.storage
        pre = {k: nf(getattr(st, k)) for k in ("observations", "actions", "values", "returns", "advantages",
                                               "actions_log_prob", "mu", "sigma", "rewards")}
        pmax = max(float(p.detach().abs().max()) for p in alg.actor_critic.parameters())
        print("  pre-update storage non-finite", pre, "adv absmax", float(st.advantages.abs().max()),
              "ret absmax", float(st.returns.abs().max()), "param absmax", pmax, flush=True)
        out = orig_update()
        torch.cuda.synchronize()
        opt = alg.optimizer
        sm = [float(opt.state[p]["step"]) if "step" in opt.state[p] else -1 for p in alg.actor_critic.parameters()][:2]
        ea = max(float(opt.state[p]["exp_avg_sq"].abs().max()) for p in alg.actor_critic.parameters())
        print("  post-update losses", out, "adam step", sm, "exp_avg_sq max", ea, flush=True)
        return out
    alg.update = upd
    g = torch.Generator(device=dev).manual_seed(0)
    acts = [0.5 * torch.randn(n, env.num_actions, device=dev, generator=g) for _ in range(8)]
    for i in range(220):
        env.step(acts[i % 8])
        if i % 20 == 19 and report(env, f"env-leg step {i}"):
            break
    for it in range(8):
        runner.learn(1, init_at_random_ep_len=(it == 0))
        ps = [p for p in runner.alg.actor_critic.parameters()]
        nonfinite = sum(int((~torch.isfinite(p)).sum()) for p in ps)
        st = runner.alg.storage
        print(f"iter {it}: losses {runner.alg._last_losses if hasattr(runner.alg, '_last_losses') else ''} lr {float(runner.alg._lr):.2e} params non-finite {nonfinite}, std {runner.alg.actor_critic.std.detach().cpu().numpy().round(3)}",
              flush=True)
        report(env, f"  after iter {it}")
        if nonfinite:
            break


if __name__ == "__main__":
    main()
