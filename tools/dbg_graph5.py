"""Debug: graph replay vs the same update run eagerly (same state, same permutation), per iteration."""
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


def main(n=4096):
    dev = "cuda:0"
    gargs = get_args(["--task", "go2", "--num_envs", str(n), "--headless"])
    env, _ = task_registry.make_env(name="go2", args=gargs)
    _, train_cfg = task_registry.get_cfgs("go2")
    runner = OnPolicyRunner(env, class_to_dict(train_cfg), log_dir=None, device=dev)
    alg = runner.alg
    alg.actor_critic.mixed_precision = os.environ.get("MP", "1") == "1"
    alg.num_learning_epochs = int(os.environ.get("EPOCHS", alg.num_learning_epochs))
    alg.num_mini_batches = int(os.environ.get("MB", alg.num_mini_batches))
    if os.environ.get("SCHED"):
        alg.schedule = os.environ["SCHED"]
    print("schedule", alg.schedule, "max_grad_norm", alg.max_grad_norm)
    print("epochs", alg.num_learning_epochs, "minibatches", alg.num_mini_batches, flush=True)
    params = list(alg.actor_critic.parameters())
    orig_update = alg.update

    def save():
        return ([p.detach().clone() for p in params],
                [{k: (v.clone() if torch.is_tensor(v) else v) for k, v in alg.optimizer.state[p].items()} for p in params],
                alg._lr.clone())

    def load(s):
        with torch.no_grad():
            for p, v in zip(params, s[0]):
                p.copy_(v)
            for p, o in zip(params, s[1]):
                for k, v in o.items():
                    if torch.is_tensor(v):
                        alg.optimizer.state[p][k].copy_(v)
            alg._lr.copy_(s[2])

    def upd():
        if alg._graph is None:
            return orig_update()
        st = alg.storage
        s0 = save()
        batch = st.num_envs * st.num_transitions_per_env
        mb = batch // alg.num_mini_batches
        perm = torch.randperm(alg.num_mini_batches * mb, device=dev)
        # eager, same permutation, same body as the graph
        if alg._diag is not None:
            alg._diag_i = 0
        alg._capturing = True  # static-grad semantics (zero_grad set_to_none=False)
        acc = torch.zeros(2, device=dev)
        adv = st.advantages.flatten(0, 1)
        R = int(os.environ.get("REPLAYS", 1))
        for _k in range(alg.num_learning_epochs * R):
            for i in range(alg.num_mini_batches):
                idx = perm[i * mb:(i + 1) * mb]
                tens = [None if t is None else t.index_select(0, idx) for t in alg._flat]
                tens[4] = adv.index_select(0, idx)
                alg._minibatch_step(*tens, (None, None), None, acc)
                if os.environ.get("TRACE") and alg._diag is not None:
                    print(f"    eager step {_k}: {alg._diag[(alg._diag_i - 1) % alg._diag.shape[0]].tolist()[:3]} psum {sum(float(p.double().sum()) for p in params):.9e} std0 {float(params[-1].view(-1)[0]) if params[-1].numel() else 0:.9e}", flush=True)
        alg._capturing = False
        pe = [p.detach().clone() for p in params]
        de = alg._diag.clone() if alg._diag is not None else None
        lre = float(alg._lr)
        load(s0)
        alg._perm.copy_(perm)
        mode = os.environ.get("REPLAY_MODE", "plain")
        if mode == "sync":
            torch.cuda.synchronize()
            alg._graph.replay()
        elif mode == "side":
            side = alg._side
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                alg._graph.replay()
            torch.cuda.current_stream().wait_stream(side)
        elif mode == "plainsync":
            for _r in range(int(os.environ.get("REPLAYS", 1))):
                alg._graph.replay()
                torch.cuda.synchronize()
                if os.environ.get("TRACE") and alg._diag is not None:
                    print(f"    graph rep  {_r}: {alg._diag[0].tolist()[:3]} psum {sum(float(p.double().sum()) for p in params):.9e} std0 {float(params[-1].view(-1)[0]) if params[-1].numel() else 0:.9e}", flush=True)
        elif mode == "stream":
            s2 = alg._side
            s2.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s2):
                for _r in range(int(os.environ.get("REPLAYS", 1))):
                    alg._graph.replay()
            torch.cuda.current_stream().wait_stream(s2)
        else:
            for _r in range(int(os.environ.get("REPLAYS", 1))):
                alg._graph.replay()
        torch.cuda.synchronize()
        if de is not None:
            torch.set_printoptions(precision=6, linewidth=200, sci_mode=True)
            print("   diag eager:", de.cpu())
            print("   diag graph:", alg._diag.cpu())
        d = max(float((p.detach() - q).abs().max()) for p, q in zip(params, pe))
        fin = all(bool(torch.isfinite(p).all()) for p in params)
        print(f"  replay vs eager: max |dparam| {d:.3e}  lr eager {lre:.3e} graph {float(alg._lr):.3e}  "
              f"graph finite {fin}  eager finite {all(bool(torch.isfinite(q).all()) for q in pe)}  "
              f"acc graph {alg._acc.tolist()} eager {acc.tolist()}", flush=True)
        means = (alg._acc / (alg.num_learning_epochs * alg.num_mini_batches)).tolist()
        st.clear()
        return means[0], means[1]

    alg.update = upd
    if os.environ.get("DIAG"):
        alg._diag = torch.zeros(alg.num_learning_epochs * alg.num_mini_batches, 8, device=dev)
    runner.learn(1, init_at_random_ep_len=True)  # eager
    runner.learn(1)  # capture (orig_update path via _graph None) -> builds the graph
    for it in range(int(os.environ.get("ITERS", 4))):
        runner.learn(1)


if __name__ == "__main__":
    main()
