"""OnPolicyRunner (rsl_rl v1.0.2 API; call sites task_registry.py:119,126,
train.py:14, play.py:34,39).  Checkpoint dict keys and log tags are the same."""
import json
import os
import statistics
import time
import warnings
from collections import deque

import torch
import torch.distributed as dist

from rsl_rl.algorithms import PPO  # noqa: F401  (eval'd by name)
from rsl_rl.env import VecEnv
from rsl_rl.modules import ActorCritic, ActorCriticRecurrent  # noqa: F401  (eval'd by name)


class _JsonlWriter:
    """Fallback when tensorboard is not installed: one JSON line per scalar."""

    def __init__(self, log_dir, flush_secs=10):
        os.makedirs(log_dir, exist_ok=True)
        self._f = open(os.path.join(log_dir, "scalars.jsonl"), "a")

    def add_scalar(self, tag, value, step):
        self._f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step)}) + "\n")

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def _make_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=log_dir, flush_secs=10)
    except Exception:
        return _JsonlWriter(log_dir)


class _RolloutGraph:
    """The collection loop of OnPolicyRunner.learn (num_steps_per_env x act -> env.step
    -> process_env_step) captured once and replayed every iteration.

    Every tensor the loop reads or writes is static: the env's parity-double-buffered
    obs/reset buffers (num_steps_per_env is even, so the parity returns), the rollout
    storage slots, the policy's buffers, and the env's device-side step counter, which
    the native step advances itself so replays draw fresh noise/commands.  Episode
    logging (the eager loop's .nonzero()/.cpu() per step) becomes per-step device
    records read back once per iteration, in the same order."""

    def __init__(self, runner, obs, critic_obs, cur_reward_sum, cur_episode_length):
        self.runner = runner
        T, N = runner.num_steps_per_env, runner.env.num_envs
        if T % 2:
            raise ValueError("rollout graph needs an even num_steps_per_env (env buffer parity)")
        dev = runner.device
        self.T = T
        self.log = runner.log_dir is not None
        with torch.inference_mode(False):  # ordinary tensors: the graph writes them in place
            self.done = torch.zeros(T, N, dtype=torch.bool, device=dev)
            self.done_rew = torch.zeros(T, N, device=dev)
            self.done_len = torch.zeros(T, N, device=dev)
        self.ep_infos = []
        env, storage = runner.env, runner.alg.storage
        step0, storage0 = env.common_step_counter, storage.step
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        # captured outside inference mode: the graph's RNG offset tensors must stay
        # ordinary tensors (replays update them in place)
        with torch.inference_mode(False), torch.no_grad(), torch.cuda.graph(self.graph):
            for t in range(T):
                obs, critic_obs, rewards, dones, infos = runner._collect_step(obs, critic_obs)
                if self.log:
                    if "episode" in infos:
                        self.ep_infos.append(infos["episode"])
                    cur_reward_sum += rewards
                    cur_episode_length += 1
                    d = dones > 0
                    self.done[t].copy_(d)
                    self.done_rew[t].copy_(cur_reward_sum)
                    self.done_len[t].copy_(cur_episode_length)
                    cur_reward_sum.masked_fill_(d, 0.0)
                    cur_episode_length.masked_fill_(d, 0.0)
        # capture issued nothing: restore the host-side counters the loop advanced
        env.common_step_counter = step0
        storage.step = storage0
        self.obs, self.critic_obs = obs, critic_obs
        # the fused rollout's last process_env_step is deferred (FusedRollout.store): every
        # replay leaves it pending exactly as the captured loop did
        ro = runner.alg._rollout
        self.pending = getattr(ro, "pending", None)

    def matches(self, obs, critic_obs):
        """The loop's inputs are the buffers it was captured on (same env-buffer parity)."""
        return obs is self.obs and critic_obs is self.critic_obs

    def replay(self):
        with torch.inference_mode(False):
            self.graph.replay()
        self.runner.env.account_replayed_steps(self.T)
        self.runner.alg.storage.step = self.T
        if self.pending is not None:
            self.runner.alg._rollout.pending = self.pending
        return self.obs, self.critic_obs

    def finished_episodes(self, rewbuffer, lenbuffer):
        """Extend the logging deques exactly as the eager loop would (step-major, env order)."""
        done = self.done.cpu()
        if done.any():
            rewbuffer.extend(self.done_rew.cpu()[done].tolist())
            lenbuffer.extend(self.done_len.cpu()[done].tolist())


class OnPolicyRunner:
    def __init__(self, env: VecEnv, train_cfg, log_dir=None, device="cpu"):
        self.cfg = train_cfg["runner"]
        self.alg_cfg = train_cfg["algorithm"]
        self.policy_cfg = train_cfg["policy"]
        self.device = device
        self.env = env
        num_critic_obs = self.env.num_privileged_obs if self.env.num_privileged_obs is not None else self.env.num_obs
        actor_critic_class = eval(self.cfg["policy_class_name"])
        actor_critic = actor_critic_class(self.env.num_obs, num_critic_obs, self.env.num_actions,
                                          **self.policy_cfg).to(self.device)
        alg_class = eval(self.cfg["algorithm_class_name"])
        self.alg: PPO = alg_class(actor_critic, device=self.device, **self.alg_cfg)
        self.num_steps_per_env = self.cfg["num_steps_per_env"]
        self.save_interval = self.cfg["save_interval"]
        self.alg.init_storage(self.env.num_envs, self.num_steps_per_env, [self.env.num_obs],
                              [self.env.num_privileged_obs], [self.env.num_actions])
        self.is_main = not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
        self.log_dir = log_dir if self.is_main else None
        self.writer = None
        self.tot_timesteps = 0
        self.tot_time = 0
        self.current_learning_iteration = 0
        self._cur_reward_sum = torch.zeros(self.env.num_envs, dtype=torch.float, device=self.device)
        self._cur_episode_length = torch.zeros(self.env.num_envs, dtype=torch.float, device=self.device)
        self._rollout_graph = None
        self._eager_rollouts = 0
        self.sync_phase_times = False  # True: device-exact collection / learning times (see learn)
        _, _ = self.env.reset()

    def learn(self, num_learning_iterations, init_at_random_ep_len=False):
        if self.log_dir is not None and self.writer is None:
            self.writer = _make_writer(self.log_dir)
        if init_at_random_ep_len:
            self.env.episode_length_buf = torch.randint_like(self.env.episode_length_buf,
                                                             high=int(self.env.max_episode_length))
        obs = self.env.get_observations()
        privileged_obs = self.env.get_privileged_observations()
        critic_obs = privileged_obs if privileged_obs is not None else obs
        obs, critic_obs = obs.to(self.device), critic_obs.to(self.device)
        self.alg.actor_critic.train()

        ep_infos = []
        rewbuffer = deque(maxlen=100)
        lenbuffer = deque(maxlen=100)
        # persistent (zeroed per learn() call, as the reference's locals start at zero)
        # so that a captured rollout graph can keep accumulating into them
        cur_reward_sum, cur_episode_length = self._cur_reward_sum, self._cur_episode_length
        cur_reward_sum.zero_()
        cur_episode_length.zero_()
        # The reference times the phases on the host clock alone (its learn() never waits for
        # the device).  A device sync after the collection makes collection_time exact but idles
        # the GPU while the host then issues GAE and the update (~0.24 ms per Go2 iteration), so
        # it is opt-in (sync_phase_times: the profiling tools); the update's loss read-back
        # (PPO.update) synchronises once per iteration either way.
        exact = self.sync_phase_times and str(self.device).startswith("cuda")
        sync = (lambda: torch.cuda.synchronize(self.device)) if exact else (lambda: None)

        tot_iter = self.current_learning_iteration + num_learning_iterations
        for it in range(self.current_learning_iteration, tot_iter):
            start = time.time()
            with torch.inference_mode():
                # the env leaves each step's extras to the rollout's next policy launch
                # (LeggedRobot.defer_extras): one launch fewer per step; off outside collection
                defer = hasattr(self.env, "defer_extras")
                if defer:
                    self.env.defer_extras = self._defer_env_extras()
                try:
                    obs, critic_obs = self._collection(obs, critic_obs, ep_infos, rewbuffer, lenbuffer,
                                                       cur_reward_sum, cur_episode_length)
                finally:
                    if defer:
                        self.env.defer_extras = False
                sync()
                stop = time.time()
                collection_time = stop - start
                start = stop
                self.alg.compute_returns(critic_obs)
            if self.log_dir is not None or exact:
                mean_value_loss, mean_surrogate_loss = self.alg.update()
            else:  # nothing reads the losses: no read-back, the host stays ahead of the device
                mean_value_loss, mean_surrogate_loss = self.alg.update(host_means=False)
            sync()
            stop = time.time()
            learn_time = stop - start
            if self.log_dir is not None:
                self.log(locals())
                if it % self.save_interval == 0:
                    self.save(os.path.join(self.log_dir, f"model_{it}.pt"))
            ep_infos.clear()
            self.last_iteration_times = (collection_time, learn_time)
        self.current_learning_iteration += num_learning_iterations
        if self.log_dir is not None:
            self.save(os.path.join(self.log_dir, f"model_{self.current_learning_iteration}.pt"))

    def _collection(self, obs, critic_obs, ep_infos, rewbuffer, lenbuffer, cur_reward_sum, cur_episode_length):
        """The num_steps_per_env steps of one iteration's collection (on_policy_runner.py:106-125 of
        rsl_rl v1.0.2): the captured graph's replay, or the eager loop."""
        graph = self._rollout_graph
        if graph is not None and not graph.matches(obs, critic_obs):
            graph = self._rollout_graph = None
        if graph is None and self._eager_rollouts > 0 and self._rollout_graph_ok():
            # captured after one eager rollout has initialised everything lazily built
            graph = self._rollout_graph = self._capture_rollout(obs, critic_obs, cur_reward_sum,
                                                                cur_episode_length)
        if graph is not None:
            fused = getattr(self.alg, "_fused", None)
            if fused is not None:  # a load() since the capture: the graph reads the bf16 copies
                fused.ensure_weights()
            obs, critic_obs = graph.replay()
            if self.log_dir is not None:
                ep_infos.extend(graph.ep_infos)
                graph.finished_episodes(rewbuffer, lenbuffer)
        else:
            for _ in range(self.num_steps_per_env):
                obs, critic_obs, rewards, dones, infos = self._collect_step(obs, critic_obs)
                if self.log_dir is not None:
                    if "episode" in infos:
                        ep_infos.append(infos["episode"])
                    cur_reward_sum += rewards
                    cur_episode_length += 1
                    new_ids = (dones > 0).nonzero(as_tuple=False)
                    rewbuffer.extend(cur_reward_sum[new_ids][:, 0].cpu().numpy().tolist())
                    lenbuffer.extend(cur_episode_length[new_ids][:, 0].cpu().numpy().tolist())
                    cur_reward_sum[new_ids] = 0
                    cur_episode_length[new_ids] = 0
            self._eager_rollouts += 1
        return obs, critic_obs

    def _collect_step(self, obs, critic_obs):
        """One step of the reference's collection loop (on_policy_runner.py:106-114)."""
        actions = self.alg.act(obs, critic_obs)
        obs, privileged_obs, rewards, dones, infos = self.env.step(actions)
        critic_obs = privileged_obs if privileged_obs is not None else obs
        obs, critic_obs, rewards, dones = (obs.to(self.device), critic_obs.to(self.device),
                                           rewards.to(self.device), dones.to(self.device))
        self.alg.process_env_step(rewards, dones, infos)
        return obs, critic_obs, rewards, dones, infos

    def _capture_rollout(self, obs, critic_obs, cur_reward_sum, cur_episode_length):
        """_RolloutGraph, or None when the loop cannot be captured (e.g. a task's Python step
        hook that synchronises with the host, such as a .nonzero()): nothing inside a failed
        capture has executed on the device, so the host-side state the captured steps advanced
        (the env's buffer parity and step counter, the storage index, the rollout's deferred
        store) is put back as it was and the collection runs eagerly from then on."""
        objs = [o for o in (self.env, self.alg, self.alg.storage, getattr(self.alg, "_rollout", None))
                if o is not None]
        saved = [(o, dict(o.__dict__)) for o in objs]
        try:
            return _RolloutGraph(self, obs, critic_obs, cur_reward_sum, cur_episode_length)
        except RuntimeError as e:
            for o, d in saved:
                o.__dict__.clear()
                o.__dict__.update(d)
            if hasattr(self.env, "_stream"):
                # the native sim was pointed at the capture's stream: re-point it at the next step
                self.env._stream = None
            torch.cuda.synchronize(self.device)
            self._rollout_graph_failed = True
            warnings.warn(f"OnPolicyRunner: capturing the collection loop failed ({e}); collecting eagerly")
            return None

    def _defer_env_extras(self):
        """The fused rollout consumes deferred env extras (its store launches do the work);
        runner cfg `defer_env_extras` = False keeps the env's own extras launch."""
        return bool(self.cfg.get("defer_env_extras", True)) and getattr(self.alg, "_rollout", None) is not None

    def _rollout_graph_ok(self):
        """The whole collection loop replays as one HIP graph when nothing in it needs
        the host: a CUDA device, a feed-forward policy or a recurrent one whose memory
        steps in place on the LSTM kernels (static state buffers, masked resets), and an
        env whose step keys its noise on a device-side counter
        (LeggedRobot.account_replayed_steps)."""
        ac = self.alg.actor_critic
        return (bool(self.cfg.get("rollout_graph", True)) and str(self.device).startswith("cuda")
                and not getattr(self, "_rollout_graph_failed", False)
                and (not ac.is_recurrent or (hasattr(ac, "rollout_capturable") and ac.rollout_capturable()))
                and hasattr(self.env, "account_replayed_steps") and self.alg.storage is not None)

    def log(self, locs, width=80, pad=35):
        ws = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.tot_timesteps += self.num_steps_per_env * self.env.num_envs * ws
        self.tot_time += locs["collection_time"] + locs["learn_time"]
        iteration_time = locs["collection_time"] + locs["learn_time"]
        it = locs["it"]
        ep_string = ""
        if locs["ep_infos"]:
            for key in locs["ep_infos"][0]:
                infotensor = torch.tensor([], device=self.device)
                for ep_info in locs["ep_infos"]:
                    v = ep_info[key]
                    if not isinstance(v, torch.Tensor):
                        v = torch.Tensor([v])
                    if len(v.shape) == 0:
                        v = v.unsqueeze(0)
                    infotensor = torch.cat((infotensor, v.to(self.device)))
                value = torch.mean(infotensor)
                self.writer.add_scalar("Episode/" + key, value, it)
                ep_string += f"""{f'Mean episode {key}:':>{pad}} {value:.4f}\n"""
        mean_std = self.alg.actor_critic.std.mean()
        fps = int(self.num_steps_per_env * self.env.num_envs * ws / iteration_time)
        self.writer.add_scalar("Loss/value_function", locs["mean_value_loss"], it)
        self.writer.add_scalar("Loss/surrogate", locs["mean_surrogate_loss"], it)
        self.writer.add_scalar("Loss/learning_rate", self.alg.learning_rate, it)
        self.writer.add_scalar("Policy/mean_noise_std", mean_std.item(), it)
        self.writer.add_scalar("Perf/total_fps", fps, it)
        self.writer.add_scalar("Perf/collection time", locs["collection_time"], it)
        self.writer.add_scalar("Perf/learning_time", locs["learn_time"], it)
        if len(locs["rewbuffer"]) > 0:
            self.writer.add_scalar("Train/mean_reward", statistics.mean(locs["rewbuffer"]), it)
            self.writer.add_scalar("Train/mean_episode_length", statistics.mean(locs["lenbuffer"]), it)
            self.writer.add_scalar("Train/mean_reward/time", statistics.mean(locs["rewbuffer"]), self.tot_time)
            self.writer.add_scalar("Train/mean_episode_length/time", statistics.mean(locs["lenbuffer"]), self.tot_time)
        head = f" \033[1m Learning iteration {it}/{locs['tot_iter']} \033[0m "
        lines = [
            "#" * width, head.center(width, " "), "",
            f"""{'Computation:':>{pad}} {fps:.0f} steps/s (collection: {locs['collection_time']:.3f}s, learning {locs['learn_time']:.3f}s)""",
            f"""{'Value function loss:':>{pad}} {locs['mean_value_loss']:.4f}""",
            f"""{'Surrogate loss:':>{pad}} {locs['mean_surrogate_loss']:.4f}""",
            f"""{'Mean action noise std:':>{pad}} {mean_std.item():.2f}""",
        ]
        if len(locs["rewbuffer"]) > 0:
            lines += [f"""{'Mean reward:':>{pad}} {statistics.mean(locs['rewbuffer']):.2f}""",
                      f"""{'Mean episode length:':>{pad}} {statistics.mean(locs['lenbuffer']):.2f}"""]
        lines += [ep_string.rstrip("\n"), "-" * width,
                  f"""{'Total timesteps:':>{pad}} {self.tot_timesteps}""",
                  f"""{'Iteration time:':>{pad}} {iteration_time:.2f}s""",
                  f"""{'Total time:':>{pad}} {self.tot_time:.2f}s""",
                  f"""{'ETA:':>{pad}} {self.tot_time / (it + 1) * (locs['num_learning_iterations'] - it):.1f}s"""]
        print("\n".join(lines))

    def save(self, path, infos=None):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        torch.save({"model_state_dict": self.alg.actor_critic.state_dict(),
                    "optimizer_state_dict": self.alg.optimizer.state_dict(),
                    "iter": self.current_learning_iteration, "infos": infos}, path)

    def load(self, path, load_optimizer=True):
        loaded = torch.load(path, map_location=self.device, weights_only=True)
        self.alg.actor_critic.load_state_dict(loaded["model_state_dict"])
        if getattr(self.alg, "_fused", None) is not None:  # bf16 weight copies of the native rollout
            self.alg._fused.weights_changed = True
        if load_optimizer:
            self.alg.optimizer.load_state_dict(loaded["optimizer_state_dict"])
            # a captured autograd update reads the previous Adam state tensors: recapture
            if getattr(self.alg, "_graph", None) is not None:
                self.alg._graph = None
        self.current_learning_iteration = loaded["iter"]
        return loaded["infos"]

    def get_inference_policy(self, device=None):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.act_inference
