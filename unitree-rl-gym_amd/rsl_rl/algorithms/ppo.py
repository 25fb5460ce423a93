"""PPO with clipped surrogate / clipped value loss / adaptive-KL learning rate
(rsl_rl v1.0.2 semantics).

ROCm-specific changes that do not change the maths:
* the adaptive learning rate lives in a device tensor consumed by Adam, so the
  KL test costs no host sync per mini-batch (the reference does 1 + 2 .item()s);
* losses are accumulated on the device and read once per update;
* with torch.distributed initialised (one process per GPU, RCCL), the gradient
  is flattened into ONE bucket and all-reduced (mean) per optimizer step, the
  mini-batch KL is averaged across ranks before the LR decision, and advantages
  are normalised with global statistics — so N ranks behave like one batch of
  N x num_envs envs.
"""
import os
import warnings

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim

from rsl_rl.algorithms import fused_recurrent, fused_step
from rsl_rl.modules import ActorCritic
from rsl_rl.modules import mfma_mlp
from rsl_rl.storage import RolloutStorage
from rsl_rl.storage.rollout_storage import minibatch_permutation


def _dist_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


class PPO:
    actor_critic: ActorCritic

    def __init__(self, actor_critic, num_learning_epochs=1, num_mini_batches=1, clip_param=0.2, gamma=0.998, lam=0.95,
                 value_loss_coef=1.0, entropy_coef=0.0, learning_rate=1e-3, max_grad_norm=1.0,
                 use_clipped_value_loss=True, schedule="fixed", desired_kl=0.01, device="cpu", fused_loss=True):
        self.device = device
        self.desired_kl = desired_kl
        self.schedule = schedule
        self.actor_critic = actor_critic
        self.actor_critic.to(self.device)
        self.storage = None
        self._lr = torch.tensor(float(learning_rate), device=self.device)
        params = list(self.actor_critic.parameters())
        on_gpu = str(self.device).startswith("cuda")
        self.optimizer = None
        if on_gpu:
            for kw in (dict(fused=True, capturable=True), dict(foreach=True, capturable=True)):
                try:
                    self.optimizer = optim.Adam(params, lr=self._lr, **kw)
                    break
                except (RuntimeError, TypeError, ValueError):
                    continue
        if self.optimizer is None:
            self.optimizer = optim.Adam(params, lr=float(learning_rate))
        self._lr_is_tensor = torch.is_tensor(self.optimizer.param_groups[0]["lr"])
        self.transition = RolloutStorage.Transition()
        self.clip_param = clip_param
        self.num_learning_epochs = num_learning_epochs
        self.num_mini_batches = num_mini_batches
        self.value_loss_coef = value_loss_coef
        self.entropy_coef = entropy_coef
        self.gamma = gamma
        self.lam = lam
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.world_size = _dist_world()
        # whole-update HIP graph (MLP policies on a GPU): set use_graph=False to disable
        # (library bf16 GEMMs under autocast drift inside a captured graph on this ROCm;
        #  the MFMA MLP kernels are deterministic and capture cleanly)
        # recurrent policies train in the dense form (storage.recurrent_dense_mini_batch_generator,
        # modules/lstm_seq.py): fixed shapes and no host sync, so their update captures too.
        # The dense form covers one-layer LSTMs; a GRU (or a deeper LSTM) keeps rsl_rl's
        # padded-trajectory generator and the eager update.
        self._dense_recurrent = getattr(self.actor_critic, "is_recurrent", False) and \
            hasattr(self.actor_critic, "act_dense") and \
            all(isinstance(getattr(getattr(self.actor_critic, m, None), "rnn", None), nn.LSTM) and
                getattr(self.actor_critic, m).rnn.num_layers == 1 for m in ("memory_a", "memory_c"))
        self.use_graph = on_gpu and (not getattr(self.actor_critic, "is_recurrent", False) or
                                     self._dense_recurrent) and \
            self.optimizer.defaults.get("capturable", False) and \
            (self.world_size == 1 or (dist.get_backend() == "nccl" and
                                      os.environ.get("PPO_CAPTURE_COLLECTIVES", "1") != "0"))
        self._graph = None
        # fused PPO-loss kernels for the Gaussian MLP policy on a GPU (fused_loss=False:
        # the torch statement of the loss, _reference_loss)
        self._fused_loss = bool(fused_loss) and on_gpu and hasattr(self.actor_critic, "mean_and_value")
        self._fused = None  # FusedPPOStep, built with the storage (init_storage)
        self._rfused = None  # FusedRecurrentStep (recurrent policies), likewise
        self._rgraph = None
        self._rollout = None  # FusedRollout: act/process_env_step of the same policy
        self._stored_t = None  # storage row the fused act() filled, awaiting process_env_step
        self._fgraph = None
        self._diag, self._diag_i = None, 0
        self._graph_calls = 0
        self._capturing = False
        self._gflat = None  # world > 1: the gradient bucket (_grad_bucket)
        if self.world_size > 1:
            for p in params:  # identical initial policy on every rank
                dist.broadcast(p.data, src=0)

    # learning_rate is read by the runner's logger (rsl_rl attribute)
    @property
    def learning_rate(self):
        return float(self._lr)

    @learning_rate.setter
    def learning_rate(self, v):
        self._lr.fill_(float(v))
        if not self._lr_is_tensor:
            for g in self.optimizer.param_groups:
                g["lr"] = float(v)

    def init_storage(self, num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape, action_shape):
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape,
                                      action_shape, self.device)
        batch = num_envs * num_transitions_per_env
        if self._fused_loss and not self.actor_critic.is_recurrent and self._fused is None and \
                getattr(self.actor_critic, "mixed_precision", False) and batch % self.num_mini_batches == 0:
            try:  # whole optimizer step in ~20 launches (algorithms/fused_step.py)
                self._fused = fused_step.FusedPPOStep(self, batch // self.num_mini_batches)
                self._rollout = fused_step.FusedRollout(self._fused, num_envs) if num_envs % 8 == 0 else None
            except ValueError:
                self._fused = self._rollout = None
        if self._fused_loss and self._dense_recurrent and self._rfused is None and \
                fused_recurrent.supported(self.actor_critic, num_envs, self.num_mini_batches):
            # the recurrent optimizer step without autograd (algorithms/fused_recurrent.py)
            try:
                self._rfused = fused_recurrent.FusedRecurrentStep(self, num_envs, num_transitions_per_env)
            except ValueError:  # a shape the kernels do not take: the autograd update runs
                self._rfused = None
        if self.actor_critic.is_recurrent and self._rollout is None and str(self.device).startswith("cuda") and \
                hasattr(self.actor_critic, "rollout_capturable"):
            self._rollout = fused_step.RecurrentRollout(self, num_envs)

    def test_mode(self):
        self.actor_critic.eval()

    def train_mode(self):
        self.actor_critic.train()

    def act(self, obs, critic_obs):
        ro, st = self._rollout, self.storage
        if ro is not None and ro.usable(obs, critic_obs, st):
            # forward, sample, log-prob and the storage row in 6 launches (FusedRollout)
            t = st.step
            if t >= st.num_transitions_per_env:
                raise AssertionError("Rollout buffer overflow")
            actions = ro.act(obs, critic_obs, st, t)
            tr = self.transition
            tr.actions, tr.values, tr.actions_log_prob = st.actions[t], st.values[t], st.actions_log_prob[t]
            tr.action_mean, tr.action_sigma = st.mu[t], st.sigma[t]
            tr.observations, tr.critic_observations = obs, critic_obs
            tr.hidden_states = None
            self._stored_t = t
            return actions
        # a store deferred by an earlier fused act goes out now: it holds the env's reward /
        # done buffers, which the next env.step overwrites
        self.flush_rollout()
        if self.actor_critic.is_recurrent:
            # the state BEFORE this step, copied into the storage slot now: on the GPU the
            # memory updates its state buffers in place during act()
            self.storage._save_hidden_states(self.actor_critic.get_hidden_states())
            self.transition.hidden_states = None
        if not self.actor_critic.is_recurrent and hasattr(self.actor_critic, "act_and_value"):  # shared launches
            actions, values = self.actor_critic.act_and_value(obs, critic_obs)
            self.transition.actions, self.transition.values = actions.detach(), values.detach()
        else:
            self.transition.actions = self.actor_critic.act(obs).detach()
            self.transition.values = self.actor_critic.evaluate(critic_obs).detach()
        self.transition.actions_log_prob = self.actor_critic.get_actions_log_prob(self.transition.actions).detach()
        self.transition.action_mean = self.actor_critic.action_mean.detach()
        self.transition.action_sigma = self.actor_critic.action_std.detach()
        self.transition.observations = obs
        self.transition.critic_observations = critic_obs
        return self.transition.actions

    def process_env_step(self, rewards, dones, infos):
        t, self._stored_t = self._stored_t, None
        time_outs = infos["time_outs"] if "time_outs" in infos else None
        # the env step's extras, when the env left them to this consumer (LeggedRobot.step,
        # defer_extras): the fused store does them in its launch, any other path first
        job = infos.get("_deferred_extras") if isinstance(infos, dict) else None
        if t is not None and t == self.storage.step and \
                fused_step.FusedRollout.storable(rewards, dones, time_outs, self.storage.num_envs):
            reset_done = self._rollout.store(rewards, dones, time_outs, self.storage, t, self.gamma, job)
            self.storage.step += 1
            self.transition.clear()
            if not reset_done:  # (the recurrent store launch zeroes the done envs' memories itself)
                self.actor_critic.reset(dones)
            return
        if t is not None and isinstance(self._rollout, fused_step.RecurrentRollout):
            # the act sampled with the draw counter the skipped store launch would advance
            self._rollout.draw += 1
        if job is not None:
            job.run()
        self.transition.rewards = rewards.clone()
        self.transition.dones = dones
        if "time_outs" in infos:  # bootstrap on time-outs
            self.transition.rewards += self.gamma * torch.squeeze(
                self.transition.values * infos["time_outs"].unsqueeze(1).to(self.device), 1)
        self.storage.add_transitions(self.transition)
        self.transition.clear()
        self.actor_critic.reset(dones)

    def _global_adv_stats(self, adv):
        n = torch.tensor(float(adv.numel()), device=adv.device)
        s = torch.stack([adv.sum(), (adv * adv).sum(), n])
        dist.all_reduce(s)
        mean = s[0] / s[2]
        var = (s[1] - s[2] * mean * mean) / (s[2] - 1.0)
        return mean, torch.sqrt(var.clamp(min=0.0))

    def flush_rollout(self):
        """The fused rollout's deferred process_env_step, before anything reads the storage."""
        if self._rollout is not None and hasattr(self._rollout, "flush"):
            self._rollout.flush(self.storage)

    def compute_returns(self, last_critic_obs):
        self.flush_rollout()
        last_values = None
        if isinstance(self._rollout, fused_step.FusedRollout):  # one launch instead of the layer GEMMs
            last_values = self._rollout.values(last_critic_obs)
        if last_values is None:
            last_values = self.actor_critic.evaluate(last_critic_obs).detach()
        if self._fused is not None or (str(self.device).startswith("cuda") and last_values.is_cuda):
            # GAE + normalisation: two launches (+ a moments all-reduce across ranks)
            fused_step.gae(self.storage, last_values, self.gamma, self.lam, self.world_size)
            return
        stats = self._global_adv_stats if self.world_size > 1 else None
        self.storage.compute_returns(last_values, self.gamma, self.lam, adv_stats=stats)

    def _grad_bucket(self):
        """world > 1: ONE flat buffer whose views are every parameter's .grad, plus a
        one-float tail for the mini-batch KL.  backward() accumulates into the views in
        place, so the optimizer step's single all-reduce covers the gradient and the KL
        that drives the adaptive learning rate (no cat/copy-back, no second collective)."""
        params = list(self.actor_critic.parameters())
        if self._gflat is None:
            self._gflat = torch.zeros(sum(p.numel() for p in params) + 1, device=self.device)
            off = 0
            self._gviews = []
            for p in params:
                self._gviews.append(self._gflat[off:off + p.numel()].view_as(p))
                off += p.numel()
        for p, v in zip(params, self._gviews):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v
        return self._gflat

    def _allreduce_grads(self, kl=None):
        """Mean of the gradients over the ranks in one all-reduce.  kl (a 0-d tensor, this
        rank's mini-batch KL) rides in the same bucket; returns the ranks' mean KL."""
        params = [p for p in self.actor_critic.parameters() if p.grad is not None]
        b = self._gflat
        if b is not None and len(params) == len(self._gviews) and \
                all(p.grad.data_ptr() == v.data_ptr() for p, v in zip(params, self._gviews)):
            if kl is not None:
                b[-1:].copy_(kl.reshape(1))
            dist.all_reduce(b)
            b.div_(self.world_size)
            return b[-1] if kl is not None else None
        # gradients that are not bucket views (a caller's own backward): cat, reduce, copy back
        grads = [p.grad for p in params]
        flat = torch.cat([g.reshape(-1) for g in grads] + ([kl.reshape(1)] if kl is not None else []))
        dist.all_reduce(flat)
        flat /= self.world_size
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n
        return flat[-1] if kl is not None else None

    def _reference_loss(self, obs_batch, critic_obs_batch, actions_batch, target_values_batch, advantages_batch,
                        returns_batch, old_actions_log_prob_batch, old_mu_batch, old_sigma_batch, hid_states_batch,
                        masks_batch):
        """The loss exactly as rsl_rl v1.0.2 PPO.update states it (torch ops).  Recurrent
        policies in the dense form (masks_batch is the [T, envs] reset mask of
        recurrent_dense_mini_batch_generator): every [T, envs, .] tensor is flattened to
        T*envs rows, the rows the padded form's unpad_trajectories produces."""
        if self.actor_critic.is_recurrent and self._dense_recurrent:
            ac = self.actor_critic
            ac.act_dense(obs_batch, hid_states_batch[0], masks_batch)
            value_batch = ac.evaluate_dense(critic_obs_batch, hid_states_batch[1], masks_batch)
            flat = lambda t: t.reshape(-1, t.shape[-1])  # noqa: E731
            actions_batch, target_values_batch, advantages_batch = (flat(actions_batch), flat(target_values_batch),
                                                                     flat(advantages_batch))
            returns_batch, old_actions_log_prob_batch = flat(returns_batch), flat(old_actions_log_prob_batch)
            old_mu_batch, old_sigma_batch = flat(old_mu_batch), flat(old_sigma_batch)
            actions_log_prob_batch = ac.get_actions_log_prob(actions_batch)
        else:
            if self.actor_critic.is_recurrent:
                self.actor_critic.act(obs_batch, masks=masks_batch, hidden_states=hid_states_batch[0])
            else:  # v1.0.2 calls act() here and discards the sample; only the distribution is used
                self.actor_critic.update_distribution(obs_batch)
            actions_log_prob_batch = self.actor_critic.get_actions_log_prob(actions_batch)
            value_batch = self.actor_critic.evaluate(critic_obs_batch, masks=masks_batch,
                                                     hidden_states=hid_states_batch[1])
        mu_batch = self.actor_critic.action_mean
        sigma_batch = self.actor_critic.action_std
        entropy_batch = self.actor_critic.entropy

        self._kl_mean = None  # the adaptive-LR input; _minibatch_step applies it
        if self.desired_kl is not None and self.schedule == "adaptive":
            with torch.no_grad():
                kl = torch.sum(torch.log(sigma_batch / old_sigma_batch + 1.0e-5)
                               + (torch.square(old_sigma_batch) + torch.square(old_mu_batch - mu_batch))
                               / (2.0 * torch.square(sigma_batch)) - 0.5, axis=-1)
                self._kl_mean = torch.mean(kl)

        ratio = torch.exp(actions_log_prob_batch - torch.squeeze(old_actions_log_prob_batch))
        surrogate = -torch.squeeze(advantages_batch) * ratio
        surrogate_clipped = -torch.squeeze(advantages_batch) * torch.clamp(ratio, 1.0 - self.clip_param,
                                                                           1.0 + self.clip_param)
        surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
        if self.use_clipped_value_loss:
            value_clipped = target_values_batch + (value_batch - target_values_batch).clamp(-self.clip_param,
                                                                                            self.clip_param)
            value_losses = (value_batch - returns_batch).pow(2)
            value_losses_clipped = (value_clipped - returns_batch).pow(2)
            value_loss = torch.max(value_losses, value_losses_clipped).mean()
        else:
            value_loss = (returns_batch - value_batch).pow(2).mean()
        loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_batch.mean()
        return loss, surrogate_loss, value_loss

    def _adapt_lr(self, kl_mean):
        """KL-adaptive learning rate (rsl_rl v1.0.2), on device: no host sync.  kl_mean is
        already the ranks' mean at world > 1 (it rides in the gradient bucket)."""
        with torch.no_grad():
            lr = self._lr
            new_lr = torch.where(kl_mean > self.desired_kl * 2.0, torch.clamp(lr / 1.5, min=1e-5),
                                 torch.where((kl_mean < self.desired_kl / 2.0) & (kl_mean > 0.0),
                                             torch.clamp(lr * 1.5, max=1e-2), lr))
            self._lr.copy_(new_lr)
        if not self._lr_is_tensor:
            for g in self.optimizer.param_groups:
                g["lr"] = float(self._lr)

    def _minibatch_step(self, obs_batch, critic_obs_batch, actions_batch, target_values_batch, advantages_batch,
                        returns_batch, old_actions_log_prob_batch, old_mu_batch, old_sigma_batch, hid_states_batch,
                        masks_batch, acc):
        """One PPO optimizer step on one mini-batch (rsl_rl v1.0.2 PPO.update body)."""
        recurrent = self.actor_critic.is_recurrent
        if self._fused_loss and (not recurrent or self._dense_recurrent):
            # same loss, two fused kernels forward + two backward (modules/mfma_mlp.ppo_loss)
            if recurrent:  # dense form: every [T, envs, .] tensor flattened to T*envs rows
                mu_batch, value_batch = self.actor_critic.mean_and_value_dense(obs_batch, critic_obs_batch,
                                                                               hid_states_batch, masks_batch)
                flat = lambda t: t.reshape(-1, t.shape[-1])  # noqa: E731
                (actions_batch, target_values_batch, advantages_batch, returns_batch, old_actions_log_prob_batch,
                 old_mu_batch, old_sigma_batch) = map(flat, (actions_batch, target_values_batch, advantages_batch,
                                                             returns_batch, old_actions_log_prob_batch,
                                                             old_mu_batch, old_sigma_batch))
            else:
                mu_batch, value_batch = self.actor_critic.mean_and_value(obs_batch, critic_obs_batch)
            loss, stats = mfma_mlp.ppo_loss(mu_batch, self.actor_critic.std, value_batch, actions_batch,
                                            old_actions_log_prob_batch, old_mu_batch, old_sigma_batch,
                                            advantages_batch, returns_batch, target_values_batch, self.clip_param,
                                            self.use_clipped_value_loss, self.value_loss_coef, self.entropy_coef)
            surrogate_loss, value_loss = stats[0], stats[1]
            adaptive = self.desired_kl is not None and self.schedule == "adaptive"
            kl_mean = None
            if self.world_size == 1 and self._lr_is_tensor and self._diag is None:
                # the logged losses and the adaptive LR in one launch (pmlp_loss_bookkeeping)
                mfma_mlp._ok(mfma_mlp.load().pmlp_loss_bookkeeping(
                    mfma_mlp._p(stats), mfma_mlp._p(self._lr), mfma_mlp._p(acc),
                    float(self.desired_kl) if adaptive else 0.0, int(adaptive), mfma_mlp._stream()),
                    "pmlp_loss_bookkeeping")
                acc = None
            elif adaptive:
                kl_mean = stats[2]
        else:
            loss, surrogate_loss, value_loss = self._reference_loss(
                obs_batch, critic_obs_batch, actions_batch, target_values_batch, advantages_batch, returns_batch,
                old_actions_log_prob_batch, old_mu_batch, old_sigma_batch, hid_states_batch, masks_batch)
            kl_mean = self._kl_mean

        if self.world_size == 1:
            if kl_mean is not None:  # before this step's Adam, as rsl_rl adapts it
                self._adapt_lr(kl_mean)
            # set_to_none: backward then hands its fresh gradient buffers to .grad (no
            # zero-fill + accumulate kernels); inside the captured update these are
            # graph-pool buffers at fixed addresses, which the captured Adam step reads
            self.optimizer.zero_grad(set_to_none=True)
            loss.backward()
        else:
            # data-parallel: backward accumulates into the views of one bucket, whose
            # single all-reduce also carries the KL; the LR then adapts to the ranks' mean
            # KL, still before this step's Adam
            self._grad_bucket().zero_()
            loss.backward()
            kl_mean = self._allreduce_grads(kl_mean)
            if kl_mean is not None:
                self._adapt_lr(kl_mean)
        nn.utils.clip_grad_norm_(self.actor_critic.parameters(), self.max_grad_norm)
        self.optimizer.step()
        with torch.no_grad():
            if acc is not None:
                acc[0] += value_loss.detach()
                acc[1] += surrogate_loss.detach()
            if self._diag is not None:  # debugging aid: per-step losses (also inside a captured graph)
                row = self._diag[self._diag_i % self._diag.shape[0]]
                row[:2].copy_(torch.stack([value_loss.detach(), surrogate_loss.detach()]))
                self._diag_i += 1
        # Release this step's autograd graph.  A distribution kept alive on the
        # module pins the parameters' AccumulateGrad nodes from the stream they were
        # created on; a later capture on another stream then syncs against that
        # stream and the captured update is no longer self-contained (replays race).
        self.actor_critic.distribution = None

    def update(self, host_means=True):
        """The PPO update; returns (mean value loss, mean surrogate loss) as Python floats (a
        device read-back, as the reference's per-mini-batch .item()), or with host_means=False
        the device tensor of the two means, so a caller that does not read them (the runner
        without logging) keeps the host ahead of the device."""
        self.flush_rollout()
        num_updates = self.num_learning_epochs * self.num_mini_batches
        self._graph_calls += 1
        if self._fused is not None:
            acc = self._update_fused()
        elif self._rfused is not None:
            acc = self._update_rfused()
        elif self.use_graph and self._graph_calls >= 2:  # first call runs eagerly (warm-up)
            acc = self._update_graphed()
        else:
            acc = torch.zeros(2, device=self.device)
            if self.actor_critic.is_recurrent and self._dense_recurrent:
                gen = self.storage.recurrent_dense_mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
            elif self.actor_critic.is_recurrent:
                gen = self.storage.reccurent_mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
            else:
                gen = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
            for batch in gen:
                self._minibatch_step(*batch, acc)
        means = acc / num_updates
        self.storage.clear()
        if not host_means:
            return means
        means = means.tolist()
        return means[0], means[1]

    def _update_fused(self):
        """num_epochs x num_mini_batches fused optimizer steps (FusedPPOStep.run), replayed
        as one HIP graph from the second call on.  Same permutation rule as
        RolloutStorage.mini_batch_generator: one randperm per update, reused every epoch."""
        f, st = self._fused, self.storage
        f.sync_optimizer_state(self.optimizer)
        f.ensure_weights()  # the captured steps read the bf16 weight copies from the first one
        mb = f.M
        if self._fgraph is None and not hasattr(self, "_fperm"):
            self._fperm = torch.empty(self.num_mini_batches * mb, dtype=torch.int64, device=self.device)
            self._facc = torch.zeros(2, device=self.device)
            cobs = st.privileged_observations if st.privileged_observations is not None else st.observations
            self._fsrc = (st.observations.flatten(0, 1), cobs.flatten(0, 1) if cobs is not st.observations
                          else st.observations.flatten(0, 1), st.actions.flatten(0, 1), st.values.flatten(0, 1),
                          st.advantages.flatten(0, 1), st.returns.flatten(0, 1), st.actions_log_prob.flatten(0, 1),
                          st.mu.flatten(0, 1), st.sigma.flatten(0, 1))
            if st.privileged_observations is None:  # the critic reads the actor's observations
                self._fsrc = (self._fsrc[0], self._fsrc[0]) + self._fsrc[2:]
            self._fadv = st.advantages
        if st.advantages.data_ptr() != self._fadv.data_ptr():
            self._fadv.copy_(st.advantages)
            st.advantages = self._fadv
        mfma_mlp.permutation_(self._fperm)  # as minibatch_permutation (no device sort)

        def body():
            self._facc.zero_()
            for _ in range(self.num_learning_epochs):
                for i in range(self.num_mini_batches):
                    f.run(self._fperm[i * mb:(i + 1) * mb], self._fsrc, self._facc)

        if not (self.use_graph and self._graph_calls >= 2):
            body()
            return self._facc
        if self._fgraph is None:
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            graph = torch.cuda.CUDAGraph()
            if not self._capture(graph, side, body):
                body()
                return self._facc
            torch.cuda.current_stream(self.device).wait_stream(side)
            self._fgraph = graph
        self._fgraph.replay()
        return self._facc

    def _update_rfused(self):
        """The recurrent update as num_epochs x num_mini_batches FusedRecurrentStep.run calls
        over the dense mini-batches (contiguous env slices, as rsl_rl's recurrent generator),
        replayed as one HIP graph from the second call on."""
        rf, st = self._rfused, self.storage
        rf.sync_optimizer_state(self.optimizer)
        if not hasattr(self, "_racc"):
            self._racc = torch.zeros(2, device=self.device)
            self._radv = st.advantages
        if st.advantages.data_ptr() != self._radv.data_ptr():  # the captured graph reads this buffer
            self._radv.copy_(st.advantages)
            st.advantages = self._radv

        def body():
            self._racc.zero_()
            for batch in st.recurrent_dense_mini_batch_generator(self.num_mini_batches, self.num_learning_epochs):
                rf.run(batch, self._racc)

        if not (self.use_graph and self._graph_calls >= 2):
            body()
            return self._racc
        if self._rgraph is None:
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            graph = torch.cuda.CUDAGraph()
            if not self._capture(graph, side, body):
                body()
                return self._racc
            torch.cuda.current_stream(self.device).wait_stream(side)
            self._rgraph = graph
        self._rgraph.replay()
        return self._racc

    def _capture(self, graph, stream, body):
        """Record body() into graph on stream.  A capture that fails (e.g. a collective
        library that refuses capture of the data-parallel update's all-reduce) must not
        end the run: nothing inside a failed capture has executed, so the update runs
        eagerly from then on.  At world > 1 the ranks decide together (an all-reduce of
        the failure flag after the attempt), so no rank replays a graph while another
        runs the same collectives eagerly.  Returns True when the graph is usable."""
        err = None
        try:
            with torch.cuda.graph(graph, stream=stream):
                body()
        except RuntimeError as e:
            err = e
        failed = self._any_rank(err is not None)
        if failed:
            warnings.warn(f"PPO: capturing the update failed ({err or 'on another rank'}); updating eagerly")
            torch.cuda.synchronize(self.device)
            self.use_graph = False
        return not failed

    def _any_rank(self, flag):
        """True on every rank when flag is True on any rank (one all-reduce at world > 1)."""
        if self.world_size == 1:
            return bool(flag)
        t = torch.tensor([1.0 if flag else 0.0], device=self.device)
        dist.all_reduce(t)
        return bool(t.item() > 0)

    def _update_graphed(self):
        """All num_epochs x num_mini_batches optimizer steps replayed as ONE HIP graph.
        The mini-batch permutation is drawn outside the graph each update, exactly as
        RolloutStorage.mini_batch_generator draws it (one randperm per update)."""
        st = self.storage
        batch = st.num_envs * st.num_transitions_per_env
        mb = batch // self.num_mini_batches
        if self._graph is None:
            self._perm = None if self._dense_recurrent else \
                minibatch_permutation(self.num_mini_batches * mb, self.device)
            self._acc = torch.zeros(2, device=self.device)
            flat = [st.observations.flatten(0, 1),
                    st.privileged_observations.flatten(0, 1) if st.privileged_observations is not None
                    else st.observations.flatten(0, 1),
                    st.actions.flatten(0, 1), st.values.flatten(0, 1), None, st.returns.flatten(0, 1),
                    st.actions_log_prob.flatten(0, 1), st.mu.flatten(0, 1), st.sigma.flatten(0, 1)]
            self._flat = flat

            def body():
                self._acc.zero_()
                if self._dense_recurrent:  # contiguous env slices, no permutation (rsl_rl recurrent)
                    for batch in st.recurrent_dense_mini_batch_generator(self.num_mini_batches,
                                                                         self.num_learning_epochs):
                        self._minibatch_step(*batch, self._acc)
                    return
                adv = st.advantages.flatten(0, 1)
                for _ in range(self.num_learning_epochs):
                    for i in range(self.num_mini_batches):
                        idx = self._perm[i * mb:(i + 1) * mb]
                        tens = [None if t is None else t.index_select(0, idx) for t in flat]
                        tens[4] = adv.index_select(0, idx)
                        self._minibatch_step(*tens, (None, None), None, self._acc)

            self._side = torch.cuda.Stream(self.device)
            self._side.wait_stream(torch.cuda.current_stream(self.device))
            self._graph = torch.cuda.CUDAGraph()
            self._adv_static = st.advantages
            # snapshot: the warm-up pass below really trains, so undo it afterwards
            snap_p = [p_.detach().clone() for p_ in self.actor_critic.parameters()]
            snap_o = {id(p_): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.optimizer.state[p_].items()}
                      for p_ in self.actor_critic.parameters()}
            snap_lr = self._lr.clone()
            self._capturing = True
            with torch.cuda.stream(self._side):
                body()  # warm-up on the capture stream (allocator + autograd state)
                captured = self._capture(self._graph, self._side, body)
            self._capturing = False
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            with torch.no_grad():
                for p_, v in zip(self.actor_critic.parameters(), snap_p):
                    p_.copy_(v)
                for p_ in self.actor_critic.parameters():
                    for k, v in self.optimizer.state[p_].items():
                        if torch.is_tensor(v):
                            v.copy_(snap_o[id(p_)][k])
                self._lr.copy_(snap_lr)
            if not captured:
                self._graph = None
                body()
                return self._acc
        if st.advantages.data_ptr() != self._adv_static.data_ptr():
            self._adv_static.copy_(st.advantages)
            st.advantages = self._adv_static
        if not self._dense_recurrent:  # one randperm per update (mini_batch_generator's rule)
            self._perm.copy_(minibatch_permutation(self.num_mini_batches * mb, self.device))
        self._graph.replay()
        return self._acc
