import torch

from rsl_rl.utils import split_and_pad_trajectories


def minibatch_permutation(n, device):
    """The mini-batch permutation (rsl_rl v1.0.2: torch.randperm(n, device=device)).  On the
    GPU it is pmlp_permutation's keyed Feistel permutation (no device sort: ~10 instead of
    ~60 us per update), keyed from torch's seeded CPU generator, so the generic and the
    fused update draw the same permutation for the same seed; on the CPU torch.randperm."""
    if torch.device(device).type != "cuda":
        return torch.randperm(n, requires_grad=False, device=device)
    from rsl_rl.modules import mfma_mlp
    return mfma_mlp.permutation_(torch.empty(n, dtype=torch.int64, device=device))


class RolloutStorage:
    """[T, N, ...] rollout buffers + GAE + mini-batch generators (rsl_rl v1.0.2)."""

    class Transition:
        def __init__(self):
            self.observations = None
            self.critic_observations = None
            self.actions = None
            self.rewards = None
            self.dones = None
            self.values = None
            self.actions_log_prob = None
            self.action_mean = None
            self.action_sigma = None
            self.hidden_states = None

        def clear(self):
            self.__init__()

    def __init__(self, num_envs, num_transitions_per_env, obs_shape, privileged_obs_shape, actions_shape, device="cpu"):
        self.device = device
        self.obs_shape = obs_shape
        self.privileged_obs_shape = privileged_obs_shape
        self.actions_shape = actions_shape
        T, N = num_transitions_per_env, num_envs
        self.observations = torch.zeros(T, N, *obs_shape, device=device)
        if privileged_obs_shape[0] is not None:
            self.privileged_observations = torch.zeros(T, N, *privileged_obs_shape, device=device)
        else:
            self.privileged_observations = None
        self.rewards = torch.zeros(T, N, 1, device=device)
        self.actions = torch.zeros(T, N, *actions_shape, device=device)
        self.dones = torch.zeros(T, N, 1, device=device).byte()
        self.actions_log_prob = torch.zeros(T, N, 1, device=device)
        self.values = torch.zeros(T, N, 1, device=device)
        self.returns = torch.zeros(T, N, 1, device=device)
        self.advantages = torch.zeros(T, N, 1, device=device)
        self.mu = torch.zeros(T, N, *actions_shape, device=device)
        self.sigma = torch.zeros(T, N, *actions_shape, device=device)
        self.num_transitions_per_env = T
        self.num_envs = N
        self.saved_hidden_states_a = None
        self.saved_hidden_states_c = None
        self.step = 0

    def add_transitions(self, transition: Transition):
        if self.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        self.observations[self.step].copy_(transition.observations)
        if self.privileged_observations is not None:
            self.privileged_observations[self.step].copy_(transition.critic_observations)
        self.actions[self.step].copy_(transition.actions)
        self.rewards[self.step].copy_(transition.rewards.view(-1, 1))
        self.dones[self.step].copy_(transition.dones.view(-1, 1))
        self.values[self.step].copy_(transition.values)
        self.actions_log_prob[self.step].copy_(transition.actions_log_prob.view(-1, 1))
        self.mu[self.step].copy_(transition.action_mean)
        self.sigma[self.step].copy_(transition.action_sigma)
        self._save_hidden_states(transition.hidden_states)
        self.step += 1

    def _save_hidden_states(self, hidden_states):
        if hidden_states is None or hidden_states == (None, None):
            return
        hid_a = hidden_states[0] if isinstance(hidden_states[0], tuple) else (hidden_states[0],)
        hid_c = hidden_states[1] if isinstance(hidden_states[1], tuple) else (hidden_states[1],)
        if self.saved_hidden_states_a is None:
            # ordinary (not inference-mode) tensors: the update saves slices of them for backward
            with torch.inference_mode(False):
                self.saved_hidden_states_a = [torch.zeros(self.observations.shape[0], *h.shape, device=self.device)
                                              for h in hid_a]
                self.saved_hidden_states_c = [torch.zeros(self.observations.shape[0], *h.shape, device=self.device)
                                              for h in hid_c]
        for i in range(len(hid_a)):
            self.saved_hidden_states_a[i][self.step].copy_(hid_a[i])
            self.saved_hidden_states_c[i][self.step].copy_(hid_c[i])

    def hidden_state_slots(self, t, shapes_a, shapes_c):
        """The storage slots of step t for the saved (h, c) of both memories (the buffers
        are created as zeros on first use, as _save_hidden_states creates them)."""
        if self.saved_hidden_states_a is None:
            with torch.inference_mode(False):
                T = self.observations.shape[0]
                self.saved_hidden_states_a = [torch.zeros(T, *s, device=self.device) for s in shapes_a]
                self.saved_hidden_states_c = [torch.zeros(T, *s, device=self.device) for s in shapes_c]
        return [h[t] for h in self.saved_hidden_states_a], [h[t] for h in self.saved_hidden_states_c]

    def clear(self):
        self.step = 0

    def compute_returns(self, last_values, gamma, lam, adv_stats=None):
        """GAE(gamma, lam) backwards over T, then advantage normalisation.

        ``adv_stats`` (optional) maps the local advantages to a global (mean, std)
        so data-parallel ranks normalise identically to one big batch."""
        advantage = 0
        for step in reversed(range(self.num_transitions_per_env)):
            next_values = last_values if step == self.num_transitions_per_env - 1 else self.values[step + 1]
            not_terminal = 1.0 - self.dones[step].float()
            delta = self.rewards[step] + not_terminal * gamma * next_values - self.values[step]
            advantage = delta + not_terminal * gamma * lam * advantage
            self.returns[step] = advantage + self.values[step]
        # in place: a captured update graph reads this buffer
        torch.sub(self.returns, self.values, out=self.advantages)
        if adv_stats is None:
            mean, std = self.advantages.mean(), self.advantages.std()
        else:
            mean, std = adv_stats(self.advantages)
        self.advantages.sub_(mean).div_(std + 1e-8)

    def get_statistics(self):
        done = self.dones
        done[-1] = 1
        flat_dones = done.permute(1, 0, 2).reshape(-1, 1)
        done_indices = torch.cat((flat_dones.new_tensor([-1], dtype=torch.int64), flat_dones.nonzero(as_tuple=False)[:, 0]))
        trajectory_lengths = done_indices[1:] - done_indices[:-1]
        return trajectory_lengths.float().mean(), self.rewards.mean()

    def mini_batch_generator(self, num_mini_batches, num_epochs=8):
        batch_size = self.num_envs * self.num_transitions_per_env
        mini_batch_size = batch_size // num_mini_batches
        indices = minibatch_permutation(num_mini_batches * mini_batch_size, self.device)
        observations = self.observations.flatten(0, 1)
        critic_observations = self.privileged_observations.flatten(0, 1) if self.privileged_observations is not None else observations
        actions = self.actions.flatten(0, 1)
        values = self.values.flatten(0, 1)
        returns = self.returns.flatten(0, 1)
        old_actions_log_prob = self.actions_log_prob.flatten(0, 1)
        advantages = self.advantages.flatten(0, 1)
        old_mu = self.mu.flatten(0, 1)
        old_sigma = self.sigma.flatten(0, 1)
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                idx = indices[i * mini_batch_size:(i + 1) * mini_batch_size]
                yield (observations[idx], critic_observations[idx], actions[idx], values[idx], advantages[idx],
                       returns[idx], old_actions_log_prob[idx], old_mu[idx], old_sigma[idx], (None, None), None)

    def reccurent_mini_batch_generator(self, num_mini_batches, num_epochs=8):
        padded_obs, traj_masks = split_and_pad_trajectories(self.observations, self.dones)
        if self.privileged_observations is not None:
            padded_critic_obs, _ = split_and_pad_trajectories(self.privileged_observations, self.dones)
        else:
            padded_critic_obs = padded_obs
        mini_batch_size = self.num_envs // num_mini_batches
        for _ in range(num_epochs):
            first_traj = 0
            for i in range(num_mini_batches):
                start, stop = i * mini_batch_size, (i + 1) * mini_batch_size
                dones = self.dones.squeeze(-1)
                last_was_done = torch.zeros_like(dones, dtype=torch.bool)
                last_was_done[1:] = dones[:-1]
                last_was_done[0] = True
                trajectories_batch_size = int(torch.sum(last_was_done[:, start:stop]))
                last_traj = first_traj + trajectories_batch_size
                masks_batch = traj_masks[:, first_traj:last_traj]
                obs_batch = padded_obs[:, first_traj:last_traj]
                critic_obs_batch = padded_critic_obs[:, first_traj:last_traj]
                actions_batch = self.actions[:, start:stop]
                old_mu_batch = self.mu[:, start:stop]
                old_sigma_batch = self.sigma[:, start:stop]
                returns_batch = self.returns[:, start:stop]
                advantages_batch = self.advantages[:, start:stop]
                values_batch = self.values[:, start:stop]
                old_actions_log_prob_batch = self.actions_log_prob[:, start:stop]
                # hidden states saved as [T, layers, N, H]: take the ones at trajectory starts
                lwd = last_was_done.permute(1, 0)
                hid_a = [s.permute(2, 0, 1, 3)[lwd][first_traj:last_traj].transpose(1, 0).contiguous()
                         for s in self.saved_hidden_states_a]
                hid_c = [s.permute(2, 0, 1, 3)[lwd][first_traj:last_traj].transpose(1, 0).contiguous()
                         for s in self.saved_hidden_states_c]
                hid_a = hid_a[0] if len(hid_a) == 1 else tuple(hid_a)
                hid_c = hid_c[0] if len(hid_c) == 1 else tuple(hid_c)
                yield (obs_batch, critic_obs_batch, actions_batch, values_batch, advantages_batch, returns_batch,
                       old_actions_log_prob_batch, old_mu_batch, old_sigma_batch, (hid_a, hid_c), masks_batch)
                first_traj = last_traj

    def recurrent_dense_mini_batch_generator(self, num_mini_batches, num_epochs=8):
        """The recurrent mini-batches of reccurent_mini_batch_generator (contiguous env
        slices, every epoch in the same order) in the dense form: [T, envs, .] tensors,
        the hidden states saved at t = 0, and reset[t] = dones[t-1] (the memory zeroes its
        state there, which is where a padded trajectory would start from zeros).  Fixed
        shapes and no device->host sync (the padded form counts trajectories on the host)."""
        mb = self.num_envs // num_mini_batches
        if not hasattr(self, "_dense_reset") or self._dense_reset.shape != self.dones.shape[:2]:
            self._dense_reset = torch.zeros(self.dones.shape[:2], dtype=torch.uint8, device=self.device)
        reset = self._dense_reset
        reset[1:].copy_(self.dones[:-1, :, 0])  # in place: a captured update reads this buffer
        cobs = self.privileged_observations if self.privileged_observations is not None else self.observations
        # Once per update, every [T, N, .] tensor is regrouped into contiguous per-mini-batch
        # blocks [num_mini_batches, T, mb, .] (persistent buffers, written in place: a captured
        # update reads them), so the epochs' steps read contiguous slices and nothing is
        # copied per optimizer step.
        srcs = (self.observations, cobs, self.actions, self.values, self.advantages, self.returns,
                self.actions_log_prob, self.mu, self.sigma, reset)
        blocks = getattr(self, "_dense_blocks", None)
        if blocks is None or len(blocks) != len(srcs) or blocks[0].shape[:3] != (num_mini_batches, self.dones.shape[0],
                                                                               mb):
            blocks = [torch.empty((num_mini_batches, t.shape[0], mb) + tuple(t.shape[2:]), dtype=t.dtype,
                                  device=t.device) for t in srcs]
            self._dense_blocks = blocks
        for b, t in zip(blocks, srcs):
            b.copy_(t[:, :num_mini_batches * mb].unflatten(1, (num_mini_batches, mb)).transpose(0, 1))
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                sl = slice(i * mb, (i + 1) * mb)
                hid_a = tuple(h[0][:, sl] for h in self.saved_hidden_states_a)
                hid_c = tuple(h[0][:, sl] for h in self.saved_hidden_states_c)
                yield tuple(b[i] for b in blocks[:9]) + ((hid_a, hid_c), blocks[9][i])
