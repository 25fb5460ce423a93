import torch
import torch.nn as nn

from rsl_rl.modules import lstm_seq
from rsl_rl.modules.actor_critic import ActorCritic, get_activation  # noqa: F401
from rsl_rl.utils import unpad_trajectories


class ActorCriticRecurrent(ActorCritic):
    """LSTM/GRU memory in front of the MLP actor and critic (rsl_rl v1.0.2).

    Attribute names (``memory_a.rnn``, ``actor``, ``is_recurrent``) are what
    ``export_policy_as_jit`` / ``PolicyExporterLSTM`` read (helpers.py:151-168).
    """
    is_recurrent = True

    def __init__(self, num_actor_obs, num_critic_obs, num_actions, actor_hidden_dims=[256, 256, 256],
                 critic_hidden_dims=[256, 256, 256], activation="elu", rnn_type="lstm", rnn_hidden_size=256,
                 rnn_num_layers=1, init_noise_std=1.0, **kwargs):
        if kwargs:
            print("ActorCriticRecurrent.__init__ got unexpected arguments, which will be ignored: " + str(kwargs.keys()))
        super().__init__(num_actor_obs=rnn_hidden_size, num_critic_obs=rnn_hidden_size, num_actions=num_actions,
                         actor_hidden_dims=actor_hidden_dims, critic_hidden_dims=critic_hidden_dims,
                         activation=activation, init_noise_std=init_noise_std, mixed_precision=False)
        self.memory_a = Memory(num_actor_obs, type=rnn_type, num_layers=rnn_num_layers, hidden_size=rnn_hidden_size)
        self.memory_c = Memory(num_critic_obs, type=rnn_type, num_layers=rnn_num_layers, hidden_size=rnn_hidden_size)
        print(f"Actor RNN: {self.memory_a}")
        print(f"Critic RNN: {self.memory_c}")

    def reset(self, dones=None):
        self.memory_a.reset(dones)
        self.memory_c.reset(dones)

    def act(self, observations, masks=None, hidden_states=None):
        input_a = self.memory_a(observations, masks, hidden_states)
        return super().act(input_a.squeeze(0))

    def act_inference(self, observations):
        input_a = self.memory_a(observations)
        return super().act_inference(input_a.squeeze(0))

    def evaluate(self, critic_observations, masks=None, hidden_states=None):
        input_c = self.memory_c(critic_observations, masks, hidden_states)
        return super().evaluate(input_c.squeeze(0))

    def get_hidden_states(self):
        return self.memory_a.hidden_states, self.memory_c.hidden_states

    def rollout_capturable(self):
        """Both memories step on the LSTM kernels in place (a graph-capturable rollout)."""
        p = self.memory_a.rnn.weight_hh_l0
        probe = p.new_empty(1, 1)
        return all(lstm_seq.usable(m.rnn, probe) for m in (self.memory_a, self.memory_c))

    # ---- dense update form (no padded trajectories; rsl_rl/modules/lstm_seq.py) ----
    def act_dense(self, observations, hidden_states, reset):
        """update_distribution over a [T,B,O] sequence: the memory runs all T steps with
        resets before step t where reset[t]; the distribution covers the T*B rows."""
        input_a = self.memory_a.dense(observations, hidden_states, reset)
        self.update_distribution(input_a.reshape(-1, input_a.shape[-1]))

    def mean_and_value_dense(self, observations, critic_observations, hidden_states, reset):
        """(action mean, value) over the T*B rows of a [T,B,.] sequence pair (the fused-loss
        update: the distribution object is never built)."""
        input_a = self.memory_a.dense(observations, hidden_states[0], reset)
        input_c = self.memory_c.dense(critic_observations, hidden_states[1], reset)
        return (self.actor(input_a.reshape(-1, input_a.shape[-1])),
                self.critic(input_c.reshape(-1, input_c.shape[-1])))

    def evaluate_dense(self, critic_observations, hidden_states, reset):
        input_c = self.memory_c.dense(critic_observations, hidden_states, reset)
        return super().evaluate(input_c.reshape(-1, input_c.shape[-1]))


class Memory(torch.nn.Module):
    """rsl_rl v1.0.2 Memory.  On a GPU the one-layer LSTM runs on the sequence kernels of
    lstm_seq.py: in rollout mode one step updates the state buffers IN PLACE (static
    addresses: the collection loop can be captured in a HIP graph), and reset(dones)
    zeroes rows with a mask (no device->host sync)."""

    def __init__(self, input_size, type="lstm", num_layers=1, hidden_size=256):
        super().__init__()
        rnn_cls = nn.GRU if type.lower() == "gru" else nn.LSTM
        self.rnn = rnn_cls(input_size=input_size, hidden_size=hidden_size, num_layers=num_layers)
        self.hidden_states = None

    def forward(self, input, masks=None, hidden_states=None):
        if masks is not None:  # batch (update) mode: padded trajectories (the rsl_rl API)
            if hidden_states is None:
                raise ValueError("Hidden states not passed to memory module during policy update")
            out, _ = self.rnn(input, hidden_states)
            out = unpad_trajectories(out, masks)
        elif lstm_seq.usable(self.rnn, input):  # rollout mode on the kernel: state updated in place
            out = self.step_(input)
        else:  # rollout mode: one step, keep the state
            out, self.hidden_states = self.rnn(input.unsqueeze(0), self.hidden_states)
        return out

    def step_(self, input, save=None):
        """Rollout step on the LSTM kernel, the state buffers updated in place (created as
        zeros on first use); save = (h_dst, c_dst) receives the state the step starts from."""
        B, H = input.shape[0], self.rnn.hidden_size
        hs = self.hidden_states
        if hs is None or not isinstance(hs, tuple) or hs[0].shape != (1, B, H) or hs[0].device != input.device:
            with torch.inference_mode(False):
                self.hidden_states = (torch.zeros(1, B, H, device=input.device),
                                      torch.zeros(1, B, H, device=input.device))
        return lstm_seq.lstm_step_(self.rnn, input, self.hidden_states[0], self.hidden_states[1], save=save)

    def dense(self, input, hidden_states, reset):
        """[T,B,I] -> [T,B,H]: all T steps from hidden_states (the state saved at t = 0),
        zeroing the state before step t where reset[t] (dense form of the padded update)."""
        if not isinstance(self.rnn, nn.LSTM):
            raise NotImplementedError("dense memory update: LSTM only")
        h0, c0 = (None, None) if hidden_states is None else hidden_states
        if lstm_seq.usable(self.rnn, input):
            return lstm_seq.lstm_dense(self.rnn, input, h0, c0, reset)
        return lstm_seq.lstm_dense_reference(self.rnn, input, h0, c0, reset)

    def reset(self, dones=None):
        if self.hidden_states is None:
            return
        states = self.hidden_states if isinstance(self.hidden_states, tuple) else (self.hidden_states,)
        mask = dones.bool().view(1, -1, 1)
        for h in states:
            h.masked_fill_(mask, 0.0)
