import torch
import torch.nn as nn
from torch.distributions import Normal

from . import mfma_mlp
from .splitk_linear import SplitKLinear


def get_activation(name):
    table = {"elu": nn.ELU(), "selu": nn.SELU(), "relu": nn.ReLU(), "crelu": nn.ReLU(), "lrelu": nn.LeakyReLU(),
             "tanh": nn.Tanh(), "sigmoid": nn.Sigmoid()}
    if name not in table:
        print("invalid activation function!")
        return None
    return table[name]


def mlp(in_dim, hidden, out_dim, activation):
    layers = [SplitKLinear(in_dim, hidden[0]), activation]
    for i in range(len(hidden)):
        if i == len(hidden) - 1:
            layers.append(SplitKLinear(hidden[i], out_dim))
        else:
            layers.append(SplitKLinear(hidden[i], hidden[i + 1]))
            layers.append(activation)
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    """Gaussian MLP actor + MLP critic (rsl_rl v1.0.2 ActorCritic).

    ``mixed_precision=True`` (default) runs both MLPs' forward and backward on the
    hand-written bf16 MFMA kernels (modules/mfma_mlp.py, csrc/ppo_mlp.hip): bf16
    operands, fp32 accumulation, fp32 parameters, gradients, distribution and
    losses.  ``False`` is plain fp32 torch (the reference's arithmetic).
    """
    is_recurrent = False

    def __init__(self, num_actor_obs, num_critic_obs, num_actions, actor_hidden_dims=[256, 256, 256],
                 critic_hidden_dims=[256, 256, 256], activation="elu", init_noise_std=1.0, mixed_precision=True,
                 **kwargs):
        if kwargs:
            print("ActorCritic.__init__ got unexpected arguments, which will be ignored: " + str([k for k in kwargs]))
        super().__init__()
        act = get_activation(activation)
        self.actor = mlp(num_actor_obs, actor_hidden_dims, num_actions, act)
        self.critic = mlp(num_critic_obs, critic_hidden_dims, 1, act)
        print(f"Actor MLP: {self.actor}")
        print(f"Critic MLP: {self.critic}")
        self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        self.distribution = None
        self.mixed_precision = mixed_precision

    def _run(self, net, x):
        if self.mixed_precision and mfma_mlp.usable(net, x):
            return mfma_mlp.mlp_apply(net, x)  # hand-written bf16 MFMA forward/backward
        return net(x)

    @staticmethod
    def init_weights(sequential, scales):
        [torch.nn.init.orthogonal_(module.weight, gain=scales[idx]) for idx, module in
         enumerate(mod for mod in sequential if isinstance(mod, nn.Linear))]

    def reset(self, dones=None):
        pass

    def forward(self):
        raise NotImplementedError

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def update_distribution(self, observations):
        mean = self._run(self.actor, observations)
        # validate_args=False: v1.0.2 meant to disable validation (it assigns
        # Normal.set_default_validate_args = False, which does not); validation
        # costs a device->host sync per call and breaks graph capture.
        self.distribution = Normal(mean, mean * 0.0 + self.std, validate_args=False)

    def act(self, observations, **kwargs):
        self.update_distribution(observations)
        # = distribution.sample() (mean + std * N(0, 1) draws) through randn_like: torch.normal
        # with tensor mean/std is not capturable on this ROCm, randn is (graph-safe RNG)
        d = self.distribution
        with torch.no_grad():
            return d.mean + d.stddev * torch.randn_like(d.mean)

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def policy_mean(self, observations):
        """Actor output (the Gaussian mean) without building the distribution."""
        return self._run(self.actor, observations)

    def mean_and_value(self, observations, critic_observations):
        """Actor mean and critic value; on the MFMA path both nets share every launch."""
        if self.mixed_precision and mfma_mlp.usable(self.actor, observations) and \
                mfma_mlp.usable(self.critic, critic_observations) and \
                observations.shape[0] == critic_observations.shape[0] and \
                (len(self.actor) == len(self.critic)):
            return mfma_mlp.mlps_apply([self.actor, self.critic], [observations, critic_observations])
        return self._run(self.actor, observations), self._run(self.critic, critic_observations)

    def act_and_value(self, observations, critic_observations):
        """act() + evaluate() of one rollout step (the distribution is kept, as act() does)."""
        mean, value = self.mean_and_value(observations, critic_observations)
        std = mean * 0.0 + self.std
        self.distribution = Normal(mean, std, validate_args=False)
        # = Normal.sample() (normal_(0, 1) * std + mean, the same draws) without its
        # std >= 0 check, a device->host sync that hipGraph capture forbids
        with torch.no_grad():
            return mean + std * torch.randn_like(mean), value

    def act_inference(self, observations):
        return self._run(self.actor, observations)

    def evaluate(self, critic_observations, **kwargs):
        return self._run(self.critic, critic_observations)
