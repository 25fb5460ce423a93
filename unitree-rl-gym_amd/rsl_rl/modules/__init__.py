from .actor_critic import ActorCritic
from .actor_critic_recurrent import ActorCriticRecurrent
