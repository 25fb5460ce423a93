"""rsl_rl (v1.0.2 API) re-implemented for ROCm.

The reference pins rsl_rl v1.0.2 as an un-vendored submodule
(``/root/reference/rsl_rl`` is empty; doc/setup_en.md:87-112) and calls it at
utils/task_registry.py:8-9,119,126, scripts/train.py:14, scripts/play.py:34,39
and utils/helpers.py:151-168.  This package restates that API: OnPolicyRunner,
PPO, ActorCritic, ActorCriticRecurrent, RolloutStorage, VecEnv.

Attribution: the API, the runner's log strings and the storage layout follow the
public rsl_rl v1.0.2 (Copyright (c) 2021, ETH Zurich, Nikita Rudin; NVIDIA;
BSD-3-Clause), restated for drop-in compatibility with the reference's callers.
"""
