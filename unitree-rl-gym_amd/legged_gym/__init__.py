"""legged_gym drop-in for the MI355X-native simulator.

Same package name, module layout and public names as the reference
(`legged_gym/__init__.py:1-4`): scripts that do ``from legged_gym.envs import *``
and ``from legged_gym.utils import get_args, task_registry`` run unchanged.
"""
import os

LEGGED_GYM_ROOT_DIR = os.path.dirname(os.path.dirname(os.path.realpath(__file__)))
LEGGED_GYM_ENVS_DIR = os.path.join(LEGGED_GYM_ROOT_DIR, "legged_gym", "envs")
