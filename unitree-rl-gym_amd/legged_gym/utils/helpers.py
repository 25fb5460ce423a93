"""CLI / config / checkpoint / export helpers (reference utils/helpers.py:11-189)."""
import copy
import os
import random

import numpy as np
import torch
from isaacgym import gymapi, gymutil

from legged_gym import LEGGED_GYM_ROOT_DIR, LEGGED_GYM_ENVS_DIR  # noqa: F401


def class_to_dict(obj) -> dict:
    """Nested config object -> dict.  Keys in dir() (alphabetical) order, which the
    reward bookkeeping depends on (legged_robot.py:822-836)."""
    if not hasattr(obj, "__dict__"):
        return obj
    out = {}
    for key in dir(obj):
        if key.startswith("_"):
            continue
        val = getattr(obj, key)
        out[key] = [class_to_dict(v) for v in val] if isinstance(val, list) else class_to_dict(val)
    return out


def update_class_from_dict(obj, d):
    for key, val in d.items():
        attr = getattr(obj, key, None)
        if isinstance(attr, type):
            update_class_from_dict(attr, val)
        else:
            setattr(obj, key, val)


def set_seed(seed):
    if seed == -1:
        seed = np.random.randint(0, 10000)
    print(f"Setting seed: {seed}")
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed(seed)
        torch.cuda.manual_seed_all(seed)


def parse_sim_params(args, cfg):
    sim_params = gymapi.SimParams()
    if args.physics_engine == gymapi.SIM_FLEX:
        raise ValueError("Flex is not supported; the MI355X engine replaces PhysX only")
    sim_params.physx.use_gpu = args.use_gpu
    sim_params.physx.num_subscenes = args.subscenes
    sim_params.use_gpu_pipeline = args.use_gpu_pipeline
    if "sim" in cfg:
        gymutil.parse_sim_config(cfg["sim"], sim_params)
    if args.num_threads > 0:
        sim_params.physx.num_threads = args.num_threads
    return sim_params


def get_load_path(root, load_run=-1, checkpoint=-1):
    try:
        runs = sorted(os.listdir(root))
        if "exported" in runs:
            runs.remove("exported")
        last_run = os.path.join(root, runs[-1])
    except Exception:
        raise ValueError("No runs in this directory: " + root)
    load_run = last_run if load_run == -1 else os.path.join(root, load_run)
    if checkpoint == -1:
        models = sorted((f for f in os.listdir(load_run) if "model" in f), key=lambda m: f"{m:0>15}")
        model = models[-1]
    else:
        model = f"model_{checkpoint}.pt"
    return os.path.join(load_run, model)


def update_cfg_from_args(env_cfg, cfg_train, args):
    if env_cfg is not None and args.num_envs is not None:
        env_cfg.env.num_envs = args.num_envs
    if cfg_train is not None:
        for name, dest in (("seed", None), ("max_iterations", "max_iterations"), ("experiment_name", "experiment_name"),
                           ("run_name", "run_name"), ("load_run", "load_run"), ("checkpoint", "checkpoint")):
            val = getattr(args, name, None)
            if val is None:
                continue
            if dest is None:
                cfg_train.seed = val
            else:
                setattr(cfg_train.runner, dest, val)
        if args.resume:
            cfg_train.runner.resume = args.resume
    return env_cfg, cfg_train


CUSTOM_PARAMETERS = [
    {"name": "--task", "type": str, "default": "go2", "help": "Registered task name"},
    {"name": "--resume", "action": "store_true", "default": False, "help": "Resume training from a checkpoint"},
    {"name": "--experiment_name", "type": str, "help": "Overrides cfg.runner.experiment_name"},
    {"name": "--run_name", "type": str, "help": "Overrides cfg.runner.run_name"},
    {"name": "--load_run", "type": str, "help": "Run to load when resume=True (-1: last)"},
    {"name": "--checkpoint", "type": int, "help": "Checkpoint number to load (-1: last)"},
    {"name": "--headless", "action": "store_true", "default": False, "help": "No viewer"},
    {"name": "--horovod", "action": "store_true", "default": False, "help": "(unused, kept for CLI parity)"},
    {"name": "--rl_device", "type": str, "default": "cuda:0", "help": "Device of the RL algorithm"},
    {"name": "--num_envs", "type": int, "help": "Overrides cfg.env.num_envs"},
    {"name": "--seed", "type": int, "help": "Overrides the train cfg seed"},
    {"name": "--max_iterations", "type": int, "help": "Overrides cfg.runner.max_iterations"},
]


def get_args(argv=None):
    args = gymutil.parse_arguments(description="RL Policy", custom_parameters=CUSTOM_PARAMETERS, argv=argv)
    args.sim_device_id = args.compute_device_id
    args.sim_device = args.sim_device_type
    if args.sim_device == "cuda":
        args.sim_device += f":{args.sim_device_id}"
    return args


def export_policy_as_jit(actor_critic, path):
    """policy_1.pt (scripted MLP actor) or policy_lstm_1.pt (PolicyExporterLSTM)."""
    if hasattr(actor_critic, "memory_a"):
        PolicyExporterLSTM(actor_critic).export(path)
        return
    os.makedirs(path, exist_ok=True)
    model = _plain_linear(copy.deepcopy(actor_critic.actor).to("cpu"))
    torch.jit.script(model).save(os.path.join(path, "policy_1.pt"))


def _plain_linear(module):
    """SplitKLinear -> nn.Linear (same parameters) so the exported module scripts
    to exactly the reference's structure."""
    from rsl_rl.modules.splitk_linear import SplitKLinear
    for name, child in module.named_children():
        if isinstance(child, SplitKLinear):
            lin = torch.nn.Linear(child.in_features, child.out_features, bias=child.bias is not None)
            lin.load_state_dict(child.state_dict())
            setattr(module, name, lin)
        else:
            _plain_linear(child)
    return module


class PolicyExporterLSTM(torch.nn.Module):
    """TorchScript module with the reference export's buffers and methods
    (hidden_state / cell_state, forward(x), reset_memory())."""

    def __init__(self, actor_critic):
        super().__init__()
        self.actor = _plain_linear(copy.deepcopy(actor_critic.actor))
        self.is_recurrent = actor_critic.is_recurrent
        self.memory = copy.deepcopy(actor_critic.memory_a.rnn)
        self.memory.cpu()
        self.register_buffer("hidden_state", torch.zeros(self.memory.num_layers, 1, self.memory.hidden_size))
        self.register_buffer("cell_state", torch.zeros(self.memory.num_layers, 1, self.memory.hidden_size))

    def forward(self, x):
        out, (h, c) = self.memory(x.unsqueeze(0), (self.hidden_state, self.cell_state))
        self.hidden_state[:] = h
        self.cell_state[:] = c
        return self.actor(out.squeeze(0))

    @torch.jit.export
    def reset_memory(self):
        self.hidden_state[:] = 0.0
        self.cell_state[:] = 0.0

    def export(self, path):
        os.makedirs(path, exist_ok=True)
        self.to("cpu")
        torch.jit.script(self).save(os.path.join(path, "policy_lstm_1.pt"))
