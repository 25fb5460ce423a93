"""gymutil subset: the CLI parser and device-string helper used by legged_gym.

Flag names and defaults follow IsaacGym's parse_arguments (the common
--sim_device/--pipeline/--graphics_device_id/--physx/--flex/--num_threads/
--subscenes/--slices flags) plus the caller's custom parameters
(legged_gym/utils/helpers.py:123-137).
"""
import argparse

from . import gymapi


def parse_device_str(device_str):
    device = "cpu"
    device_id = 0
    if device_str in ("cpu", "cuda"):
        device = device_str
    elif device_str.startswith("cuda:"):
        device = "cuda"
        device_id = int(device_str.split(":")[1])
    else:
        raise ValueError(f"invalid device string {device_str!r}")
    return device, device_id


def parse_arguments(description="Isaac Gym Example", headless=False, no_graphics=False, custom_parameters=None,
                    argv=None):
    parser = argparse.ArgumentParser(description=description)
    if headless:
        parser.add_argument("--headless", action="store_true", help="Run headless without creating a viewer window")
    if no_graphics:
        parser.add_argument("--nographics", action="store_true")
    parser.add_argument("--sim_device", type=str, default="cuda:0", help="Physics device: cuda:N (the HIP engine)")
    parser.add_argument("--pipeline", type=str, default="gpu", help="Tensor API pipeline (gpu only)")
    parser.add_argument("--graphics_device_id", type=int, default=0)
    g = parser.add_mutually_exclusive_group()
    g.add_argument("--flex", action="store_true")
    g.add_argument("--physx", action="store_true")
    parser.add_argument("--num_threads", type=int, default=0)
    parser.add_argument("--subscenes", type=int, default=0)
    parser.add_argument("--slices", type=int)
    for p in custom_parameters or []:
        p = dict(p)
        name = p.pop("name")
        if "type" in p or "action" in p:
            parser.add_argument(name, **p)
        else:
            parser.add_argument(name, type=str, **p)
    args = parser.parse_args(argv)
    args.sim_device_type, args.compute_device_id = parse_device_str(args.sim_device)
    pipeline = args.pipeline.lower()
    if pipeline not in ("cpu", "gpu", "cuda"):
        raise ValueError(f"invalid pipeline {args.pipeline!r}")
    args.use_gpu_pipeline = pipeline in ("gpu", "cuda")
    if args.sim_device_type != "cuda" and args.flex:
        args.sim_device = "cuda:0"
        args.sim_device_type, args.compute_device_id = "cuda", 0
    args.physics_engine = gymapi.SIM_FLEX if args.flex else gymapi.SIM_PHYSX
    args.use_gpu = args.sim_device_type == "cuda"
    if args.slices is None:
        args.slices = args.subscenes
    return args


def parse_sim_config(cfg, sim_params):
    """Copy a class_to_dict(cfg.sim) dict into a SimParams (recursing into physx)."""
    for key, val in cfg.items():
        if key == "physx" and isinstance(val, dict):
            for k2, v2 in val.items():
                setattr(sim_params.physx, k2, v2)
        elif key == "gravity":
            sim_params.gravity = gymapi.Vec3(*val)
        else:
            setattr(sim_params, key, val)
