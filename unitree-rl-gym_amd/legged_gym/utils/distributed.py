"""Data-parallel training from the unmodified entry scripts.

The reference trains on one device; its only distributed flag, ``--horovod``, is parsed
and never read (reference utils/helpers.py:132).  Here ``train.py`` launched under
``torch.distributed.run`` (one process per GPU) shards the envs across ranks:

* ``task_registry.make_env`` / ``make_alg_runner`` call :func:`init_from_env` before
  anything is built.  When ``WORLD_SIZE`` > 1 it binds this rank to
  ``cuda:LOCAL_RANK`` (modulo the visible devices), rewrites ``args.sim_device`` /
  ``args.rl_device`` to it, and initialises the process group;
* the env offsets its RNG seed by ``RANK`` (``leggedsim/task.py``), so every rank
  simulates its own ``num_envs`` envs;
* ``PPO`` broadcasts the parameters from rank 0 and all-reduces one gradient bucket
  per optimizer step; ``OnPolicyRunner`` logs and checkpoints on rank 0 only.

Backend: ``"nccl"`` (RCCL over xGMI on ROCm) when every rank has a device of its own;
``"gloo"`` when ranks share a device (RCCL refuses two ranks on one GPU) or there is no
GPU.  ``LEGGED_GYM_DIST_BACKEND`` overrides the choice.
"""
import os

import torch
import torch.distributed as dist


def world_from_env():
    """(world_size, rank, local_rank, local_world_size) from the torch.distributed.run
    environment; (1, 0, 0, 1) outside a launcher."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    return world, rank, local, local_world


def rank_device(local_rank, n_devices):
    """The device index a rank uses: its local rank modulo the visible devices (several
    ranks share a device only when there are fewer devices than local ranks)."""
    if n_devices <= 0:
        raise ValueError("no visible device to place the rank on")
    return int(local_rank) % int(n_devices)


def choose_backend(local_world, n_devices):
    """RCCL ("nccl") when every local rank owns a device, else gloo."""
    forced = os.environ.get("LEGGED_GYM_DIST_BACKEND")
    if forced:
        return forced
    return "nccl" if n_devices > 0 and local_world <= n_devices else "gloo"


def init_from_env(args=None):
    """Set up this process's rank before the sim and the runner are built.

    Returns the world size.  Idempotent: a second call (make_alg_runner after make_env)
    only re-applies the device to ``args``.  With ``WORLD_SIZE`` unset or 1 nothing
    changes, so a single-process run behaves exactly as the reference."""
    world, rank, local, local_world = world_from_env()
    if world <= 1:
        return 1
    # torch.cuda.device_count() does not initialise the GPU on this image
    n_dev = torch.cuda.device_count()
    wants_cuda = args is None or str(getattr(args, "sim_device", "cuda")).startswith("cuda") or \
        str(getattr(args, "rl_device", "cuda")).startswith("cuda")
    dev = None
    if wants_cuda and n_dev > 0:
        idx = rank_device(local, n_dev)
        dev = f"cuda:{idx}"
        if args is not None:
            args.sim_device = args.rl_device = dev
            args.sim_device_id = args.compute_device_id = idx
    if not dist.is_initialized():
        if dev is not None:
            torch.cuda.set_device(int(dev.split(":")[1]))
        backend = choose_backend(local_world, n_dev if dev is not None else 0)
        kw = dict(backend=backend)
        if backend == "nccl" and dev is not None:
            kw["device_id"] = torch.device(dev)
        dist.init_process_group(**kw)
        if rank == 0:
            print(f"data-parallel training: {world} ranks, backend {backend}, rank 0 on {dev or 'cpu'}")
    return dist.get_world_size()


def is_main_process():
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
