"""BaseTask: VecEnv buffers and reset() contract (reference envs/base/base_task.py:9-114)."""
import torch


class BaseTask:
    def __init__(self, cfg, sim_params, physics_engine, sim_device, headless):
        self.sim_params = sim_params
        self.physics_engine = physics_engine
        self.sim_device = sim_device
        kind, self.sim_device_id = _parse_device(sim_device)
        self.headless = headless
        use_gpu_pipeline = getattr(sim_params, "use_gpu_pipeline", True)
        if kind != "cuda" or not use_gpu_pipeline:
            # The reference would fall back to CPU PhysX here; this build has one
            # physics engine, the HIP kernels, and refuses rather than silently
            # running anything else.
            raise RuntimeError(
                f"sim_device={sim_device!r} / pipeline: the MI355X-native simulator runs on a GPU "
                "(cuda:N with the gpu pipeline); there is no CPU physics path")
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible: the MI355X-native simulator needs a ROCm device")
        self.device = self.sim_device
        self.graphics_device_id = -1 if headless else self.sim_device_id

        self.num_envs = cfg.env.num_envs
        self.num_obs = cfg.env.num_observations
        self.num_privileged_obs = cfg.env.num_privileged_obs
        self.num_actions = cfg.env.num_actions

        self.extras = {}
        self.viewer = None
        self.enable_viewer_sync = True
        self.create_sim()

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    def reset_idx(self, env_ids):
        raise NotImplementedError

    def reset(self):
        """reset_idx(all envs) then one step with zero actions (base_task.py:82-86)."""
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        obs, privileged_obs, _, _, _ = self.step(
            torch.zeros(self.num_envs, self.num_actions, device=self.device, requires_grad=False))
        return obs, privileged_obs

    def step(self, actions):
        raise NotImplementedError

    def render(self, sync_frame_time=True):
        """Headless build: no viewer (the reference's render is a no-op headless)."""
        return None


def _parse_device(dev):
    if dev in ("cpu", "cuda"):
        return dev, 0
    if dev.startswith("cuda:"):
        return "cuda", int(dev.split(":")[1])
    raise ValueError(f"invalid device string {dev!r}")
