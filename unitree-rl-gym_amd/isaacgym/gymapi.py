"""gymapi subset: enums and parameter containers read by legged_gym."""
from types import SimpleNamespace

SIM_PHYSX = 1
SIM_FLEX = 0
UP_AXIS_Y = 0
UP_AXIS_Z = 1


class Vec3(SimpleNamespace):
    def __init__(self, x=0.0, y=0.0, z=0.0):
        super().__init__(x=float(x), y=float(y), z=float(z))


class PhysXParams(SimpleNamespace):
    def __init__(self):
        super().__init__(num_threads=0, solver_type=1, num_position_iterations=4, num_velocity_iterations=1,
                         contact_offset=0.02, rest_offset=0.001, bounce_threshold_velocity=0.2,
                         max_depenetration_velocity=100.0, max_gpu_contact_pairs=1024 * 1024,
                         default_buffer_size_multiplier=2.0, contact_collection=1, use_gpu=True,
                         num_subscenes=0)


class SimParams(SimpleNamespace):
    def __init__(self):
        super().__init__(dt=1.0 / 60.0, substeps=2, gravity=Vec3(0.0, 0.0, -9.81), up_axis=UP_AXIS_Z,
                         use_gpu_pipeline=True, physx=PhysXParams())


def acquire_gym():
    raise RuntimeError("the MI355X build has no PhysX gym; environments are created by legged_gym on leggedsim")
