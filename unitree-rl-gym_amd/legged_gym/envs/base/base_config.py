import inspect


class BaseConfig:
    """Nested-class config container (reference: envs/base/base_config.py:9-25).

    Instantiating the outer class instantiates every nested class recursively,
    so ``cfg.env.num_envs = 8`` mutates this instance only.
    """

    def __init__(self) -> None:
        self.init_member_classes(self)

    @staticmethod
    def init_member_classes(obj):
        members = [(name, getattr(obj, name)) for name in dir(obj) if name != "__class__"]
        for name, member in members:
            if not inspect.isclass(member):
                continue
            child = member()
            setattr(obj, name, child)
            BaseConfig.init_member_classes(child)
