"""gymtorch subset: leggedsim state tensors are already torch tensors."""


def wrap_tensor(t):
    return t


def unwrap_tensor(t):
    return t
