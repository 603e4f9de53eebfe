from .qctn import QCTN
from .tn_tensor import TNTensor

__all__ = ["Engine", "QCTN", "TNTensor"]


def __getattr__(name):
    # Engine imports the contractor, which imports core: resolved on first use
    if name == "Engine":
        from .engine import Engine
        return Engine
    raise AttributeError(name)
