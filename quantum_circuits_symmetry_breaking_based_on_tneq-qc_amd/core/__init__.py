from .qctn import QCTN
from .tn_tensor import TNTensor

__all__ = ["QCTN", "TNTensor"]
