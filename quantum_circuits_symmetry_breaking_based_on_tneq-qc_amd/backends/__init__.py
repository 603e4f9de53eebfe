from .backend_factory import BackendFactory
from .backend_hip import BackendHIP
from .backend_interface import BackendInfo, ComputeBackend

__all__ = ["BackendFactory", "BackendHIP", "BackendInfo", "ComputeBackend"]
