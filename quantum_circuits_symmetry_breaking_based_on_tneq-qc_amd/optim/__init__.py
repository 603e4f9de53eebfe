"""Optimizers of the symmetry-breaking training loop (mirror of tneq_qc/optim)."""
from .stiefel_optimizer_complex import SGDG

__all__ = ["SGDG"]
