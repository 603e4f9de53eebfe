"""TNTensor: a device tensor with a host scalar scale (mirror of tneq_qc/core/tn_tensor.py:4-125).

Executors multiply the scales of the operands of a contraction and keep the product on the
host (reference: greedy_strategy.py:912-957, einsum_strategy.py:87-106); only `scale_to` /
`auto_scale` touch the device data.
"""
from __future__ import annotations

import math
from typing import Any, Optional


class TNTensor:
    def __init__(self, tensor: Any, scale: Any = 1.0, log_scale: Optional[float] = None):
        self._tensor = tensor
        self.scale = float(scale)
        if log_scale is not None:
            self.log_scale = log_scale
        else:
            self.log_scale = math.log(abs(self.scale)) if self.scale != 0 else float("-inf")

    @property
    def tensor(self) -> Any:
        return self._tensor

    @property
    def ndim(self) -> int:
        return self._tensor.ndim

    @property
    def shape(self) -> tuple:
        return self._tensor.shape

    @property
    def dtype(self) -> Any:
        return self._tensor.dtype

    def is_complex(self) -> bool:
        # the reference's TNTensor lacks this, which breaks its symmetric greedy path for
        # TNTensor cores; providing it is harmless.
        f = getattr(self._tensor, "is_complex", None)
        return bool(f()) if callable(f) else False

    def auto_scale(self):
        """Scale the data so that max |x| == 1 and fold the factor into `scale` (tn_tensor.py:67-85)."""
        m = self._tensor.abs().max()
        mv = m.item() if hasattr(m, "item") else float(m)
        if mv == 0:
            return
        self._tensor = self._tensor / mv
        self.scale *= mv
        self.log_scale += math.log(abs(mv))

    def scale_to(self, new_scale: float):
        """Rescale so that `scale == new_scale`, value unchanged (tn_tensor.py:87-104)."""
        new_scale = float(new_scale)
        if new_scale == 0:
            raise ValueError("Cannot scale to 0.")
        factor = self.scale / new_scale
        self._tensor = self._tensor * factor
        self.scale = new_scale
        self.log_scale = math.log(abs(self.scale))

    def scale_with(self, factor: float):
        """tn_tensor.py:106-121."""
        factor = float(factor)
        if factor == 0:
            raise ValueError("Cannot scale with factor 0.")
        self._tensor = self._tensor / factor
        self.scale *= factor
        self.log_scale += math.log(abs(factor))

    def __repr__(self):
        return f"TNTensor(shape={getattr(self._tensor, 'shape', 'unknown')}, scale={self.scale})"
