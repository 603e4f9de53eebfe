from .slice_reduce import (AllReduceSum, SlicedContraction, allreduce_partials, allreduce_with_grad,
                           shard_slices)

__all__ = ["AllReduceSum", "SlicedContraction", "allreduce_partials", "allreduce_with_grad", "shard_slices"]
