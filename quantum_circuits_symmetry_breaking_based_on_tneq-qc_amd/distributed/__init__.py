from .slice_reduce import (AllReduceSum, SlicedContraction, allreduce_partials, allreduce_with_grad,
                           shard_slices)
from .tree import TreeContraction, partition_terms

__all__ = ["AllReduceSum", "SlicedContraction", "allreduce_partials", "allreduce_with_grad", "shard_slices",
           "TreeContraction", "partition_terms"]
