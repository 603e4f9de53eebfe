from .comm import (CommBase, CommTorch, DistributedContext, MockCommTorch, ReduceOp, get_comm_backend,
                   get_comm_torch)
from .engine import ContractStage, DistributedContractPlan, DistributedEngineSiamese, PartitionConfig
from .slice_reduce import (AllReduceSum, SlicedContraction, align_log_scales, allreduce_partials,
                           allreduce_with_grad, shard_slices)
from .tree import TreeContraction, partition_terms

__all__ = ["AllReduceSum", "SlicedContraction", "align_log_scales", "allreduce_partials", "allreduce_with_grad",
           "shard_slices", "TreeContraction", "partition_terms", "DistributedEngineSiamese", "PartitionConfig",
           "ContractStage", "DistributedContractPlan", "CommBase", "CommTorch", "MockCommTorch",
           "ReduceOp", "DistributedContext", "get_comm_backend", "get_comm_torch"]
