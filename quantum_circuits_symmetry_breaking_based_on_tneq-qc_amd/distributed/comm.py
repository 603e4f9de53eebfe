"""The reference's communication-backend surface over torch.distributed ("nccl" = RCCL on ROCm).

Reference: `tneq_qc/distributed/comm/comm_interface.py` (CommBase, ReduceOp, DistributedContext),
`comm_torch.py:51-175,205-560` (TorchAsyncHandle, CommTorch), `comm_torch.py:563-690`
(MockCommTorch, get_comm_torch) and `comm_factory.py:25-82,118-210` (get_comm_backend,
detect_best_backend).  A reference caller builds its comm object with
`get_comm_backend('torch' | 'mock' | 'auto', ...)` (`distributed_trainer.py:228-283`) and hands it to
`DistributedEngineSiamese(comm=...)` (`distributed_engine.py:220-251`), which reads `comm.rank` /
`comm.world_size`; the engine here also accepts a plain process group.

Only the torch backends exist: mpi4py is not part of this stack, so the 'mpi' kind raises (the
reference falls back to a mock communicator when mpi4py is missing; an explicit 'mpi' request here
is a configuration error, not a silent single-process run).  Every collective goes through
`torch.distributed` on the communicator's `group` (None = WORLD); on device tensors with the
"nccl" backend that is RCCL over xGMI.
"""
from __future__ import annotations

import os
from abc import ABC, abstractmethod
from dataclasses import dataclass
from enum import Enum
from typing import Any, List, Optional, Tuple, Union

import torch
import torch.distributed as dist

__all__ = ["ReduceOp", "DistributedContext", "CommBase", "TorchAsyncHandle", "CommTorch", "MockCommTorch",
           "CommBackendType", "get_comm_backend", "get_comm_torch", "get_auto_backend", "get_mock_backend",
           "detect_best_backend", "comm_group", "comm_rank_size"]


class ReduceOp(Enum):
    """comm_interface.py:21-28; AVG = SUM then divide by the world size."""
    SUM = "SUM"
    AVG = "AVG"
    MAX = "MAX"
    MIN = "MIN"
    PRODUCT = "PRODUCT"


_TORCH_OPS = {ReduceOp.SUM: "SUM", ReduceOp.AVG: "SUM", ReduceOp.MAX: "MAX", ReduceOp.MIN: "MIN",
              ReduceOp.PRODUCT: "PRODUCT"}


def _op(op: ReduceOp):
    if isinstance(op, str):
        op = ReduceOp(op.upper())
    return getattr(dist.ReduceOp, _TORCH_OPS[op])


@dataclass
class DistributedContext:
    """comm_interface.py:31-41."""
    world_size: int
    rank: int
    node_rank: int
    num_nodes: int
    is_main_process: bool
    backend: str

    def __repr__(self):
        return (f"DistributedContext(rank={self.rank}/{self.world_size}, node={self.node_rank}/{self.num_nodes}, "
                f"main={self.is_main_process}, backend={self.backend})")


class CommBase(ABC):
    """comm_interface.py:44-344: the abstract communicator the reference's engines take."""

    @property
    @abstractmethod
    def rank(self) -> int: ...

    @property
    @abstractmethod
    def world_size(self) -> int: ...

    @property
    def node_rank(self) -> int:
        return 0

    @property
    def num_nodes(self) -> int:
        return 1

    #: the torch.distributed group the collectives run on (None = WORLD)
    group = None

    @abstractmethod
    def get_context(self) -> DistributedContext: ...

    def is_main_process(self) -> bool:
        return self.rank == 0

    @abstractmethod
    def is_initialized(self) -> bool: ...

    @abstractmethod
    def barrier(self) -> None: ...

    @abstractmethod
    def broadcast(self, tensor, src: int = 0): ...

    @abstractmethod
    def broadcast_object(self, obj: Any, src: int = 0) -> Any: ...

    @abstractmethod
    def allreduce(self, tensor, op: ReduceOp = ReduceOp.SUM): ...

    @abstractmethod
    def allreduce_inplace(self, tensor, op: ReduceOp = ReduceOp.SUM): ...

    @abstractmethod
    def allgather(self, tensor) -> List: ...

    @abstractmethod
    def send(self, tensor, dest: int, tag: int = 0) -> None: ...

    @abstractmethod
    def recv(self, src: int, tag: int = 0, **kwargs): ...

    def allreduce_list(self, tensors, op: ReduceOp = ReduceOp.AVG):
        return [self.allreduce(t, op) for t in tensors]

    def destroy(self) -> None:
        pass


class TorchAsyncHandle:
    """comm_torch.py:51-99: waits the pending all-reduces, AVG divided on completion."""

    def __init__(self, work_handles: List, tensors: List[torch.Tensor], op: ReduceOp, world_size: int):
        self.work_handles = work_handles
        self.tensors = tensors
        self.op = op
        self.world_size = world_size
        self._done = False

    def wait(self) -> List[torch.Tensor]:
        if not self._done:
            for w in self.work_handles:
                if w is not None:
                    w.wait()
            if self.op == ReduceOp.AVG and self.work_handles:
                for t in self.tensors:
                    t.div_(self.world_size)
            self._done = True
        return self.tensors

    def is_completed(self) -> bool:
        return self._done or all(w is None or w.is_completed() for w in self.work_handles)


class CommTorch(CommBase):
    """comm_torch.py:102-560 over torch.distributed.  Joins an initialised process group, or (with
    `auto_init`) initialises one from the launcher's environment (RANK / WORLD_SIZE / MASTER_*);
    "nccl" falls back to "gloo" without a GPU, as the reference does.  `group` restricts the
    collectives to a subgroup (the reference always uses WORLD)."""

    def __init__(self, torch_backend: str = "nccl", init_method: Optional[str] = None,
                 world_size: Optional[int] = None, rank: Optional[int] = None, node_rank: Optional[int] = None,
                 num_nodes: Optional[int] = None, auto_init: bool = True, group=None):
        if not dist.is_available():
            raise RuntimeError("torch.distributed is not available")
        if dist.is_initialized():
            self._initialized = True
        elif auto_init:
            world_size = int(os.environ.get("WORLD_SIZE", 1)) if world_size is None else world_size
            rank = int(os.environ.get("RANK", 0)) if rank is None else rank
            if init_method is None:
                addr = os.environ.get("MASTER_ADDR")
                init_method = f"tcp://{addr}:{os.environ.get('MASTER_PORT', '29500')}" if addr else "env://"
            if torch_backend == "nccl" and not torch.cuda.is_available():
                torch_backend = "gloo"
            if world_size > 1:
                kw = {}
                if torch_backend == "nccl":
                    kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
                dist.init_process_group(backend=torch_backend, init_method=init_method, world_size=world_size,
                                        rank=rank, **kw)
            self._initialized = dist.is_initialized()
        else:
            self._initialized = False
        self.group = group
        if self._initialized:
            self._rank = dist.get_rank(group)
            self._world_size = dist.get_world_size(group)
            self._backend_name = dist.get_backend(group)
        else:
            self._rank = rank if rank is not None else 0
            self._world_size = world_size if world_size is not None else 1
            self._backend_name = torch_backend
        self._node_rank = node_rank if node_rank is not None else int(os.environ.get("NODE_RANK", 0))
        self._num_nodes = num_nodes if num_nodes is not None else int(os.environ.get("NNODES", 1))
        self._context = DistributedContext(self._world_size, self._rank, self._node_rank, self._num_nodes,
                                           self._rank == 0, "torch")

    @property
    def rank(self) -> int:
        return self._rank

    @property
    def world_size(self) -> int:
        return self._world_size

    @property
    def node_rank(self) -> int:
        return self._node_rank

    @property
    def num_nodes(self) -> int:
        return self._num_nodes

    def get_context(self) -> DistributedContext:
        return self._context

    def is_initialized(self) -> bool:
        return self._initialized

    def _global(self, r: int) -> int:
        return r if self.group is None else dist.get_global_rank(self.group, r)

    def barrier(self) -> None:
        if self._initialized:
            dist.barrier(group=self.group)

    def broadcast(self, tensor: torch.Tensor, src: int = 0) -> torch.Tensor:
        if not self._initialized:
            return tensor.clone()
        tensor = tensor.contiguous()
        dist.broadcast(tensor, src=self._global(src), group=self.group)
        return tensor

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self._initialized:
            return obj
        box = [obj] if self._rank == src else [None]
        dist.broadcast_object_list(box, src=self._global(src), group=self.group)
        return box[0]

    def allreduce(self, tensor: torch.Tensor, op: ReduceOp = ReduceOp.SUM) -> torch.Tensor:
        if not self._initialized:
            return tensor.clone()
        return self.allreduce_inplace(tensor.clone().contiguous(), op)

    def allreduce_inplace(self, tensor: torch.Tensor, op: ReduceOp = ReduceOp.SUM) -> torch.Tensor:
        if not self._initialized:
            return tensor
        t = torch.view_as_real(tensor) if tensor.is_complex() else tensor
        dist.all_reduce(t, op=_op(op), group=self.group)
        if ReduceOp(op) == ReduceOp.AVG:
            tensor.div_(self._world_size)
        return tensor

    def allreduce_scalar(self, value: float, op: ReduceOp = ReduceOp.SUM, device=None) -> float:
        if device is None:
            device = torch.device("cuda" if (torch.cuda.is_available() and self._backend_name == "nccl") else "cpu")
        return float(self.allreduce(torch.tensor([value], device=device, dtype=torch.float64), op).item())

    def allgather(self, tensor: torch.Tensor) -> List[torch.Tensor]:
        if not self._initialized:
            return [tensor.clone()]
        tensor = tensor.contiguous()
        out = [torch.zeros_like(tensor) for _ in range(self._world_size)]
        dist.all_gather(out, tensor, group=self.group)
        return out

    def reduce_scatter(self, tensor: torch.Tensor, op: ReduceOp = ReduceOp.SUM) -> torch.Tensor:
        chunk = tensor.numel() // self._world_size
        if not self._initialized:
            return tensor.flatten()[:chunk].clone()
        out = torch.zeros(chunk, dtype=tensor.dtype, device=tensor.device)
        if dist.get_backend(self.group) == "gloo":
            # gloo has no reduce_scatter: all-reduce and keep this rank's chunk
            full = self.allreduce(tensor.flatten(), ReduceOp.SUM if ReduceOp(op) == ReduceOp.AVG else op)
            out.copy_(full[self._rank * chunk:(self._rank + 1) * chunk])
        else:
            dist.reduce_scatter(out, list(tensor.flatten()[:chunk * self._world_size].chunk(self._world_size)),
                                op=_op(op), group=self.group)
        if ReduceOp(op) == ReduceOp.AVG:
            out = out / self._world_size
        return out

    def send(self, tensor: torch.Tensor, dest: int, tag: int = 0) -> None:
        if self._initialized:
            dist.send(tensor.contiguous(), dst=self._global(dest), group=self.group, tag=tag)

    def recv(self, src: int, tag: int = 0, **kwargs) -> torch.Tensor:
        tensor = kwargs.get("tensor")
        if tensor is None:
            raise ValueError("tensor buffer is required for torch recv")
        if self._initialized:
            dist.recv(tensor, src=self._global(src), group=self.group, tag=tag)
        return tensor

    def isend(self, tensor: torch.Tensor, dest: int, tag: int = 0):
        if not self._initialized:
            return None
        return dist.isend(tensor.contiguous(), dst=self._global(dest), group=self.group, tag=tag)

    def irecv(self, src: int, tag: int = 0, **kwargs) -> Tuple[torch.Tensor, Any]:
        tensor = kwargs.get("tensor")
        if tensor is None:
            raise ValueError("tensor buffer is required for torch irecv")
        if not self._initialized:
            return tensor, None
        return tensor, dist.irecv(tensor, src=self._global(src), group=self.group, tag=tag)

    def allreduce_list_async(self, tensors: List[torch.Tensor], op: ReduceOp = ReduceOp.AVG) -> TorchAsyncHandle:
        if not self._initialized:
            return TorchAsyncHandle([], [t.clone() for t in tensors], op, self._world_size)
        works, outs = [], []
        for t in tensors:
            r = t.clone().contiguous()
            outs.append(r)
            works.append(dist.all_reduce(torch.view_as_real(r) if r.is_complex() else r, op=_op(op),
                                         group=self.group, async_op=True))
        return TorchAsyncHandle(works, outs, ReduceOp(op), self._world_size)

    def destroy(self) -> None:
        if self._initialized and self.group is None:
            dist.destroy_process_group()
            self._initialized = False


class MockCommTorch(CommBase):
    """comm_torch.py:563-666: single-process stand-in with a configurable rank / world size;
    every collective returns the local value."""

    def __init__(self, rank: Optional[int] = None, world_size: Optional[int] = None,
                 node_rank: Optional[int] = None, num_nodes: Optional[int] = None):
        self._rank = 0 if rank is None else rank
        self._world_size = 1 if world_size is None else world_size
        self._node_rank = 0 if node_rank is None else node_rank
        self._num_nodes = 1 if num_nodes is None else num_nodes
        self._context = DistributedContext(self._world_size, self._rank, self._node_rank, self._num_nodes,
                                           self._rank == 0, "torch")

    @property
    def rank(self) -> int:
        return self._rank

    @property
    def world_size(self) -> int:
        return self._world_size

    @property
    def node_rank(self) -> int:
        return self._node_rank

    @property
    def num_nodes(self) -> int:
        return self._num_nodes

    def get_context(self) -> DistributedContext:
        return self._context

    def is_initialized(self) -> bool:
        return False

    def barrier(self) -> None:
        pass

    def broadcast(self, tensor, src: int = 0):
        return tensor.clone()

    def broadcast_object(self, obj, src: int = 0):
        return obj

    def allreduce(self, tensor, op: ReduceOp = ReduceOp.SUM):
        return tensor.clone()

    def allreduce_inplace(self, tensor, op: ReduceOp = ReduceOp.SUM):
        return tensor

    def allreduce_scalar(self, value: float, op: ReduceOp = ReduceOp.SUM, device=None) -> float:
        return value

    def allgather(self, tensor):
        return [tensor.clone()]

    def reduce_scatter(self, tensor, op: ReduceOp = ReduceOp.SUM):
        return tensor.flatten()[:tensor.numel() // self._world_size].clone()

    def send(self, tensor, dest: int, tag: int = 0) -> None:
        pass

    def recv(self, src: int, tag: int = 0, **kwargs):
        t = kwargs.get("tensor")
        return torch.zeros(1) if t is None else t

    def isend(self, tensor, dest: int, tag: int = 0):
        return None

    def irecv(self, src: int, tag: int = 0, **kwargs):
        t = kwargs.get("tensor")
        return (torch.zeros(1) if t is None else t), None

    def allreduce_list(self, tensors, op: ReduceOp = ReduceOp.AVG):
        return [t.clone() for t in tensors]


class CommBackendType(Enum):
    """comm_factory.py:18-22."""
    MPI = "mpi"
    TORCH = "torch"
    MOCK = "mock"


def detect_best_backend() -> str:
    """comm_factory.py:170-208 without the MPI probes: "torch" when a process group is initialised
    or a launcher set WORLD_SIZE, else "mock"."""
    if dist.is_available() and dist.is_initialized():
        return "torch"
    if dist.is_available() and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return "torch"
    return "mock"


def get_comm_backend(backend: Union[str, CommBackendType] = "torch", **kwargs) -> CommBase:
    """comm_factory.py:25-82.  'torch' / 'pytorch' -> CommTorch (MockCommTorch when
    torch.distributed cannot be set up, as the reference falls back), 'mock' -> MockCommTorch,
    'auto' -> detect_best_backend(); 'mpi' raises (no mpi4py in this stack)."""
    if isinstance(backend, CommBackendType):
        backend = backend.value
    kind = str(backend).lower()
    if kind == "auto":
        kind = detect_best_backend()
    if kind in ("torch", "pytorch", "hip", "cuda"):
        try:
            return CommTorch(**{k: v for k, v in kwargs.items() if k in (
                "torch_backend", "init_method", "world_size", "rank", "node_rank", "num_nodes", "auto_init", "group")})
        except Exception as e:  # the reference's fallback (comm_factory.py:152-156)
            ws = kwargs.get("world_size") or int(os.environ.get("WORLD_SIZE", "1"))
            if ws > 1:
                # a multi-rank launch whose process group failed must not continue as a mock:
                # its collectives would silently be no-ops
                raise RuntimeError(f"torch.distributed could not be initialised for world size {ws}: {e}") from e
            print(f"Warning: PyTorch distributed not available ({e}), falling back to MockCommTorch")
            return MockCommTorch(kwargs.get("rank"), kwargs.get("world_size"), kwargs.get("node_rank"),
                                 kwargs.get("num_nodes"))
    if kind == "mock":
        return MockCommTorch(kwargs.get("rank"), kwargs.get("world_size"), kwargs.get("node_rank"),
                             kwargs.get("num_nodes"))
    if kind == "mpi":
        raise ValueError("the 'mpi' communicator needs mpi4py, which this stack does not use; "
                         "use 'torch' (RCCL / gloo through torch.distributed) or 'mock'")
    raise ValueError(f"Unknown backend type: {backend}. Supported: 'torch', 'mock', 'auto'")


def get_comm_torch(auto_init: bool = True, torch_backend: str = "nccl") -> CommBase:
    """comm_torch.py:669-683."""
    try:
        return CommTorch(torch_backend=torch_backend, auto_init=auto_init)
    except Exception as e:
        print(f"Warning: PyTorch distributed not available ({e}), falling back to MockCommTorch")
        return MockCommTorch()


def get_auto_backend(**kwargs) -> CommBase:
    return get_comm_backend("auto", **kwargs)


def get_mock_backend(**kwargs) -> CommBase:
    return get_comm_backend("mock", **kwargs)


def comm_group(comm):
    """The torch.distributed group behind `comm`: a CommBase's `group`, or `comm` itself when it is
    a process group (or None = WORLD)."""
    if isinstance(comm, CommBase):
        return comm.group
    return comm


def comm_rank_size(comm) -> Tuple[int, int]:
    """(rank, world size) of `comm`: the CommBase's own numbers, else the process group's (1 rank
    without an initialised group).  A mock runs no collectives (`comm_group` is WORLD), so a mock
    configured with world_size > 1 is refused here rather than set up as partitions whose
    exchanges would reach torch.distributed with no process group."""
    if isinstance(comm, MockCommTorch):
        if comm.world_size > 1:
            raise ValueError(f"MockCommTorch(world_size={comm.world_size}) runs no collectives; a multi-rank "
                             "engine needs a torch process group (CommTorch / get_comm_backend('torch'))")
        return 0, 1
    if isinstance(comm, CommBase):
        return comm.rank, comm.world_size
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(comm), dist.get_world_size(comm)
    return 0, 1
