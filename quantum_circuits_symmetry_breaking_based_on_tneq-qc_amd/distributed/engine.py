"""DistributedEngineSiamese drop-in (tneq_qc/distributed/engine/distributed_engine.py:188-2131).

The reference's caller API, unchanged:
    engine = DistributedEngineSiamese(backend=...)
    plan = engine.init_distributed(qctn, partitions=None)              # :368-415
    result = engine.contract_distributed(states, measure_inputs)       # :876-964
    loss, grads = engine.contract_distributed_with_gradient(...)       # :1866-1984
    engine.train_step(states, measure_inputs, optimizer)               # :2021-2056

What it computes: the L·M·R sandwich that EngineSiamese.contract_with_compiled_strategy
computes for the whole QCTN (greedy_strategy.py:41-1080: states, cores, Mx, conj cores,
states), split across the ranks by the reference's partition rule (cores in QCTN order into W
contiguous blocks, :415-457).  Rank p owns the L and R copies of its cores, the circuit state of
every qubit whose input edge lands on one of its cores and the Mx of every qubit whose output
edge leaves one of them (the reference's local-state / local-Mx extraction, :905-931).

MI355X design (distributed/tree.py): the sandwich is ONE flat einsum (contractor/
greedy_symbolic.py replays the reference's group sweep on axis labels); stage 0 contracts a
rank's own operands on the native plan (the reference: the greedy strategy on the local QCTN,
:966-995), the merge stages exchange blocks point-to-point in one batched round and K-shard the
merge by index slicing, partials summed at the stage leader with TNTensor log-scales aligned
(:1108-1664, :1437-1472).  No shape handshakes or barriers (every rank derives every shape from
the same equation), no per-stage process groups.

Deviations, on purpose:
  * the Born rule (|.|^2 of a complex result, engine_siamese.py:332-349) is applied to the FINAL
    sandwich, as the single-process contract_with_compiled_strategy does; the reference applies
    it to every rank's stage-0 partial (its _contract_local asks for ret_type='TNTensor'), which
    for complex cores is not the Born rule of the network (for real cores, where no |.|^2 is
    taken, both agree);
  * the returned TNTensor carries a scale consistent with its log_scale (the reference returns
    TNTensor(result, log_scale=...) with scale left at 1.0);
  * no process group is required at world size 1.
Gradients follow the reference exactly: the exchanges and sums carry their adjoints, so with the
same loss on every rank a rank's gradient is W x the single-process gradient of its cores.
"""
from __future__ import annotations

import math
from copy import deepcopy
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from ..contractor.greedy_symbolic import greedy_equation
from ..core.tn_tensor import TNTensor
from .comm import comm_group, comm_rank_size, get_comm_backend
from .tree import TreeContraction


@dataclass
class PartitionConfig:
    """distributed_engine.py:35-49."""
    strategy: str = "layer"
    num_partitions: int = 1
    min_cores_per_partition: int = 1
    balance_partitions: bool = True


@dataclass
class ContractStage:
    """distributed_engine.py:52-82."""
    stage_idx: int
    stage_type: str
    local_cores: List[str] = field(default_factory=list)
    group_ranks: List[int] = field(default_factory=list)
    group_size: int = 1
    is_group_leader: bool = False
    partner_rank: int = -1


@dataclass
class DistributedContractPlan:
    """distributed_engine.py:85-185."""
    num_stages: int
    stages: List[ContractStage] = field(default_factory=list)
    local_partition_idx: int = 0
    local_cores: List[str] = field(default_factory=list)
    inter_node_graph: Optional[Dict[str, Any]] = None


class _LocalQCTN:
    """The rank's partition as the reference builds it (_create_local_qctn :728-807): its cores,
    their weights (the optimizer updates these), their adjacency entries."""

    def __init__(self, qctn, cores, table, rank):
        self.graph = None
        self.nqubits = qctn.nqubits
        self.cores = list(cores)
        self.ncores = len(self.cores)
        self.adjacency_table = table
        self.cores_weights = {c: qctn.cores_weights[c] for c in self.cores if c in qctn.cores_weights}
        self.backend = getattr(qctn, "backend", None)
        self.partition_idx = rank
        qs = sorted({e["qubit_idx"] for t in table for e in t["in_edge_list"] + t["out_edge_list"]})
        self.qubit_indices = qs if rank == 0 else qs[::-1]


def _present(container, q) -> bool:
    if container is None:
        return False
    if isinstance(container, dict):
        return q in container
    return q < len(container)


class DistributedEngineSiamese:
    def __init__(self, backend=None, strategy_mode: str = "balanced", mx_K: int = 100, comm=None,
                 partition_config: Optional[PartitionConfig] = None, comm_timeout: float = 300.0,
                 enable_comm_retry: bool = True, max_comm_retries: int = 3,
                 executor: Optional[Callable] = None):
        """`comm`: the reference's communicator (`distributed.comm.CommTorch` / `MockCommTorch`,
        as `get_comm_backend('torch' | 'mock' | 'auto')` builds it for `distributed_trainer.py:228-233`)
        or a torch.distributed process group; None = `get_comm_backend('auto')` (WORLD when a group
        is initialised, else a 1-rank mock) as the reference's `comm or get_comm_backend(...)`
        (`:248`).  Collectives run on the communicator's group.  `executor` is passed to
        TreeContraction (None = the native plan; CPU tests inject a torch executor)."""
        self._backend_arg = backend
        self.strategy_mode = strategy_mode
        self.mx_K = mx_K
        self._base = None
        self.comm = comm if comm is not None else get_comm_backend("auto")
        self.group = comm_group(self.comm)
        self.rank, self.world_size = comm_rank_size(self.comm)
        self.comm_timeout = comm_timeout
        self.enable_comm_retry = enable_comm_retry
        self.max_comm_retries = max_comm_retries
        self.partition_config = partition_config or PartitionConfig(num_partitions=self.world_size)
        self.num_stages = math.ceil(math.log2(self.world_size)) + 1 if self.world_size > 1 else 1
        self.executor = executor
        self._is_initialized = False
        self._qctn = None
        self._local_qctn: Optional[_LocalQCTN] = None
        self._contract_plan: Optional[DistributedContractPlan] = None
        self._jobs: Dict[tuple, tuple] = {}
        self._last_job = None

    # ---------------------------------------------------------------- proxies (:334-365)
    @property
    def _base_engine(self):
        if self._base is None:
            from ..core.engine_siamese import EngineSiamese
            self._base = EngineSiamese(backend=self._backend_arg, strategy_mode=self.strategy_mode,
                                       mx_K=self.mx_K)
        return self._base

    @property
    def backend(self):
        return self._base_engine.backend

    @property
    def contractor(self):
        return self._base_engine.contractor

    @property
    def strategy_compiler(self):
        return self._base_engine.strategy_compiler

    def generate_data(self, x, K=None, ret_type="tensor"):
        return self._base_engine.generate_data(x, K=K, ret_type=ret_type)

    def contract_with_compiled_strategy(self, qctn, circuit_states_list, measure_input_list=None, **kw):
        return self._base_engine.contract_with_compiled_strategy(qctn, circuit_states_list, measure_input_list, **kw)

    def contract_with_compiled_strategy_for_gradient(self, qctn, circuit_states_list=None,
                                                     measure_input_list=None, **kw):
        return self._base_engine.contract_with_compiled_strategy_for_gradient(
            qctn, circuit_states_list, measure_input_list, **kw)

    def is_main_process(self) -> bool:
        return self.rank == 0

    def check_comm_health(self, timeout: float = 5.0) -> bool:
        """:293-332: an all-gather of the ranks' ids."""
        if self.world_size == 1:
            return True
        dev = torch.device("cpu")
        if dist.get_backend(self.group) != "gloo":
            dev = torch.device("cuda", torch.cuda.current_device())
        t = torch.tensor([float(self.rank)], device=dev)
        out = [torch.zeros_like(t) for _ in range(self.world_size)]
        dist.all_gather(out, t, group=self.group)
        return abs(sum(float(x) for x in out) - sum(range(self.world_size))) < 1e-6

    # ---------------------------------------------------------------- init (:368-807)
    def init_distributed(self, qctn, partitions=None) -> DistributedContractPlan:
        self._qctn = qctn
        parts = self._partition_qctn(qctn, partitions)
        if len(parts) != self.world_size:
            raise ValueError(f"need one partition per rank ({self.world_size}), got {len(parts)}")
        plan = self._compute_contract_plan(qctn, parts)
        local = parts[self.rank] if self.rank < len(parts) else []
        plan.local_partition_idx = self.rank
        plan.local_cores = list(local)
        plan.stages[0].local_cores = list(local)
        self._contract_plan = plan
        self._partitions = parts
        tables = plan.inter_node_graph["partition_adjacency_tables"]
        self._local_qctn = _LocalQCTN(qctn, local, tables[self.rank], self.rank) if local else None
        self._jobs.clear()
        self._is_initialized = True
        return plan

    def _partition_qctn(self, qctn, partitions=None) -> List[List[str]]:
        """:417-457: cores in QCTN order, W contiguous blocks, the first ncores % W one larger."""
        if partitions is not None:
            return [list(p) for p in partitions]
        n = self.partition_config.num_partitions
        cores = list(qctn.cores)
        if len(cores) < n:
            return [[cores[i]] if i < len(cores) else [] for i in range(n)]
        base, rem = divmod(len(cores), n)
        out, idx = [], 0
        for i in range(n):
            size = base + (1 if i < rem else 0)
            out.append(cores[idx:idx + size])
            idx += size
        return out

    def _compute_contract_plan(self, qctn, partitions) -> DistributedContractPlan:
        """:459-595: stage list + the cross-partition edges and per-partition tables."""
        n = self.world_size
        n_reduce = int(math.ceil(math.log2(n))) if n > 1 else 0
        stages = [ContractStage(0, "local", local_cores=list(partitions[0]) if partitions else [])]
        for s in range(1, 1 + n_reduce):
            G = 2 ** s
            g0 = (self.rank // G) * G
            ranks = list(range(g0, min(g0 + G, n)))
            H = G // 2
            pos = self.rank - g0
            partner = (g0 + pos + H) if pos < H else (g0 + pos - H)
            stages.append(ContractStage(s, "reduce", group_ranks=ranks, group_size=G,
                                        is_group_leader=pos == 0,
                                        partner_rank=partner if partner < n else -1))
        where = {c: p for p, cs in enumerate(partitions) for c in cs}
        at = {c: i for cs in partitions for i, c in enumerate(cs)}
        raw, cross = [], []
        for info in qctn.adjacency_table:
            c = info["core_name"]
            for e in info["out_edge_list"]:
                nb = e["neighbor_name"]
                if nb and nb in where and where[c] != where[nb]:
                    raw.append({"from_core": c, "to_core": nb, "from_partition": where[c],
                                "to_partition": where[nb], "edge_rank": e["edge_rank"], "qubit_idx": e["qubit_idx"]})
                    cross.append({"from_core": f"P{where[c]}", "to_core": f"P{where[nb]}",
                                  "from_partition": where[c], "to_partition": where[nb],
                                  "from_core_idx": at[c], "to_core_idx": at[nb],
                                  "edge_rank": e["edge_rank"], "qubit_idx": e["qubit_idx"],
                                  "from_core_raw": c, "to_core_raw": nb})
        tables = []
        for p, cs in enumerate(partitions):
            tab = []
            for info in qctn.adjacency_table:
                if info["core_name"] not in cs:
                    continue
                ent = deepcopy(info)
                for e in ent["in_edge_list"] + ent["out_edge_list"]:
                    e["is_cross_partition"] = bool(e["neighbor_name"]) and where.get(e["neighbor_name"]) != p
                tab.append(ent)
            tables.append(tab)
        graph = {"raw_cross_edges": raw, "cross_edges": cross, "partition_adjacency_tables": tables,
                 "num_partitions": len(partitions), "partition_sizes": [len(p) for p in partitions]}
        return DistributedContractPlan(num_stages=1 + n_reduce, stages=stages, inter_node_graph=graph)

    # ---------------------------------------------------------------- contraction (:876-1069)
    def _job(self, states, mx, cores):
        qctn = self._qctn
        key = (tuple((q, tuple(s.shape)) for q, s in states.items()),
               tuple((q, tuple(m.shape)) for q, m in mx.items()),
               tuple((c, tuple(t.shape)) for c, t in cores.items()))
        hit = self._jobs.get(key)
        if hit is not None:
            return hit
        eq, recipe = greedy_equation(
            qctn, {q: s.shape[0] for q, s in states.items()},
            {q: (m.ndim, m.shape[-2], m.shape[-1]) for q, m in mx.items()},
            {c: len(t.shape) for c, t in cores.items()}, "symmetric")
        shape_of = {("S", q): tuple(s.shape) for q, s in states.items()}
        shape_of.update({("M", q): tuple(m.shape) for q, m in mx.items()})
        for c, t in cores.items():
            shape_of[("L", c)] = shape_of[("R", c)] = tuple(t.shape)
        shapes = [shape_of[r] for r in recipe]
        # owners: a core's partition; a state -> the core holding the qubit's input edge, an Mx
        # -> the core holding its output edge (distributed_engine.py:905-931)
        where = {c: p for p, cs in enumerate(self._partitions) for c in cs}
        first, last = {}, {}
        for info in qctn.adjacency_table:
            for e in info["in_edge_list"]:
                if e["neighbor_idx"] == -1:
                    first[e["qubit_idx"]] = where[info["core_name"]]
            for e in info["out_edge_list"]:
                if e["neighbor_idx"] == -1:
                    last[e["qubit_idx"]] = where[info["core_name"]]
        parts = [[] for _ in range(self.world_size)]
        for i, (kind, k) in enumerate(recipe):
            p = where[k] if kind in ("L", "R") else (first.get(k, 0) if kind == "S" else last.get(k, 0))
            parts[p].append(i)
        job = TreeContraction(eq, shapes, group=self.group, partitions=parts, executor=self.executor)
        hit = (job, recipe)
        self._jobs[key] = hit
        return hit

    def contract_distributed(self, circuit_states_list, measure_input_list, measure_is_matrix: bool = True):
        """:876-964 -> TNTensor when a core is a TNTensor (else a tensor), replicated on every
        rank: the Born rule of the whole sandwich (see the module docstring)."""
        if not self._is_initialized:
            raise RuntimeError("Must call init_distributed() before contract_distributed()")
        qctn = self._qctn
        qs = qctn.qubit_indices
        states = {q: circuit_states_list[q] for q in qs if _present(circuit_states_list, q)}
        mx = {q: measure_input_list[q] for q in qs
              if _present(measure_input_list, q) and measure_input_list[q] is not None}
        local = self._local_qctn.cores_weights if self._local_qctn is not None else {}
        # shapes of every core (remote ones from the full QCTN: only their shapes are read)
        cores = {c: local.get(c, qctn.cores_weights.get(c)) for c in qctn.cores}
        job, recipe = self._job(states, mx, cores)
        mine = set(job.parts[self.rank])
        ops: List[Any] = []
        for i, (kind, k) in enumerate(recipe):
            if i not in mine:
                ops.append(None)
                continue
            if kind in ("L", "R"):
                t = cores[k]
                if kind == "R":
                    raw = t.tensor if isinstance(t, TNTensor) else t
                    if raw.is_complex():
                        raw = raw.conj_physical()
                    t = TNTensor(raw, t.scale, t.log_scale) if isinstance(t, TNTensor) else raw
            elif kind == "S":
                t = states[k]
            else:
                t = mx[k]
            ops.append(t)
        if not mine:   # an empty partition still needs a dtype / device to build its scalar 1
            ref = next(iter(cores.values()))
            ops[0] = ref.tensor if isinstance(ref, TNTensor) else ref
        if not mine and torch.is_grad_enabled():
            # an empty partition joins the backward through TreeContraction.leaf
            ops[0] = ops[0].detach().requires_grad_() if not ops[0].requires_grad else ops[0]
        res = job(*ops)
        self._last_job = job
        if isinstance(res, TNTensor):
            if res.tensor.is_complex():
                return TNTensor(res.tensor.abs() ** 2, res.scale, res.log_scale)
            return res
        return res.abs() ** 2 if res.is_complex() else res

    # ---------------------------------------------------------------- gradients (:1866-2056)
    def contract_distributed_with_gradient(self, circuit_states_list, measure_input_list,
                                           measure_is_matrix: bool = True, target=None):
        """(loss, grads of the local partition's cores) with the reference's cross-entropy loss
        -mean(target * (log(clamp(P, 1e-10)) + log_scale)) (:1986-2019)."""
        raws = []
        for name in (self._local_qctn.cores if self._local_qctn is not None else []):
            w = self._local_qctn.cores_weights[name]
            t = w.tensor if isinstance(w, TNTensor) else w
            t.requires_grad_(True)
            if t.grad is not None:
                t.grad.zero_()
            raws.append(t)
        result = self.contract_distributed(circuit_states_list, measure_input_list, measure_is_matrix)
        loss = self._compute_cross_entropy_loss(result, target)
        job = self._last_job
        extra = [job.leaf] if job is not None and job.leaf is not None else []   # an empty partition
        grads = torch.autograd.grad(loss, raws + extra, allow_unused=True)[:len(raws)]
        return loss, [torch.zeros_like(t) if g is None else g.contiguous() for g, t in zip(grads, raws)]

    @staticmethod
    def _compute_cross_entropy_loss(result, target=None):
        if isinstance(result, TNTensor):
            res, ls = result.tensor, result.log_scale
        else:
            res, ls = result, 0.0
        if target is None:
            target = torch.ones_like(res)
        return -torch.mean(target * (torch.log(torch.clamp(res, min=1e-10)) + ls))

    def train_step(self, circuit_states_list, measure_input_list, optimizer, measure_is_matrix: bool = True,
                   target=None) -> float:
        """:2021-2056: forward + backward, then optimizer.step(local_qctn, grads)."""
        loss, grads = self.contract_distributed_with_gradient(circuit_states_list, measure_input_list,
                                                              measure_is_matrix, target)
        optimizer.step(self._local_qctn, grads)
        return float(loss.detach())
