"""Partitioned contraction across ranks with log2(W) merge stages.

Reference: DistributedEngineSiamese (tneq_qc/distributed/engine/distributed_engine.py)
  * _partition_qctn (:415-457): cores in QCTN order split into W contiguous partitions, the
    first `ncores % W` partitions one core larger (or a caller-given partition);
  * stage 0 (_contract_local :966-995): every rank contracts its own partition;
  * stages 1..ceil(log2 W) (_contract_reduce_stage :997-1069): in stage s groups of 2^s ranks
    merge the left half's tensor with the right half's over their shared bonds by a K-sharded
    partial matmul + all_reduce(SUM) inside the group (_tensor_parallel_matmul :1108-1664),
    with P2P shard exchanges, shape / scale handshakes and barriers around every stage.

MI355X design: the partition, every stage's equation and every shape are derived from the same
einsum on every rank, so no handshake or barrier is needed.  A stage is three collectives on the
group's process group (RCCL over xGMI on the node): broadcast of the left half's tensor from its
leader, broadcast of the right half's from its leader, and one all_reduce(SUM) of the partial
products.  The K-sharding reuses index slicing: the merge expression slices the contracted bond
legs and rank p of the group contracts slices p, p+G, ... on the native plan (slice-invariant
work hoisted, partial sums accumulated in place).  The result ends replicated on every rank of
the final group, in the global output's mode order.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..einsum import parse_equation


def partition_terms(n_terms: int, world: int, partitions: Optional[Sequence[Sequence[int]]] = None):
    """distributed_engine.py:415-457 over operand indices (cores in QCTN order)."""
    if partitions is not None:
        return [list(p) for p in partitions]
    if n_terms < world:
        return [[i] if i < n_terms else [] for i in range(world)]
    base, rem = divmod(n_terms, world)
    out, idx = [], 0
    for i in range(world):
        size = base + (1 if i < rem else 0)
        out.append(list(range(idx, idx + size)))
        idx += size
    return out


class _Stage:
    """One merge: left tensor (modes ml) x right tensor (modes mr) -> modes mo, K-sharded."""

    def __init__(self, s, g, ml, mr, mo, ext, sym, group_size):
        self.s, self.g, self.ml, self.mr, self.mo = s, g, ml, mr, mo
        contracted = [m for m in ml if m in mr and m not in mo]
        # slice the contracted legs (largest first) until there are >= group_size slices
        sl, n = [], 1
        for m in sorted(contracted, key=lambda m: -ext[m]):
            if n >= group_size:
                break
            sl.append(m)
            n *= ext[m]
        self.sliced = sl
        self.eq = ("".join(sym[m] for m in ml) + "," + "".join(sym[m] for m in mr) + "->"
                   + "".join(sym[m] for m in mo))
        self.shapes = (tuple(ext[m] for m in ml), tuple(ext[m] for m in mr))
        self.out_shape = tuple(ext[m] for m in mo)
        self.slice_syms = [sym[m] for m in sl]


class TreeContraction:
    """Runs einsum `eq` over `shapes` partitioned across the ranks of `group`.

    `executor(eq, shapes, operands, slices, slice_range)` contracts one (sub-)network and
    defaults to the native plan (HipContractExpression); CPU tests inject the oracle."""

    def __init__(self, eq: str, shapes: Sequence[Sequence[int]], group=None,
                 partitions: Optional[Sequence[Sequence[int]]] = None,
                 executor: Optional[Callable] = None, optimize="greedy"):
        self.net = parse_equation(eq, shapes)
        net = self.net
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.parts = partition_terms(len(net.terms), self.world, partitions)
        if len(self.parts) != self.world:
            raise ValueError(f"need one partition per rank ({self.world}), got {len(self.parts)}")
        self.optimize = optimize
        self.executor = executor
        ext, sym = net.extents, net.symbols
        # the global ranks of the group, in group-rank order
        self.granks = (list(range(self.world)) if group is None or not dist.is_initialized()
                       else [dist.get_global_rank(group, r) for r in range(self.world)])
        # modes each block carries: the modes of its terms still needed outside it
        owners: Dict[int, set] = {}
        for p, terms in enumerate(self.parts):
            for t in terms:
                for m in net.terms[t]:
                    owners.setdefault(m, set()).add(p)
        out = list(net.out)

        def keep(block_parts: set, modes: List[int]) -> List[int]:
            res = []
            for m in modes:
                if m in res:
                    continue
                if m in out or owners.get(m, set()) - block_parts:
                    res.append(m)
            return res

        # stage 0: rank p contracts its partition
        self.local = []
        for p, terms in enumerate(self.parts):
            modes = [m for t in terms for m in net.terms[t]]
            self.local.append(keep({p}, modes))
        # merge stages
        self.n_stages = int(math.ceil(math.log2(self.world))) if self.world > 1 else 0
        self.stages: List[List[Optional[_Stage]]] = []
        block = {p: self.local[p] for p in range(self.world)}      # leader -> modes
        for s in range(1, self.n_stages + 1):
            G, H = 2 ** s, 2 ** (s - 1)
            row = []
            for g in range(0, self.world, G):
                if g + H >= self.world:        # no right half: carried over unchanged
                    row.append(None)
                    continue
                ml, mr = block[g], block[g + H]
                parts = set(range(g, min(g + G, self.world)))
                final = s == self.n_stages
                mo = out if final else keep(parts, ml + mr)
                row.append(_Stage(s, g, ml, mr, mo, ext, sym, min(G, self.world - g)))
                block[g] = mo
                del block[g + H]
            self.stages.append(row)
        if self.world == 1:
            self.local[0] = out
        # stage exchanges are point-to-point within `group` (no per-stage process groups: they
        # would have to be created by every rank of the world, and `group` may be a subgroup)
        self._exprs = {}

    # -- execution -----------------------------------------------------------------------
    def _contract(self, key, eq, shapes, operands, slices=(), slice_range=None):
        if self.executor is not None:
            return self.executor(eq, shapes, operands, slices, slice_range)
        from ..expression import HipContractExpression
        e = self._exprs.get(key)
        if e is None:
            e = self._exprs[key] = HipContractExpression(eq, *shapes, optimize=self.optimize, slices=slices)
        if slice_range is not None and slice_range[0] >= e.n_slices:
            dt = operands[0].dtype
            for t in operands[1:]:
                dt = torch.promote_types(dt, t.dtype)
            return torch.zeros(e.out_shape, dtype=dt, device=operands[0].device)
        return e(*operands, slice_range=slice_range)

    def local_equation(self, p: int) -> Tuple[str, List[Tuple[int, ...]]]:
        net, sym = self.net, self.net.symbols
        terms = self.parts[p]
        eq = ",".join("".join(sym[m] for m in net.terms[t]) for t in terms)
        eq += "->" + "".join(sym[m] for m in self.local[p])
        return eq, [tuple(net.extents[m] for m in net.terms[t]) for t in terms]

    def __call__(self, *operands) -> torch.Tensor:
        """operands: all of the network's operands (replicated inputs; each rank reads its own)."""
        r = self.rank
        eq, shapes = self.local_equation(r)
        if self.parts[r]:
            cur = self._contract(("local", r), eq, shapes, [operands[t] for t in self.parts[r]])
        else:   # more ranks than operands: an empty partition is the scalar 1
            cur = torch.ones((), dtype=operands[0].dtype, device=operands[0].device)
        for row in self.stages:
            for st in row:
                if st is None:
                    continue
                G = min(2 ** st.s, self.world - st.g)
                if not (st.g <= r < st.g + G):
                    continue
                pos = r - st.g
                H = 2 ** (st.s - 1)
                members = [self.granks[q] for q in range(st.g, st.g + G)]
                left = cur if pos < H else torch.empty(st.shapes[0], dtype=cur.dtype, device=cur.device)
                right = cur if pos >= H else torch.empty(st.shapes[1], dtype=cur.dtype, device=cur.device)
                left, right = left.contiguous(), right.contiguous()
                # the left block (leader st.g) and the right block (leader st.g + H) to every
                # member (the reference's SendRecvGrad exchange, distributed_engine.py:1697-1766)
                _p2p_bcast([left, right], [members[0], members[H]], members, self.granks[r], self.group)
                part = self._contract(("stage", st.s, st.g), st.eq, st.shapes, [left, right],
                                      st.slice_syms, (pos, None, G)).contiguous()
                # sum of the members' K-shard partials (allreduce_grad.py:13-60), in member order
                _p2p_allreduce(part, members, self.granks[r], self.group)
                cur = part
        return cur


def _view(t: torch.Tensor) -> torch.Tensor:
    return torch.view_as_real(t) if t.is_complex() else t


def _staged(t: torch.Tensor, group) -> bool:
    """gloo moves host memory only: device tensors go through a host copy there (RCCL takes
    them directly)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _p2p_bcast(tensors, srcs, members, me, group):
    """tensors[i] from global rank srcs[i] to every other member: receives posted first, then
    sends, then one wait (no ordering deadlock)."""
    reqs, back = [], []
    for t, src in zip(tensors, srcs):
        if me != src:
            buf = torch.empty(t.shape, dtype=t.dtype) if _staged(t, group) else t
            reqs.append(dist.irecv(_view(buf), src=src, group=group))
            if buf is not t:
                back.append((buf, t))
    for t, src in zip(tensors, srcs):
        if me == src:
            buf = t.cpu() if _staged(t, group) else t
            for m in members:
                if m != src:
                    reqs.append(dist.isend(_view(buf), dst=m, group=group))
    for q in reqs:
        q.wait()
    for buf, t in back:
        t.copy_(buf)


def _p2p_allreduce(t: torch.Tensor, members, me, group):
    """In-place SUM over the members: the leader adds the partials in member order and sends
    the total back (deterministic; a stage group holds at most 2^s ranks)."""
    if len(members) == 1:
        return
    lead = members[0]
    host = t.cpu() if _staged(t, group) else t
    v = _view(host)
    if me == lead:
        bufs = [torch.empty_like(v) for _ in members[1:]]
        reqs = [dist.irecv(b, src=m, group=group) for b, m in zip(bufs, members[1:])]
        for q in reqs:
            q.wait()
        for b in bufs:
            v += b
        reqs = [dist.isend(v, dst=m, group=group) for m in members[1:]]
    else:
        dist.isend(v, dst=lead, group=group).wait()
        reqs = [dist.irecv(v, src=lead, group=group)]
    for q in reqs:
        q.wait()
    if host is not t:
        t.copy_(host)
