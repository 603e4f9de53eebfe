"""Partitioned contraction across ranks with log2(W) merge stages.

Reference: DistributedEngineSiamese (tneq_qc/distributed/engine/distributed_engine.py)
  * _partition_qctn (:415-457): cores in QCTN order split into W contiguous partitions, the
    first `ncores % W` partitions one core larger (or a caller-given partition);
  * stage 0 (_contract_local :966-995): every rank contracts its own partition;
  * stages 1..ceil(log2 W) (_contract_reduce_stage :997-1069): in stage s groups of 2^s ranks
    merge the left half's tensor with the right half's over their shared bonds by a K-sharded
    partial matmul + all_reduce(SUM) inside the group (_tensor_parallel_matmul :1108-1664),
    with P2P shard exchanges (SendRecvGrad, allreduce_grad.py:149-207), TNTensor log-scale
    exchange + max alignment (:1437-1472), shape handshakes and barriers around every stage;
  * the whole pipeline is differentiable (contract_distributed_with_gradient :1866-1984): the
    exchanges and the all-reduce carry their adjoints (allreduce_grad.py:13-60, 149-207).

MI355X design: the partition, every stage's equation and every shape are derived from the same
einsum on every rank, so no handshake or barrier is needed.  A stage is two point-to-point
rounds inside the group, each issued as ONE batch (dist.batch_isend_irecv: a single
ncclGroupStart/End under RCCL, so a pair's send and receive cannot block each other): the left
half's leader sends its block (and its log-scale) to every member, the right half's leader its
block; then the members' K-shard partials are summed at the stage leader (log-scales aligned to
the max, as the reference) and the total sent back.  The K-sharding reuses index slicing: the
merge expression slices the contracted bond legs and rank p of the group contracts slices p,
p+G, ... on the native plan.  The result ends replicated on every rank of the final group, in the
global output's mode order.

Gradients (torch autograd): `_StageExchange` and `_StageReduce` are autograd Functions whose
backward is the exact adjoint of their forward (the block broadcast's adjoint sums the members'
gradients at the sending leader; the reduce's adjoint sums the members' output gradients and
returns the total to every member), the local and K-shard contractions differentiate through the
native reverse tree (HipContractExpression, sliced ranges included).  As in the reference, the
gradient a rank receives is that of the SUM of every rank's loss: when each rank computes the
same loss on the replicated result, W x the single-process gradient.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..core.tn_tensor import TNTensor
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
    defaults to the native plan (HipContractExpression); CPU tests inject the oracle (or, for
    gradients, a differentiable torch executor).  Operands may be TNTensors: their scales are
    carried as log-scales through the stages and the result is a TNTensor.

    Gradients: every rank must run its backward (the stage adjoints are collectives); a rank
    whose partition is empty differentiates w.r.t. `self.leaf` (its scalar 1), since
    torch.autograd.grad only runs the nodes on a path to the requested inputs.

    `scaled`: whether log-scales travel with the stage blocks (TNTensor operands).  Every rank of
    the group must agree -- a rank sees only its own partition's operands -- so it is either
    given here or agreed on the first call by one all-reduce (MAX) of the ranks' "I hold a
    TNTensor" flags, then fixed: a later call with TNTensor operands on an unscaled contraction
    raises instead of posting messages the other ranks would never match."""

    def __init__(self, eq: str, shapes: Sequence[Sequence[int]], group=None,
                 partitions: Optional[Sequence[Sequence[int]]] = None,
                 executor: Optional[Callable] = None, optimize="greedy", scaled: Optional[bool] = None):
        self.scaled = scaled
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
        self._warm = False

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

    def __call__(self, *operands):
        """operands: all of the network's operands in equation order; a rank reads only those of
        its own partition (the others may be None).  TNTensor operands -> TNTensor result."""
        r = self.rank
        mine = self.parts[r]
        ref = next(o for o in operands if o is not None)
        ref = ref.tensor if isinstance(ref, TNTensor) else ref
        tn_here = any(isinstance(o, TNTensor) for o in operands if o is not None)
        if self.scaled is None:
            self.scaled = _agree_any(tn_here, ref, self.group) if self.world > 1 else tn_here
        elif tn_here and not self.scaled:
            raise ValueError("TreeContraction: TNTensor operands on a contraction agreed unscaled (its first "
                             "call had none on any rank); construct it with scaled=True")
        tn = self.scaled
        raw, log_scale, sign = [], 0.0, 1.0
        for t in mine:
            o = operands[t]
            if isinstance(o, TNTensor):
                log_scale += o.log_scale
                sign = -sign if o.scale < 0 else sign
                o = o.tensor
            raw.append(o)
        # autograd when an operand requires grad (an empty partition looks at every operand it
        # was given: its rank still has to run the stage adjoints in backward)
        pool = raw if mine else [o.tensor if isinstance(o, TNTensor) else o for o in operands if o is not None]
        grad = torch.is_grad_enabled() and any(getattr(o, "requires_grad", False) for o in pool)
        self.leaf = None
        if self.world > 1 and not self._warm:
            _first_use(ref, self.group)
            self._warm = True
        eq, shapes = self.local_equation(r)
        if mine:
            cur = self._contract(("local", r), eq, shapes, raw)
        else:   # more ranks than operands: an empty partition is the scalar 1
            cur = torch.ones((), dtype=ref.dtype, device=ref.device)
            if grad:
                # the rank's backward must reach the stage Functions: differentiate w.r.t. this
                # leaf (torch.autograd.grad only runs the nodes on a path to its inputs)
                cur.requires_grad_()
                self.leaf = cur
        if sign < 0:
            cur = -cur
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
                meta = _StageMeta(members, H, self.granks[r], self.group, st.shapes, cur.dtype, cur.device, tn)
                # the left block (leader st.g) and the right block (leader st.g + H) to every
                # member (the reference's SendRecvGrad exchange, distributed_engine.py:1697-1766),
                # with their log-scales
                sides = [k for k in (0, 1) if meta.me != meta.leads[k]]
                if grad:
                    *recv, logs = _StageExchange.apply(cur, meta, log_scale)
                    rec, logs = dict(zip(sides, recv)), logs.tolist()
                else:
                    got = _exchange(cur.detach(), meta, log_scale)
                    rec = {k: t for k, (t, _) in got.items()}
                    logs = [got[k][1] if k in got else log_scale for k in (0, 1)]
                left, right, log_l, log_r = _blocks(cur, rec, logs)
                part = self._contract(("stage", st.s, st.g), st.eq, st.shapes, [left, right],
                                      st.slice_syms, (pos, None, G))
                if grad and not part.requires_grad:
                    # a member without a K shard (fewer slices than members) still runs the
                    # stage adjoints in backward: keep its zero partial on the graph
                    part = part + 0 * sum(x.sum() for x in (left, right) if x.requires_grad)
                # sum of the members' K-shard partials (allreduce_grad.py:13-60), in member
                # order, log-scales aligned to the max (distributed_engine.py:1462-1472)
                pair = log_l + log_r
                if grad:
                    cur, log_scale = _StageReduce.apply(part.contiguous(), meta, pair)
                    log_scale = float(log_scale)
                else:
                    cur, log_scale = _reduce(part.detach().contiguous(), meta, pair)
        if tn:
            return TNTensor(cur, scale=_exp(log_scale), log_scale=log_scale)
        if log_scale != 0.0:
            cur = cur * _exp(log_scale)
        return cur


def _exp(x: float) -> float:
    return math.exp(x) if x < 709.0 else float("inf")


class _StageMeta:
    """Static description of one stage as seen by one member."""
    __slots__ = ("members", "me", "group", "shapes", "dtype", "device", "H", "scaled")

    def __init__(self, members, H, me, group, shapes, dtype, device, scaled=True):
        self.members, self.H, self.me, self.group = members, H, me, group
        self.shapes, self.dtype, self.device = shapes, dtype, device
        # log-scales travel with the blocks only when the call has TNTensor operands (every
        # rank passes the same operand kinds); otherwise they are all 0: no extra messages and
        # no host reads (.item()), so a plain distributed step stays asynchronous
        self.scaled = scaled

    @property
    def leads(self):
        """(left leader, right leader): global ranks of members[0] and members[H]."""
        return self.members[0], self.members[self.H]


def _view(t: torch.Tensor) -> torch.Tensor:
    return torch.view_as_real(t) if t.is_complex() else t


def _staged(t: torch.Tensor, group) -> bool:
    """gloo moves host memory only: device tensors go through a host copy there (RCCL takes
    them directly)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _agree_any(flag: bool, ref: torch.Tensor, group) -> bool:
    """True on every rank of `group` when `flag` is True on any (one all-reduce MAX)."""
    on_dev = ref.is_cuda and dist.get_backend(group) != "gloo"
    t = torch.tensor([1.0 if flag else 0.0], device=ref.device if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(t.item() > 0)


def _first_use(ref: torch.Tensor, group):
    """Under RCCL the first batched point-to-point call of a group must involve all of its ranks
    (torch.distributed.batch_isend_irecv): a tiny all-reduce on the group initialises its
    communicator before any stage subset talks."""
    if dist.get_backend(group) == "gloo":
        return
    dist.all_reduce(torch.zeros(1, device=ref.device), group=group)


def _p2p(ops, group):
    """ops: (kind 'send'|'recv', tensor, global peer).  Issued as ONE batch and waited for."""
    if not ops:
        return
    p2p = [dist.P2POp(dist.isend if k == "send" else dist.irecv, _view(t), peer, group)
           for k, t, peer in ops]
    for q in dist.batch_isend_irecv(p2p):
        q.wait()


class _Wire:
    """Device tensors as they travel: host copies under gloo, the tensors themselves under RCCL."""

    def __init__(self, group):
        self.group = group
        self.back = []

    def out(self, t):
        return t.cpu() if _staged(t, self.group) else t

    def into(self, shape, dtype, device):
        probe = torch.empty((), dtype=dtype, device=device)
        if _staged(probe, self.group):
            buf = torch.empty(shape, dtype=dtype)
            dst = torch.empty(shape, dtype=dtype, device=device)
            self.back.append((buf, dst))
            return buf, dst
        buf = torch.empty(shape, dtype=dtype, device=device)
        return buf, buf

    def finish(self):
        for buf, dst in self.back:
            dst.copy_(buf)


def _exchange(cur, meta: _StageMeta, log_scale: float):
    """Forward of the block broadcast: returns {0: (left, log), 1: (right, log)} for the blocks
    this rank receives (a leader keeps its own)."""
    mem, me = meta.members, meta.me
    leads = meta.leads
    w = _Wire(meta.group)
    ops, got = [], {}
    for side, src in enumerate(leads):
        if me == src:
            payload = w.out(cur.contiguous())
            ls = w.out(torch.tensor([log_scale], dtype=torch.float64, device=cur.device)) if meta.scaled else None
            for m in mem:
                if m != src:
                    ops.append(("send", payload, m))
                    if meta.scaled:
                        ops.append(("send", ls, m))
        else:
            buf, dst = w.into(meta.shapes[side], meta.dtype, meta.device)
            ops.append(("recv", buf, src))
            ldst = None
            if meta.scaled:
                lbuf, ldst = w.into((1,), torch.float64, meta.device)
                ops.append(("recv", lbuf, src))
            got[side] = (dst, ldst)
    _p2p(ops, meta.group)
    w.finish()
    return {side: (t, float(ls.item()) if ls is not None else 0.0) for side, (t, ls) in got.items()}


def _blocks(cur, rec: Dict[int, torch.Tensor], logs: Sequence[float]):
    """(left, right, log_left, log_right) on this rank: the received blocks, its own for the
    side it leads."""
    left = rec.get(0, cur)
    right = rec.get(1, cur)
    return left, right, float(logs[0]), float(logs[1])


class _StageExchange(torch.autograd.Function):
    """Block broadcast with its adjoint (SendRecvGrad, allreduce_grad.py:149-207): forward sends
    a leader's block to every member of the stage; backward returns to each leader the sum of the
    members' gradients of its block."""

    @staticmethod
    def forward(ctx, cur, meta: _StageMeta, log_scale: float):
        got = _exchange(cur.detach(), meta, log_scale)
        ctx.meta = meta
        ctx.sides = sorted(got)
        ctx.cur_meta = (tuple(cur.shape), cur.dtype, cur.device)
        logs = torch.tensor([log_scale if meta.me == src else got[k][1]
                             for k, src in enumerate(meta.leads)], dtype=torch.float64)
        ctx.mark_non_differentiable(logs)
        return (*[got[k][0] for k in ctx.sides], logs)

    @staticmethod
    def backward(ctx, *grads):
        meta = ctx.meta
        mem, me = meta.members, meta.me
        shape, dtype, device = ctx.cur_meta
        gs = dict(zip(ctx.sides, grads[:len(ctx.sides)]))
        w = _Wire(meta.group)
        ops, acc = [], []
        for side, src in enumerate(meta.leads):
            if me == src:
                for m in mem:
                    if m != src:
                        buf, dst = w.into(shape, dtype, device)
                        ops.append(("recv", buf, m))
                        acc.append(dst)
            else:
                g = gs.get(side)
                g = torch.zeros(meta.shapes[side], dtype=meta.dtype, device=meta.device) if g is None else g
                ops.append(("send", w.out(g.contiguous()), src))
        _p2p(ops, meta.group)
        w.finish()
        total = torch.zeros(shape, dtype=dtype, device=device)
        for a in acc:       # member order: deterministic
            total = total + a
        return total, None, None


def _reduce(part, meta: _StageMeta, log_scale: float):
    """Sum of the members' partials at the leader, log-scales aligned to their max, the total
    (and the common log-scale) sent back to every member.  Returns (total, log_scale)."""
    mem, me = meta.members, meta.me
    if len(mem) == 1:
        return part, log_scale
    lead = mem[0]
    sc = meta.scaled
    w = _Wire(meta.group)
    if me == lead:
        bufs, lbufs, ops = [], [], []
        for m in mem[1:]:
            buf, dst = w.into(tuple(part.shape), part.dtype, part.device)
            ops.append(("recv", buf, m))
            bufs.append(dst)
            if sc:
                lbuf, ldst = w.into((1,), torch.float64, part.device)
                ops.append(("recv", lbuf, m))
                lbufs.append(ldst)
        _p2p(ops, meta.group)
        w.finish()
        scales = [log_scale] + ([float(l.item()) for l in lbufs] if sc else [0.0] * len(bufs))
        top = max(scales)
        total = part * _exp_rel(scales[0], top) if scales[0] != top else part
        for b, s in zip(bufs, scales[1:]):
            total = total + (b * _exp_rel(s, top) if s != top else b)
        w2 = _Wire(meta.group)
        payload = w2.out(total.contiguous())
        lt = w2.out(torch.tensor([top], dtype=torch.float64, device=part.device)) if sc else None
        ops = []
        for m in mem[1:]:
            ops.append(("send", payload, m))
            if sc:
                ops.append(("send", lt, m))
        _p2p(ops, meta.group)
        return total, top
    ops = [("send", w.out(part.contiguous()), lead)]
    if sc:
        ops.append(("send", w.out(torch.tensor([log_scale], dtype=torch.float64, device=part.device)), lead))
    _p2p(ops, meta.group)
    w2 = _Wire(meta.group)
    buf, dst = w2.into(tuple(part.shape), part.dtype, part.device)
    rops = [("recv", buf, lead)]
    ldst = None
    if sc:
        lbuf, ldst = w2.into((1,), torch.float64, part.device)
        rops.append(("recv", lbuf, lead))
    _p2p(rops, meta.group)
    w2.finish()
    return dst, (float(ldst.item()) if sc else 0.0)


def _exp_rel(s: float, top: float) -> float:
    return 1.0 if s == top else (math.exp(s - top) if s > -math.inf else 0.0)


class _StageReduce(torch.autograd.Function):
    """The members' K-shard partial sum with its adjoint (AllReduceGrad, allreduce_grad.py:
    13-60): every member's partial gets exp(ls_r - ls_max) x the sum of the members' output
    gradients."""

    @staticmethod
    def forward(ctx, part, meta: _StageMeta, log_scale: float):
        total, top = _reduce(part, meta, log_scale)
        ctx.meta = meta
        ctx.factor = _exp_rel(log_scale, top)
        if total is part:
            total = part.clone()
        top_t = torch.tensor(top, dtype=torch.float64)
        ctx.mark_non_differentiable(top_t)
        return total, top_t

    @staticmethod
    def backward(ctx, g, _g_log):
        meta = ctx.meta
        g = g.contiguous()
        total, _ = _reduce(g, meta, 0.0)
        return total * ctx.factor if ctx.factor != 1.0 else total, None, None
