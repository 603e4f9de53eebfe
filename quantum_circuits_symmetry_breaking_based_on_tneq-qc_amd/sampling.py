"""Many amplitude blocks of one network: several in flight on one GPU, and several per launch.

An amplitude workload that samples more than one block of bitstrings ("shard
bitstrings instead of slices") contracts the same network again and again with other fixed bits:
only the closed qubits' projector operands change (circuits.with_batch), so one compiled plan
serves every block.  The sweeps of one block are latency-bound: a 2^19-element
level is one workgroup lifetime of dependent passes.  `BlockPipeline` fills the GPU two ways:

* **blocks as lanes** (`group`): G blocks contract in ONE lockstep schedule
  (`expression.run_group` -> `tq_plan_execute_group`): every sweep level of the G blocks is one
  kernel launch over G x the ops, so G blocks cost the launches, prologues and pass latencies of
  about one;
* **groups in flight** (`inflight`): consecutive groups run on their own HIP streams, each with
  its own plans (arenas), so one group's GEMM / permute / latency tails overlap another's sweeps.

Block k goes to member k mod G of slot (k div G) mod inflight; a slot's group is launched when
its last member is enqueued (or by `flush()`).  Block b's projector vectors come from a device
table built once (`blocks` given up front); a group launch first copies its members' rows into
the members' projector buffers on the slot's stream (one copy when the rows are consecutive).

Operand contract: the pipeline OWNS its operands and binds every member's plan to them once
(`HipContractExpression.bind`, private plans): the projector buffers are updated IN PLACE between
launches (ordinary stream-ordered copies) and the bound plans read the new values at run time --
no re-validation of the 606 operands per block, and no `.data` rebinding trick.  Outputs are
written on the slot's stream: `wait()` (current stream waits) or `synchronize()` before reading.

The product path is the native plan only (no CPU fallback): the plans raise when the HIP library
is missing.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch

from .circuits import AmplitudeTask, with_batch
from .expression import HipContractExpression, run_group

__all__ = ["BlockPipeline"]


class _Slot:
    __slots__ = ("stream", "pbuf", "bound", "outs", "event", "pending")

    def __init__(self, stream, pbuf, bound, outs):
        self.stream, self.pbuf, self.bound, self.outs = stream, pbuf, bound, outs
        self.event = torch.cuda.Event()
        self.pending: List[int] = []   # table rows of the members enqueued since the last launch


class BlockPipeline:
    """`inflight` slots x `group` members contracting blocks `blocks[k]` (with_batch indices) in
    order; `step()` enqueues the next block and returns its output tensor (written when its
    group is launched and has run: `wait()` / `synchronize()`)."""

    def __init__(self, task: AmplitudeTask, blocks: Sequence[int], inflight: int = 2, group: int = 1,
                 device: Optional[torch.device] = None, dtype: torch.dtype = torch.complex64,
                 min_chunks: Optional[int] = None):
        if inflight < 1 or group < 1:
            raise ValueError("inflight and group must be >= 1")
        if len(blocks) == 0:
            raise ValueError("no blocks")
        self.task = task
        self.blocks = [int(b) for b in blocks]
        self.inflight = int(inflight)
        self.group = int(group)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.dtype = dtype
        self.proj = [i for i, (kind, _) in enumerate(task.kinds) if kind == "proj"]
        # device table: block k's projector vectors (n_proj x 2), built once
        tab = np.zeros((len(self.blocks), len(self.proj), 2), dtype=np.complex128)
        for k, b in enumerate(self.blocks):
            tb = with_batch(task, b)
            for j, i in enumerate(self.proj):
                tab[k, j] = tb.operands[i]
        self.table = torch.from_numpy(tab).to(self.device, dtype)
        # the cores and input vectors are read-only: every member reads the same device copies
        base_ops = [torch.from_numpy(o).to(self.device, dtype) for o in task.operands]
        self.expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
        plan = self.expr.plan(dtype, None, self.device.index)
        if min_chunks is None and self.inflight >= 4:
            # deep pipelines: fewer, wider chunks per sweep op -- the other streams fill the CUs
            # one launch leaves idle (r06, same box: 4 in flight 0.389 -> 0.375 ms per block at
            # 64 instead of 128 chunks; one block at a time it is slower, 0.646 -> 0.714)
            min_chunks = 64
        if min_chunks:
            plan.set("min_chunks", int(min_chunks))
        if self.group > 1:
            # compiled for lockstep groups: wider sweep chunks (G ops share every launch)
            plan.set("group_hint", self.group)
        self.slots: List[_Slot] = []
        for s in range(self.inflight):
            stream = torch.cuda.current_stream(self.device) if s == 0 else torch.cuda.Stream(self.device)
            pbuf = torch.zeros((self.group, len(self.proj), 2), dtype=dtype, device=self.device)
            bound, outs = [], []
            for m in range(self.group):
                ops = list(base_ops)
                for j, i in enumerate(self.proj):
                    ops[i] = pbuf[m, j]
                bound.append(self.expr.bind(*ops, private_plan=True))
                outs.append(torch.empty(self.expr.out_shape, dtype=dtype, device=self.device))
            self.slots.append(_Slot(stream, pbuf, bound, outs))
        self.k = 0
        torch.cuda.synchronize(self.device)   # the table and operands exist before any slot stream reads them

    def plan(self, slot: int = 0, member: int = 0):
        """The native plan of one member (queries / profiling)."""
        return self.slots[slot].bound[member].plan

    def _launch(self, slot: _Slot) -> None:
        rows = slot.pending
        n = len(rows)
        if n == 0:
            return
        with torch.cuda.stream(slot.stream):
            r0 = rows[0]
            if rows == list(range(r0, r0 + n)):
                slot.pbuf[:n].copy_(self.table[r0:r0 + n])
            else:
                for m, r in enumerate(rows):
                    slot.pbuf[m].copy_(self.table[r])
            if n == 1:
                slot.bound[0].run(slot.outs[0], slot.stream)
            else:
                run_group(slot.bound[:n], slot.outs[:n], slot.stream)
            slot.event.record(slot.stream)
        slot.pending = []

    def step(self) -> torch.Tensor:
        """Enqueue block blocks[k mod len(blocks)] as member k mod group of slot
        (k div group) mod inflight; launches the slot's group once it is full.  Returns that
        member's output tensor (overwritten when the slot runs again)."""
        k = self.k
        slot = self.slots[(k // self.group) % self.inflight]
        m = k % self.group
        if m == 0 and slot.pending:   # (after a reset: a partial group left behind)
            self._launch(slot)
        slot.pending.append(k % len(self.blocks))
        self.k += 1
        if m == self.group - 1:
            self._launch(slot)
        return slot.outs[m]

    def flush(self) -> None:
        """Launch every partially filled group."""
        for slot in self.slots:
            self._launch(slot)

    def wait(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Flush, then make `stream` (default: the current one) wait for every launched group:
        the outputs may then be read on it."""
        self.flush()
        st = stream or torch.cuda.current_stream(self.device)
        for slot in self.slots:
            if slot.stream is not st:
                st.wait_event(slot.event)

    def reset(self) -> None:
        """Flush and start again at block 0 (slot 0, member 0)."""
        self.flush()
        self.k = 0

    def run(self, n: Optional[int] = None) -> List[torch.Tensor]:
        """Contract the next `n` blocks (default: every block once); returns host copies of their
        amplitudes in order (a checking helper: `step()` is the pipelined form)."""
        n = len(self.blocks) if n is None else n
        res = []
        pend = []
        for _ in range(n):
            pend.append(self.step())
            if self.k % self.group == 0:
                self.synchronize()
                res.extend(o.cpu() for o in pend)
                pend = []
        if pend:
            self.synchronize()
            res.extend(o.cpu() for o in pend)
        return res

    def synchronize(self) -> None:
        self.flush()
        torch.cuda.synchronize(self.device)
