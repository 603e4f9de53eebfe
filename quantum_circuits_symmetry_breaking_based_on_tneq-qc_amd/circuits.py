"""Random brick-wall circuits and the amplitude workloads of the configs (BASELINE.json).

Graph generation follows the reference workload: build_brick_wall_IM + incidence_to_graph
(symmetry_breaking_quantum.py:15-125; cores named get_symbol(column), column = time order:
per cell the even bonds (0,1),(2,3).. then the odd bonds (1,2),(3,4)..).  Depth d = 2 * cells.

An *amplitude task* is the vector-inputs network of the reference
(EinsumStrategy.build_with_vector_inputs_expression, einsum_strategy.py:258-318) with |0> inputs,
plus projectors <x_q| on the fixed output qubits; the remaining (open) outputs form a correlated
batch of 2^open amplitudes, axes in the reference's core order.  For the multi-GPU configs the
network is cut between two qubit lines: each half is swept line by line (every step absorbs one
gate or vector: the APPLY lowering), the halves meet in one boundary GEMM over the cut legs, and
`n_slice` of the cut legs are sliced.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from .contractor.einsum_strategy import EinsumStrategy
from .core.qctn import QCTN
from .einsum import (Network, choose_slices, deferred_search, get_symbol, linear_path, parse_equation, partition_path,
                     vector_absorptions)


def build_brick_wall_IM(n_qubits: int, n_cells: int, rank: int = 2) -> np.ndarray:
    """Incidence matrix qubits x cores of a 1-D brick wall (symmetry_breaking_quantum.py:107-125)."""
    n_cores = (n_qubits - 1) * n_cells
    IM = np.zeros((n_qubits, n_cores), dtype=int)
    for cell in range(n_cells):
        col = cell * (n_qubits - 1)
        for start in (0, 1):
            for q in range(start, n_qubits - 1, 2):
                IM[q, col] = rank
                IM[q + 1, col] = rank
                col += 1
    return IM


def incidence_to_graph(incidence: np.ndarray, core_symbols=None, mask_list=None, *,
                       for_display: bool = False, keep_zeros: bool = False, mask_char: str = "█",
                       pad_dim=None) -> str:
    """Incidence matrix -> QCTN graph string (symmetry_breaking_quantum.py:15-102)."""
    if incidence.ndim != 2:
        raise ValueError("incidence must be 2D (n_qubits x n_cores)")
    if (incidence < 0).any():
        raise ValueError("incidence entries must be >= 0")
    nq, nc = incidence.shape
    if core_symbols is None:
        core_symbols = [get_symbol(i) for i in range(nc)]
    if len(core_symbols) != nc:
        raise ValueError("core_symbols length must match n_cores")
    masks = set(mask_list or [])
    for m in masks:
        if m < 0 or m >= nc:
            raise IndexError(f"mask_index={m} out of range: 0 ~ {nc - 1}")
    sym = lambda c: mask_char if (for_display and c in masks) else core_symbols[c]
    if for_display and keep_zeros:
        widths = []
        for c in range(nc):
            v = incidence[:, c][incidence[:, c] > 0]
            dim = int(v.max()) if len(v) else (int(pad_dim) if pad_dim is not None else 1)
            widths.append(len(f"-{dim}-{sym(c)}"))
        rows = []
        for q in range(nq):
            row = ""
            for c in range(nc):
                d = int(incidence[q, c])
                if d > 0:
                    slot = f"-{d}-{sym(c)}"
                    row += slot + "-" * (widths[c] - len(slot))
                else:
                    row += "-" * widths[c]
            rows.append(row + "-")
        return "\n".join(rows)
    rows = []
    for q in range(nq):
        ent = [(core_symbols[c], int(incidence[q, c])) for c in range(nc) if incidence[q, c] > 0]
        if not ent:
            raise ValueError(f"Row {q} has no cores; graph line would be invalid.")
        row = f"-{ent[0][1]}-{ent[0][0]}"
        for core, dim in ent[1:]:
            row += f"-{dim}-" + core
        rows.append(row + f"-{ent[-1][1]}-")
    return "\n".join(rows)


def haar_unitary(rng: np.random.Generator, n: int) -> np.ndarray:
    """Haar-random unitary: complex Gaussian QR with the phase of diag(R) removed
    (the construction of backend_pytorch.py:470-495, seeded numpy RNG)."""
    z = (rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))) / np.sqrt(2.0)
    q, r = np.linalg.qr(z)
    ph = np.diag(r) / np.abs(np.diag(r))
    return q * ph.conj()[None, :]


def random_unitary_cores(qctn: QCTN, seed: int) -> Dict[str, np.ndarray]:
    """complex128 cores of shape input_shape + output_shape, unitary as [in_dim, out_dim] matrices."""
    rng = np.random.default_rng(seed)
    cores = {}
    for info in qctn.adjacency_table:
        din, dout = info["input_dim"], info["output_dim"]
        if din != dout:
            raise ValueError("unitary cores need input_dim == output_dim")
        u = haar_unitary(rng, din)
        cores[info["core_name"]] = np.ascontiguousarray(u.reshape(info["input_shape"] + info["output_shape"]))
    return cores


@dataclass
class BrickWall:
    n_qubits: int
    depth: int
    seed: int = 0
    mask: Sequence[int] = ()

    def __post_init__(self):
        if self.depth % 2:
            raise ValueError("depth must be even (2 layers per brick-wall cell)")
        IM = build_brick_wall_IM(self.n_qubits, self.depth // 2, 2)
        if len(self.mask):
            IM[:, list(self.mask)] = 0
        self.IM = IM
        self.graph = incidence_to_graph(IM)
        self.qctn = QCTN(self.graph)
        # time of each core = column's layer (2*cell + parity of its bond)
        nb = self.n_qubits - 1
        self.core_time: Dict[str, int] = {}
        self.core_qubits: Dict[str, Tuple[int, int]] = {}
        for c in range(IM.shape[1]):
            rows = np.nonzero(IM[:, c])[0]
            if len(rows) == 0:
                continue
            name = get_symbol(c)
            cell, k = divmod(c, nb)
            even = (self.n_qubits) // 2
            self.core_time[name] = 2 * cell + (0 if k < even else 1)
            self.core_qubits[name] = (int(rows.min()), int(rows.max()))
        self.cores = random_unitary_cores(self.qctn, 1000 + self.seed)


@dataclass
class AmplitudeTask:
    circuit: BrickWall
    eq: str
    shapes: List[Tuple[int, ...]]
    operands: List[np.ndarray]
    kinds: List[Tuple[str, object]]          # ('in', q) | ('core', name) | ('proj', q)
    open_qubits: List[int]                   # output axes (core order of the reference)
    fixed_bits: Dict[int, int]
    path: List[Tuple[int, int]]
    sliced: List[str] = field(default_factory=list)
    cut: Optional[int] = None

    @property
    def n_amplitudes(self) -> int:
        return 2 ** len(self.open_qubits)

    def network(self) -> Network:
        return parse_equation(self.eq, self.shapes)


def amplitude_task(circ: BrickWall, open_qubits: Sequence[int], fixed_bits: Optional[Dict[int, int]] = None,
                   cut: Optional[int] = None, n_slice: int = 0, bit_seed: int = 7,
                   absorb_vectors: bool = True, tile: int = 4,
                   defer: Union[None, str, Tuple[int, int]] = None) -> AmplitudeTask:
    """Build the amplitude network; fixed bits default to a seeded uniform bitstring.
    With a cut, each half is swept in diamond tiles of `tile` x `tile` gates (diamond_order;
    0 = line by line); `defer` = (left, right) tensors at the end of each half's sweep absorbed
    after the boundary contraction (einsum.partition_path), "auto" = einsum.deferred_search."""
    n = circ.n_qubits
    open_set = set(int(q) for q in open_qubits)
    if fixed_bits is None:
        rng = np.random.default_rng(bit_seed)
        fixed_bits = {q: int(rng.integers(0, 2)) for q in range(n) if q not in open_set}
    if set(fixed_bits) | open_set != set(range(n)) or set(fixed_bits) & open_set:
        raise ValueError("fixed_bits and open_qubits must partition the qubits")
    eq, shapes, in_q, proj_q, open_q = EinsumStrategy.build_amplitude_expression(circ.qctn, fixed_bits)
    zero = np.array([1.0, 0.0], dtype=np.complex128)
    operands: List[np.ndarray] = []
    kinds: List[Tuple[str, object]] = []
    for q in in_q:
        operands.append(zero.copy())
        kinds.append(("in", q))
    for name in circ.qctn.cores:
        operands.append(circ.cores[name])
        kinds.append(("core", name))
    for q in proj_q:
        e = np.zeros(2, dtype=np.complex128)
        e[fixed_bits[q]] = 1.0
        operands.append(e)
        kinds.append(("proj", q))
    net = parse_equation(eq, shapes)

    def sweep_key(k, upward=True):
        kind, v = k
        if kind == "core":
            lo, hi = circ.core_qubits[v]
            line = lo if upward else hi
            t = circ.core_time[v]
        else:
            line, t = v, (-1 if kind == "in" else 10 ** 6)
        return (line if upward else -line, t)

    # inputs |0> and output projectors are folded into their gates first (no sweep step then
    # grows the running tensor by a leg that a vector removes right after)
    pre = vector_absorptions(net) if absorb_vectors else []
    if cut is None:
        order = sorted(range(len(kinds)), key=lambda i: sweep_key(kinds[i]))
        path = linear_path(net, order, pre=pre)[0]
        sliced_ids: List[int] = []
    else:
        # cores go left when their lower qubit is < cut (the gates straddling the cut are
        # left); every boundary vector follows the core it is attached to
        side = {}
        owner = {}
        for i, k in enumerate(kinds):
            if k[0] == "core":
                side[i] = circ.core_qubits[k[1]][0] < cut
                for m in net.terms[i]:
                    owner[m] = i
        for i, k in enumerate(kinds):
            if k[0] != "core":
                side[i] = side[owner[net.terms[i][0]]]
        left = [i for i in range(len(kinds)) if side[i]]
        right = [i for i in range(len(kinds)) if not side[i]]
        if tile:
            lord = diamond_order(circ, kinds, net, left, True, cut - 1, tile)
            rord = diamond_order(circ, kinds, net, right, False, cut, tile)
        else:
            lord = sorted(left, key=lambda i: sweep_key(kinds[i], True))
            rord = sorted(right, key=lambda i: sweep_key(kinds[i], False))
        path = partition_path(net, [left, right], [lord, rord], pre=pre)
        lm = set(m for i in left for m in net.terms[i])
        rm = set(m for i in right for m in net.terms[i])
        cut_modes = sorted((lm & rm) - set(net.out))
        sliced_ids = choose_slices(net, path, n_slice, cut_modes) if n_slice else []
        if defer == "auto":
            defer = deferred_search(net, [left, right], [lord, rord], pre, sliced_ids)
        if defer and any(defer):
            path = partition_path(net, [left, right], [lord, rord], pre=pre, defer=defer)
            sliced_ids = choose_slices(net, path, n_slice, cut_modes) if n_slice else []
    return AmplitudeTask(circ, eq, shapes, operands, kinds, list(open_q), dict(fixed_bits), path,
                         [net.symbols[m] for m in sliced_ids], cut)


def diamond_order(circ: BrickWall, kinds, net: Network, ids: Sequence[int], upward: bool,
                  boundary_pair: int, tile: int) -> List[int]:
    """Sweep order of one half of a cut brick wall in diamond tiles.

    Gate (pair r, time t) takes its two line-r legs from gates (r-1, t-1) and (r-1, t+1)
    (r counted away from the half's far edge).  In the rotated coordinates a = (t+r-p)/2,
    d = (r-t-p)/2 those are (a-1, d) and (a, d-1), so tiles of tile x tile gates taken in order
    of (A+D, A) and row-major inside are a valid sweep, and a tile only ever holds 2*tile live
    legs of the running tensor: one butterfly-sweep op (tq_sweep2) absorbs tile^2 gates where
    the line-by-line order fits tile.  The gates on the cut's pair (whose legs the slicing
    fixes) come last, in time order, so everything before them is slice-invariant."""
    n = circ.n_qubits
    owner = {}
    for i in ids:
        if kinds[i][0] == "core":
            for m in net.terms[i]:
                owner[m] = i
    par = {(circ.core_time[kinds[i][1]] + circ.core_qubits[kinds[i][1]][0]) % 2
           for i in ids if kinds[i][0] == "core"}
    p = par.pop() if len(par) == 1 else 0

    def core_key(i):
        lo = circ.core_qubits[kinds[i][1]][0]
        t = circ.core_time[kinds[i][1]]
        if lo == boundary_pair:
            return (1, t, 0, 0, 0)
        r = lo if upward else (n - 2) - lo
        a, d = (t + r - p) // 2, (r - t - p) // 2
        A, D = a // tile, d // tile
        return (0, A + D, A, a, d)

    def key(i):
        if kinds[i][0] == "core":
            return core_key(i) + (0,)
        return core_key(owner[net.terms[i][0]]) + (-1 if kinds[i][0] == "in" else 1,)

    return sorted(ids, key=key)


# ---- the BASELINE.json configurations ------------------------------------------------------

def config_task(name: str, seed: int = 0, batch: int = 0) -> AmplitudeTask:
    """C1..C4 amplitude workloads; C5 is the symmetry-breaking ansatz
    (see ansatz_qctn).  `batch` selects another block of amplitudes of the same network
    (amplitude_task: other fixed bits, same plan) -- bench.py's bitstring sharding."""
    if batch:
        return with_batch(config_task(name, seed), batch)
    if name == "C1":   # 10q d8, one amplitude (CPU plumbing config)
        return amplitude_task(BrickWall(10, 8, seed), [])
    if name == "C2":   # 30q d14, one amplitude, no slicing
        return amplitude_task(BrickWall(30, 14, seed), [])
    if name == "C3":   # 40q d16, cut 20|20, 8+8 open, 6 sliced cut legs -> 64 slices
        return amplitude_task(BrickWall(40, 16, seed), list(range(12, 28)), cut=20, n_slice=6)
    if name == "C3d":  # C3 with deferred tails (10 / 8): 3.2e9 -> 5.3e8 complex MACs, but measured
        # slower (1.74 vs 0.68 ms per execute, profiles/defer_sweep_r05.txt): the per-slice tails run
        # as per-lane launches, where C3's per-slice boundary GEMMs run lane-batched
        return amplitude_task(BrickWall(40, 16, seed), list(range(12, 28)), cut=20, n_slice=6, defer=(10, 8))
    if name == "C4":   # 53q d20, cut 27|26, 10+10 open, 3 sliced cut legs -> 8 slices
        # the last 20 / 16 tensors of the two sweeps absorbed after the boundary contraction
        # (einsum.deferred_search on this network: 5.6e11 -> 3.5e9 complex MACs per execute)
        return amplitude_task(BrickWall(53, 20, seed), list(range(17, 37)), cut=27, n_slice=3, defer=(20, 16))
    if name == "C4x4":  # C4's network with qubits 16 and 37 open too: 4 blocks of C4 in one contraction
        # (2^22 amplitudes; C4's fixed bits elsewhere, so the (q16, q37) = C4's-bits sub-block IS C4's
        # block).  Larger correlated batches amortise the hoisted sweeps: 0.32 ms per 2^20 amplitudes
        # on one stream against C4's 0.74 (profiles/open_batch_r05.txt)
        rng = np.random.default_rng(7)
        bits = {q: int(rng.integers(0, 2)) for q in range(53) if not 17 <= q < 37}
        bits.pop(16)
        bits.pop(37)
        return amplitude_task(BrickWall(53, 20, seed), list(range(16, 38)), fixed_bits=bits, cut=27, n_slice=3,
                              defer=(20, 16))
    if name == "C4g":  # C4 on the r02-r05 path: each half swept whole, then ONE boundary contraction
        # (per slice a 1024 x 1024 x 65536 complex GEMM fed by the dense sweeps: the big-GEMM path)
        return amplitude_task(BrickWall(53, 20, seed), list(range(17, 37)), cut=27, n_slice=3)
    raise ValueError(f"unknown config {name!r}")


def with_batch(task: AmplitudeTask, batch: int) -> AmplitudeTask:
    """Amplitude block `batch` of the same network: the closed qubits' fixed bits with the lowest
    ones flipped by the binary digits of `batch` (blocks b != b' hold disjoint bitstrings), i.e.
    only the output projector operands change -- equation, shapes, path and slicing are the
    task's own, so one compiled plan serves every block (bench.py's bitstring sharding)."""
    import dataclasses
    closed = sorted(task.fixed_bits)
    if not 0 <= batch < 2 ** len(closed):
        raise ValueError(f"batch {batch} out of range for {len(closed)} closed qubits")
    bits = dict(task.fixed_bits)
    for i, q in enumerate(closed):
        if (batch >> i) & 1:
            bits[q] ^= 1
    ops = list(task.operands)
    for i, (kind, q) in enumerate(task.kinds):
        if kind == "proj":
            e = np.zeros(2, dtype=np.complex128)
            e[bits[q]] = 1.0
            ops[i] = e
    return dataclasses.replace(task, operands=ops, fixed_bits=bits)


TRAIN_MASK = [2, 3, 5, 8, 9, 12, 13, 14, 15, 17, 18, 20, 21, 23, 25, 26, 29, 31, 32, 33]  # train.py:30


def ansatz_qctn(n_qubits: int = 8, n_cells: int = 5, mask: Sequence[int] = TRAIN_MASK) -> BrickWall:
    """C5: the symmetry-breaking brick-wall ansatz of train.py:16-30 (8 qubits, 5 cells, target mask)."""
    return BrickWall(n_qubits, 2 * n_cells, seed=5, mask=mask)
