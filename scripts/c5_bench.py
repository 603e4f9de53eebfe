#!/usr/bin/env python3
"""C5 bench: the symmetry-breaking training step (symmetry_breaking_quantum.py:184-230) on the
HIP engine, complex128 (BASELINE.json configs[4]: "ansatz, fp64").

Workload: the 8-qubit 5-cell brick wall (35 cores); target = the core-only contraction of the
train.py:30-masked ansatz (15 cores); 8 pruning candidates = the full ansatz minus one core each
(the first round of symmetry_breaking(): candidate = [idx], 34 cores), each fitted with
SGDG(lr=1e-2, stiefel=True, momentum=0.9).  A step = for every candidate: core-only forward
(2^16 amplitudes), fidelity loss, backward (reverse mode through the pairwise path), one SGDG
step.  Metric: candidate training steps/s (8 per step).

Forward = the split/merge contractor path (BASELINE.json configs[4]; examples/
example_qctn_merge_split.py:59-66): every candidate's QCTN is split by QCTN.split (qctn.py:
1296-1401, cores[:n//2] | cores[n//2:]), each half is swept on its own and the halves are joined
by the boundary contraction (einsum.partition_path), all in one native plan per candidate.

Ranks: under a launcher (RANK / WORLD_SIZE / LOCAL_RANK set, as bench.py's ranks pass on) the 8
candidates are dealt round-robin over the ranks (candidate k on rank k mod N: independent fits,
no collective on the data path, the reference's loop symmetry_breaking_quantum.py:196-238 run
concurrently); a gloo group on --port only times the step (barrier + max over ranks).  The line
splits the step time into host issue time (the Python / launch work until the last candidate's
launches are queued) and the wall time (until the GPU is done).

CPU baseline ("port"): the same step with torch on the host — pairwise torch.tensordot along the
same path (what opt_einsum's ContractExpression executes), torch autograd, and the reference's
SGDG math (oracle/optim_ref.py) — timed on a bounded sample.
    python scripts/c5_bench.py [--steps 20] [--warmup 3] [--cpu-steps 3]
"""
import argparse
import datetime
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tneq_qc_amd.circuits import BrickWall, TRAIN_MASK  # noqa: E402
from tneq_qc_amd.contractor import EinsumStrategy  # noqa: E402
from tneq_qc_amd.einsum import parse_equation, partition_path  # noqa: E402
from tneq_qc_amd.expression import HipContractExpression  # noqa: E402
from tneq_qc_amd.graphs import capture_step, gc_paused  # noqa: E402
from tneq_qc_amd.optim import SGDG  # noqa: E402

N_Q, DEPTH = 8, 10
CANDIDATES = [0, 1, 4, 6, 7, 10, 11, 16]   # cores outside the target mask


def split_merge_expression(qctn):
    """The core-only expression (einsum_strategy.py:136-194) contracted along QCTN.split's two
    halves: each half swept, then the boundary contraction (the merge)."""
    eq, sh = EinsumStrategy.build_core_only_expression(qctn)
    left, right = qctn.split()
    idx = {c: i for i, c in enumerate(qctn.cores)}
    groups = [[idx[c] for c in left.cores], [idx[c] for c in right.cores]]
    return HipContractExpression(eq, *sh, optimize=partition_path(parse_equation(eq, sh), groups)), eq


def setup(dev, ks=None):
    tgt_bw = BrickWall(N_Q, DEPTH, seed=5, mask=TRAIN_MASK)
    eq_t, sh_t = EinsumStrategy.build_core_only_expression(tgt_bw.qctn)
    ex_t = EinsumStrategy.create_contract_expression(eq_t, sh_t)
    target = ex_t(*[torch.from_numpy(tgt_bw.cores[c]).to(dev) for c in tgt_bw.qctn.cores]).reshape(-1)
    cands = []
    for k, idx in enumerate(CANDIDATES):
        if ks is not None and k not in ks:
            continue
        bw = BrickWall(N_Q, DEPTH, seed=100 + k, mask=[idx])
        expr, eq = split_merge_expression(bw.qctn)
        params = [torch.nn.Parameter(torch.from_numpy(bw.cores[c].copy()).to(dev)) for c in bw.qctn.cores]
        # the candidate's own stream of the SGDG retraction draws (the reference draws from the
        # global `random`; SGDG's rng= gives each concurrently trained candidate its own):
        # results independent of the rank layout
        rng = random.Random(1000 + k)
        opt = SGDG(params, lr=1e-2, stiefel=True, momentum=0.9, rng=rng)
        cands.append((expr, params, opt, bw, eq, rng))
    return target, cands


# the GPU step's loss: the fused kernels (tneq_qc_amd.ops.fidelity_loss, one launch each way)
# unless C5_TORCH_LOSS=1 (the reference's torch expression, ~25 launches)
USE_FUSED_LOSS = os.environ.get("C5_TORCH_LOSS", "0") != "1"


def fidelity_loss(out, tgt):
    """symmetry_breaking_quantum.py:224-228; on the HIP device the fused op, on the host (the CPU
    baseline and the parity checker) the reference's torch expression."""
    if out.is_cuda and USE_FUSED_LOSS:
        from tneq_qc_amd.ops import fidelity_loss as fused
        return fused(out, tgt)
    out_f = out.reshape(-1)
    num = torch.vdot(tgt, out_f).abs() ** 2
    den = (torch.vdot(tgt, tgt).real * torch.vdot(out_f, out_f).real).clamp_min(1e-12)
    return 1.0 - num / den


def capture(target, cands, dev):
    """Each candidate's forward + fidelity loss + backward as one hipGraph (graphs.capture_step):
    a step then replays it and runs SGDG eagerly (the host-side retraction draw stays per step)."""
    graphs = []
    for (expr, params, _, _, _, _) in cands:
        def fb(expr=expr, params=params):
            loss = fidelity_loss(expr(*params), target)
            loss.backward()
            return loss
        graphs.append(capture_step(fb, params, dev))
    return graphs


def capture_all(target, cands, dev, warmup=2):
    """Every candidate's forward + loss + backward in ONE hipGraph: candidate k on a stream of
    its own inside the capture (fork / join), so the graph holds 8 independent branches."""
    cap = torch.cuda.Stream(dev)
    sts = [torch.cuda.Stream(dev) for _ in cands]

    def run_all():
        losses = []
        cur = torch.cuda.current_stream(dev)
        for (expr, params, _, _, _, _), st in zip(cands, sts):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                loss = fidelity_loss(expr(*params), target)
                loss.backward()
            losses.append(loss)
        for st in sts:
            cur.wait_stream(st)
        return losses

    allp = [p for c in cands for p in c[1]]
    cap.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cap):
        for _ in range(warmup):
            for p in allp:
                p.grad = None
            run_all()
    torch.cuda.current_stream(dev).wait_stream(cap)
    torch.cuda.synchronize(dev)
    for p in allp:
        p.grad = None
    g = torch.cuda.CUDAGraph()
    with gc_paused(), torch.cuda.graph(g, stream=cap):
        losses = run_all()
    torch.cuda.synchronize(dev)
    return g, losses


def gpu_step_one_graph(target, cands, graph_all):
    """capture_all's graph replayed once, then every candidate's SGDG step."""
    g, losses = graph_all
    g.replay()
    for (_, _, opt, _, _, _) in cands:
        opt.step()
    return losses


def gpu_step(target, cands, streams=None, graphs=None):
    """One training step of every candidate.  With `streams`, candidate k runs on streams[k]: the
    candidates are independent fits, so their latency-bound launch chains (each plan replays its
    own hipGraphs) overlap on the GPU instead of queueing behind each other.  With `graphs`
    (capture()), forward + loss + backward of candidate k is one graph replay."""
    losses = []
    cur = torch.cuda.current_stream()
    for k, (expr, params, opt, _, _, _) in enumerate(cands):
        st = streams[k] if streams else cur
        if streams:
            st.wait_stream(cur)
        with torch.cuda.stream(st):
            if graphs is not None:
                g, loss = graphs[k]
                g.replay()
            else:
                opt.zero_grad()
                loss = fidelity_loss(expr(*params), target)
                loss.backward()
            opt.step()
        losses.append(loss)
    if streams:
        for st in streams:
            cur.wait_stream(st)
    return losses


def launch_stats(cands, dtype=torch.complex128):
    """Per candidate-step: kernel launches and algorithmic HBM bytes of the native plans the
    graphed step replays (the reverse tree's forward step plans, every gradient step plan, one
    SGDG launch), from the plans' own counters (tq_plan_query n_launch_* / bytes_moved).  The
    fidelity loss's few torch kernels are not counted."""
    launches, nbytes, n_plans = [], [], []
    for expr, params, _, _, _, _ in cands:
        rev = expr.reverse_tree(dtype)
        L, B, n = 1, 0, 0                       # + the SGDG launch
        for (i, j, k, fwd, bwd) in rev.steps:
            plans = [fwd.plan(dtype)] + [g.plan(dtype) for (_, _, g, _) in bwd]
            for pl in plans:
                L += pl.query("n_launch_once") + pl.query("n_launch_slice")
                B += pl.query("bytes_moved")
                n += 1
        launches.append(L)
        nbytes.append(B)
        n_plans.append(n)
    return {"launches_per_candidate_step": sum(launches) / len(launches),
            "algorithmic_bytes_per_candidate_step": sum(nbytes) / len(nbytes),
            "plans_per_candidate": sum(n_plans) / len(n_plans)}


def _log(msg):
    print(f"[c5_bench] {msg}", file=sys.stderr, flush=True)


def cpu_forward(expr, ts):
    """The forward as opt_einsum's ContractExpression executes it, on torch-CPU: pairwise
    torch.tensordot along the expression's own path (the contraction ORDER is the only thing
    taken from the HIP expression), single-side sums, then the permute into the step's result
    order.  Differentiable by torch autograd."""
    from tneq_qc_amd.einsum import _State
    st = _State(expr.net)
    vals = dict(enumerate(ts))
    modes = {i: tuple(t) for i, t in enumerate(expr.net.terms)}
    for s, (i, j) in enumerate(expr.path):
        res = st.result(i, j)
        k = st.contract(i, j)
        mi, mj = modes[i], modes[j]
        ci = [q for q, m in enumerate(mi) if m in mj]
        cj = [mj.index(mi[q]) for q in ci]
        out = torch.tensordot(vals[i], vals[j], dims=(ci, cj))
        om = [m for m in mi if m not in mj] + [m for m in mj if m not in mi]
        final = tuple(expr.net.out) if s == len(expr.path) - 1 else res
        keep = [m for m in om if m in final]
        if len(keep) != len(om):   # single-side sums
            out = out.sum(dim=[q for q, m in enumerate(om) if m not in final])
        out = out.permute([keep.index(m) for m in final])
        vals[k], modes[k] = out, final
    return vals[max(vals)]


def cpu_train_step(expr, ps, state, tgt, rng=random):
    """One candidate-step on the host: cpu_forward + fidelity loss + torch autograd + the
    reference SGDG math (oracle/optim_ref.py, the retraction draw from `rng`).  `ps` (numpy
    arrays) are updated in place; returns (loss, gradients)."""
    from oracle.optim_ref import sgdg_step
    ts = [torch.tensor(p, requires_grad=True) for p in ps]
    loss = fidelity_loss(cpu_forward(expr, ts), tgt)
    grads = [g.numpy().copy() for g in torch.autograd.grad(loss, ts)]
    sgdg_step(ps, [g.copy() for g in grads], state, lr=1e-2, momentum=0.9, stiefel=True, rng=rng)
    return float(loss.detach()), grads


def cpu_step_sample(target_np, cands, steps, budget_s=10.0):
    """torch-CPU pairwise tensordot along the same path + autograd + the reference SGDG math:
    up to `steps` steps of every candidate, stopping once `budget_s` seconds of work are done
    (at least one candidate-step)."""
    tgt = torch.from_numpy(target_np)
    items = []
    for expr, params, _, bw, _, _ in cands:
        items.append((expr, [p.detach().cpu().numpy().copy() for p in params], {}))
    t0 = time.perf_counter()
    n = 0
    for _ in range(steps):
        for expr, ps, state in items:
            if n and time.perf_counter() - t0 > budget_s:
                return (time.perf_counter() - t0), n
            cpu_train_step(expr, ps, state, tgt)
            n += 1
    return (time.perf_counter() - t0), n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--one-stream", action="store_true", help="candidates one after another on one stream")
    ap.add_argument("--streams", type=int, default=0,
                    help="candidate k on stream k mod N (0: one stream per candidate)")
    ap.add_argument("--eager", action="store_true",
                    help="forward / loss / backward issued eagerly every step (default: one hipGraph per candidate)")
    ap.add_argument("--port", type=int, default=0, help="gloo timing group port (multi-rank)")
    ap.add_argument("--one-graph", action="store_true",
                    help="every candidate's forward + loss + backward in ONE hipGraph (branches on forked streams)")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", init_method=f"tcp://{os.environ.get('MASTER_ADDR', '127.0.0.1')}:{a.port}",
                                rank=rank, world_size=world, timeout=datetime.timedelta(seconds=240))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    random.seed(rank)
    mine = list(range(rank, len(CANDIDATES), world))
    _log(f"rank {rank}: setting up {len(mine)} candidates")
    target, cands = setup(dev, set(mine))
    if a.one_stream:
        streams = None
    else:
        pool = [torch.cuda.Stream(dev) for _ in range(a.streams if a.streams > 0 else len(cands))]
        streams = [pool[k % len(pool)] for k in range(len(cands))]
    graph_all = capture_all(target, cands, dev) if a.one_graph else None
    graphs = None if (a.eager or a.one_graph) else capture(target, cands, dev)
    step = (lambda: gpu_step_one_graph(target, cands, graph_all)) if graph_all else \
        (lambda: gpu_step(target, cands, streams, graphs))
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    _log(f"rank {rank}: warmup done; timing {a.steps} steps")
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        losses = step()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt_local = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    times = torch.tensor([dt, dt_local, t_issue], dtype=torch.float64)
    my_losses = {int(k): float(l.detach()) for k, l in zip(mine, losses)}
    if world > 1:
        allt = [torch.zeros_like(times) for _ in range(world)]
        dist.all_gather(allt, times)
        dt = max(float(t[0]) for t in allt)
        parts = [None] * world
        dist.all_gather_object(parts, my_losses)
        for d in parts:
            my_losses.update(d)
    else:
        allt = [times]
    dt /= a.steps
    res = {"metric": "candidate training steps/s (forward + backward + SGDG), C5 ansatz",
           "value": len(CANDIDATES) / dt, "unit": "candidate-steps/s", "ms_per_step": dt * 1e3,
           "n_gpus": world, "candidates": len(CANDIDATES),
           "candidates_per_rank": [len(range(r, len(CANDIDATES), world)) for r in range(world)],
           "cores_per_candidate": len(cands[0][1]), "dtype": "c128",
           "streams": len({id(x) for x in streams}) if streams else 1,
           "step_graphs": "one graph, a branch per candidate" if graph_all else graphs is not None,
           "forward": "QCTN.split halves swept + boundary contraction (split/merge path), one native plan",
           "amplitudes_per_forward": int(np.prod(cands[0][0].out_shape)),
           "host_issue_ms_per_step": [float(t[2]) / a.steps * 1e3 for t in allt],
           "wall_ms_per_step_per_rank": [float(t[1]) / a.steps * 1e3 for t in allt],
           "loss_after": [my_losses[k] for k in sorted(my_losses)]}
    try:
        res.update(launch_stats(cands))
    except Exception as e:  # the stats must never hide the timing
        res["launch_stats_error"] = repr(e)
    if world > 1:
        dist.destroy_process_group()
    if rank != 0:
        return
    if a.cpu_steps > 0 and world == 1:
        # every host core and 16 (the box's CPU share per GPU): the faster counts
        host = os.cpu_count() or 1
        runs = []
        for th in sorted({host, min(16, host)}, reverse=True):
            torch.set_num_threads(th)
            _log(f"cpu baseline at {th} threads")
            secs, n = cpu_step_sample(target.cpu().numpy(), cands, a.cpu_steps)
            runs.append({"value": n / secs, "cores": torch.get_num_threads(), "sample": f"{n} candidate-steps"})
        best = max(runs, key=lambda r: r["value"])
        res["cpu_baseline"] = {"value": best["value"], "unit": "candidate-steps/s", "cores": best["cores"],
                               "host_cpus": host, "by_threads": runs,
                               "kind": "port", "sample": f"{best['sample']} (torch CPU pairwise tensordot "
                               "along the same path + autograd + oracle SGDG), complex128, at every host "
                               "core and at 16 threads; value = the faster"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
