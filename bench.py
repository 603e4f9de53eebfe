#!/usr/bin/env python3
"""bench.py — amplitudes/sec of sliced random-circuit amplitude batches on MI355X.

Workload (BASELINE.json metric "amplitudes/sec + achieved MFMA TFLOP/s, 53q depth-20 RQC"):
config C4 of SURVEY.md §8(d): a 53-qubit depth-20 brick-wall random circuit (520 Haar-random
2-qubit cores, the reference's build_brick_wall_IM + incidence_to_graph family), |0> inputs,
33 output bits fixed, 20 open (2^20 correlated bitstrings), cut between qubits 26|27, 3 cut legs
sliced -> 8 slices.  One "step" = all 2^20 amplitudes: every rank contracts slices
rank, rank+N, ... (left/right line sweeps + boundary MFMA GEMM, slice-invariant work hoisted)
into a partial-amplitude buffer, then one RCCL all-reduce (SUM) over xGMI.  Total work is fixed
as N grows ("scaling": "strong").  Inputs (cores, vectors) are resident in HBM before timing.

Prints ONE JSON line on rank 0 with `roofline` (dominant kernel = the boundary GEMM, timed with
HIP events on its stream inside the timed region) and, at N=1, `cpu_baseline` (the oracle's
numpy pairwise executor on a bounded sample of the same network).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, f32-in MFMA
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
N_OPEN_CPU = 20                 # open outputs in the CPU-baseline sample (one slice: ~10-30 s of numpy)


def _pmc_traffic(config: str):
    """HBM bytes per GEMM launch from the committed rocprofv3 PMC summary, if present."""
    path = os.path.join(ROOT, "profiles", "pmc_gemm.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("config") == config:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def cpu_baseline(circ_cfg: str, min_seconds: float = 12.0):
    """Oracle (numpy, complex128 pairwise tensordot) on a bounded sample of the same workload:
    the C4 network with the same path, cut and slicing and N_OPEN_CPU open outputs, timed over
    whole slices until ~min_seconds of CPU work; amplitudes/sec = 2^N_OPEN_CPU / (8 * mean
    t_slice) (the slices are identical sub-contractions, so the extrapolation is linear)."""
    import numpy as np
    from oracle.contract_ref import contract as ref_contract
    from tneq_qc_amd.circuits import BrickWall, amplitude_task
    import tneq_qc_amd.einsum as E

    circ = BrickWall(53, 20, 0)
    open_q = list(range(27 - N_OPEN_CPU // 2, 27 + N_OPEN_CPU // 2))
    t = amplitude_task(circ, open_q, cut=27, n_slice=3)
    net = t.network()
    sl = [net.symbols.index(s) for s in t.sliced]
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
    except Exception:
        threads = os.cpu_count() or 1
    eq_terms = t.eq.split("->")[0].split(",")
    terms = ["".join(ch for ch in term if ch not in t.sliced) for term in eq_terms]
    eq = ",".join(terms) + "->" + t.eq.split("->")[1]
    n_sl = 2 ** len(sl)
    ext = [net.extents[m] for m in sl]
    done, dt = 0, 0.0
    while done < n_sl and dt < min_seconds:   # whole slices until ~min_seconds of CPU work
        idx, rem = {}, done
        for s_, e_ in zip(reversed(t.sliced), reversed(ext)):
            idx[s_] = rem % e_
            rem //= e_
        ops = []
        for term, op in zip(eq_terms, t.operands):
            ix = tuple(idx[ch] if ch in t.sliced else slice(None) for ch in term)
            ops.append(np.ascontiguousarray(op[ix]))
        t0 = time.perf_counter()
        ref_contract(eq, *ops, path=t.path)
        dt += time.perf_counter() - t0
        done += 1
    n_amp = 2 ** len(open_q)
    return {
        "value": n_amp / (n_sl * dt / done),
        "unit": "amplitudes/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"oracle = numpy pairwise transpose+matmul executor (complex128, BLAS threads="
                   f"{threads}) on the C4 53q depth-20 network, same path/cut/slicing, "
                   f"{len(open_q)} open outputs ({n_amp} amplitudes); {done} of {n_sl} slices timed "
                   f"({dt:.2f} s), extrapolated linearly to all {n_sl}"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    import tneq_qc_amd
    from tneq_qc_amd import _lib
    from tneq_qc_amd.circuits import config_task
    from tneq_qc_amd.expression import HipContractExpression

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    t_plan0 = time.perf_counter()
    task = config_task(args.config)
    expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
    ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in task.operands]
    plan = expr.plan(torch.complex64)
    n_slices = plan.n_slices
    out = torch.empty(expr.out_shape, dtype=torch.complex64, device=dev)
    t_plan = time.perf_counter() - t_plan0

    from tneq_qc_amd.distributed import SlicedContraction
    job = SlicedContraction(expr)   # slices rank, rank+N, ... + one RCCL all-reduce (SUM)

    def step():
        job(*ops, out=out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    plan.profile(_lib.TQ_OP_GEMM)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    gemm = plan.profile_read(_lib.TQ_OP_GEMM)
    plan.profile(None)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # one untimed profiled step for the HBM-bound kernels (evidence for DESIGN.md)
    plan.profile(-1)
    step()
    torch.cuda.synchronize()
    kinds = {k: plan.profile_read(getattr(_lib, f"TQ_OP_{k}")) for k in ("APPLY", "SWEEP", "PERMUTE", "GEMM")}
    plan.profile(None)

    n_amp = task.n_amplitudes
    g3m = bool(_lib.lib().tq_library_query(b"gemm_3m") == 1)
    value = n_amp * args.steps / dt
    avg_gemm_s = gemm["ms"] / 1e3 / max(1, gemm["launches"])
    gemm_flops = gemm["flops"] / max(1, gemm["launches"])
    achieved = gemm_flops / avg_gemm_s / 1e12 if avg_gemm_s > 0 else 0.0
    apply_ = kinds["APPLY"]
    sweep_ = kinds["SWEEP"]
    res = {
        "metric": "amplitudes/sec + achieved MFMA TFLOP/s, 53q depth-20 RQC",
        "value": value,
        "unit": "amplitudes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "c64",
        "data": "synthetic (Haar-random 2-qubit cores, seeded; |0> inputs; seeded fixed bits)",
        "config": {
            "workload": f"{args.config}: {task.circuit.n_qubits}q depth-{task.circuit.depth} brick-wall RQC, "
                        f"{n_amp} correlated amplitudes ({len(task.open_qubits)} open), cut {task.cut}, "
                        f"{n_slices} slices ({len(task.sliced)} sliced cut legs) over {world} GPU(s), RCCL all-reduce",
            "n_qubits": task.circuit.n_qubits,
            "depth": task.circuit.depth,
            "amplitudes_per_step": n_amp,
            "slices": n_slices,
            "parallelism": f"slices{world}",
        },
        "roofline": {
            "bound": "mfma",
            "kernel": ("boundary GEMM (complex64, LDS-DMA fed v_mfma_f32_32x32x2_f32, "
                       + ("Gauss 3M: 3 real f32 MFMA per complex MAC" if g3m else "4 real f32 MFMA per complex MAC") + ")"),
            "achieved": achieved,
            "peak": PEAK_FP32_MFMA_TFLOPS,
            "unit": "TFLOP/s",
            "frac": achieved / PEAK_FP32_MFMA_TFLOPS,
            "achieved_definition": "algorithmic complex-GEMM flops 8*M*N*K per launch / avg launch time",
            "mfma_executed_tflops": achieved * (0.75 if g3m else 1.0),
            "mfma_frac": achieved * (0.75 if g3m else 1.0) / PEAK_FP32_MFMA_TFLOPS,
            "traffic": _pmc_traffic(args.config),
            "avg_launch_ms": avg_gemm_s * 1e3,
            "flops_per_launch": gemm_flops,
            "launches_timed": gemm["launches"],
        },
        "hbm_kernels": {
            "apply_GBps": (apply_["bytes"] / (apply_["ms"] / 1e3) / 1e9) if apply_["ms"] else None,
            "apply_ms_per_step": apply_["ms"],
            "sweep_GBps": (sweep_["bytes"] / (sweep_["ms"] / 1e3) / 1e9) if sweep_["ms"] else None,
            "sweep_ms_per_step": sweep_["ms"],
            "sweep_launches_per_step": sweep_["launches"],
            "permute_ms_per_step": kinds["PERMUTE"]["ms"],
            "gemm_ms_per_step": kinds["GEMM"]["ms"],
            "peak_GBps": PEAK_HBM_GBS,
        },
        "plan": {
            "compile_s": t_plan,
            "kernels_per_slice": plan.query("n_kernels"),
            "hoisted_kernels": plan.query("n_ops_once"),
            "arena_GiB": plan.query("arena_bytes") / 2 ** 30,
        },
    }
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(args.config)
        except Exception as e:  # the baseline must never hide the GPU number
            res["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
