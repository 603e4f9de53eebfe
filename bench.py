#!/usr/bin/env python3
"""bench.py — amplitudes/sec of sliced random-circuit amplitude batches on MI355X.

Workload (BASELINE.json metric "amplitudes/sec + achieved MFMA TFLOP/s, 53q depth-20 RQC"):
config C4 of SURVEY.md §8(d): a 53-qubit depth-20 brick-wall random circuit (520 Haar-random
2-qubit cores, the reference's build_brick_wall_IM + incidence_to_graph family), |0> inputs,
33 output bits fixed, 20 open (a block of 2^20 correlated bitstrings), cut between qubits 26|27,
3 cut legs sliced -> 8 slices.  One "step" = one block per rank: left/right line sweeps, the
boundary MFMA GEMM, the sweeps' deferred tails per slice (slice-invariant work hoisted).

Ranks (`--shard`):
* bitstrings (default): rank r contracts amplitude blocks r, r + N, r + 2N, ... (a different block
  every step, a window of 64 cycled) -- the same network with the closed qubits' fixed bits
  flipped by the block index's binary digits (circuits.with_batch), so one compiled plan -- over
  all its slices, four blocks in flight (`--inflight`) on their own plans and streams
  (sampling.BlockPipeline),
  with no collective on the data path: per-GPU work is fixed as N grows
  ("scaling": "weak"; value = N blocks x 2^20 amplitudes / max-over-ranks time).  The same ranks
  then time ONE block with its slices sharded over them + one RCCL all-reduce (SUM) of the
  partial amplitudes over xGMI (`slices_strong`, the reference's sliced path,
  distributed_engine.py:1384-1497).
* slices: that sliced path as the headline ("scaling": "strong").
Inputs (cores, vectors) are resident in HBM before timing.
`--config C2 / C3 / C4g / C3d` time the other amplitude configs the same way (C3 = 64 slices,
C2 = one amplitude, no slicing; C4g / C3d: other paths of the C4 / C3 networks).

Timing: the headline (`value`, `ms_per_step`) is the production launch path — every step replays
the plan's captured hipGraph, no events inside (several blocks in flight, see above).  The dominant
kernel's duration (`roofline`) is then measured in separate single-stream passes of the same steps
in which the plan launches eagerly with HIP events around every launch of that kernel kind on its
stream (the kernels are identical); rocprofv3's average for the same command, committed under
profiles/, is reported beside it (`*_rocprof`).

Output: the LAST stdout line on rank 0 is ONE compact JSON headline (<= 2 KB, `headline_line`)
with `roofline` and, at N=1, `cpu_baseline` (the oracle's numpy pairwise executor on a bounded
sample of the same network, in the same dtype) and one [value, ms, frac] triple per secondary
line; the secondary sections in full go to stderr (`[bench-detail]` lines) and, with `--details
PATH`, to a JSON file.

Ranks: under torch.distributed.run (WORLD_SIZE set) every process is one rank on cuda:LOCAL_RANK.
`--gpus N` without WORLD_SIZE launches the N ranks itself (the env launch of the reference,
comm_torch.py:146-168): N child processes started before anything touches the GPU, rank 0's JSON
line passed through.  `--devices 0,0 --dist-backend gloo` puts several ranks on one GPU (tests).
"""
from __future__ import annotations

import argparse
import math
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, f32-in MFMA
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16 / F16 dense MFMA peak (no sparsity) at 2.4 GHz
PEAK_CLOCK_GHZ = 2.4
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
N_OPEN_CPU = 20                 # open outputs in the CPU-baseline sample (one slice: ~5-15 s of numpy)


_T0 = time.perf_counter()


def _log(msg: str) -> None:
    """Progress on stderr (the JSON line stays the only stdout line): one line per phase."""
    print(f"[bench {time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def _profile_json(name: str, config: str):
    """A committed rocprofv3 PMC summary under profiles/ (or None)."""
    path = os.path.join(ROOT, "profiles", name)
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("config") == config:
            return d
    except Exception:
        pass
    return None


def _rocprof_avg_ns(name: str, kernel: str):
    """Average duration (ns) over every dispatch of kernels whose name contains `kernel` in a
    committed rocprofv3 --stats CSV under profiles/ (or None)."""
    import csv
    try:
        calls, tot = 0, 0.0
        with open(os.path.join(ROOT, "profiles", name)) as f:
            for r in csv.DictReader(f):
                if kernel in r["Name"]:
                    calls += int(r["Calls"])
                    tot += float(r["TotalDurationNs"])
        return tot / calls if calls else None
    except Exception:
        return None


ROCPROF_STATS = "rocprof_r06_bench_kernel_stats.csv"   # rocprofv3 --kernel-trace --stats of the bench command


def _kernel_clock():
    """In-kernel clocks of the benchmarked kernels (scripts/kernel_clock.py, committed)."""
    try:
        with open(os.path.join(ROOT, "profiles", "kclock_r06.json")) as f:
            return json.load(f)
    except Exception:
        return None


def _cgroup_cpu_max():
    """The cgroup v2 CPU quota of this process ("max 100000" = none), if readable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            return f.read().strip()
    except Exception:
        return None


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def _cpu_sample(t, n_sl, min_seconds, threads):
    """The oracle's complex64 executor on the sliced job at `threads` BLAS threads, hoisting the
    slice-invariant steps once as the GPU plan does (oracle.contract_ref.contract_sliced): the
    whole job timed when it fits ~min_seconds (repeated up to that budget), else one slice and two
    slices timed and the per-slice part extrapolated to all slices.  Returns (seconds per whole job,
    sample description, BLAS threads in effect)."""
    import numpy as np
    from oracle.contract_ref import contract_sliced
    from threadpoolctl import threadpool_info, threadpool_limits
    ops64 = [o.astype(np.complex64) for o in t.operands]
    sliced = list(t.sliced)

    def run(ids):
        t0 = time.perf_counter()
        contract_sliced(t.eq, ops64, sliced, t.path, slice_ids=ids, exact=False)
        return time.perf_counter() - t0

    with threadpool_limits(limits=threads):
        used = max([i.get("num_threads", 1) for i in threadpool_info()] + [1])
        t1 = run([0])
        t2 = run([0, 1]) if n_sl > 1 else t1
        per = max(t2 - t1, 0.0) if n_sl > 1 else t1
        once = max(t1 - per, 0.0)
        if once + n_sl * per <= min_seconds:
            done, dt = 0, 0.0
            while done == 0 or dt < 0.5 * min_seconds:
                dt += run(list(range(n_sl)))
                done += 1
            return dt / done, f"the whole job ({n_sl} slices, hoisted steps once) timed {done}x ({dt:.2f} s)", used
        return once + n_sl * per, (f"1 and 2 slices timed ({t1:.2f} / {t2:.2f} s): hoisted part {once:.2f} s "
                                   f"+ {n_sl} x {per:.2f} s per slice"), used


def cpu_baseline(circ_cfg: str, min_seconds: float = 12.0):
    """Oracle (numpy pairwise transpose+matmul, complex64 — the GPU path's dtype) on a bounded
    sample of the same workload: the config's network with the same path, cut and slicing,
    timed over whole slices until ~min_seconds of CPU work; amplitudes/sec = n_amplitudes /
    (n_slices * mean t_slice) (the slices are identical sub-contractions, so the extrapolation is
    linear).  Timed twice: at BLAS threads = os.cpu_count() (every host core) and
    at 16 threads (the box's CPU share per GPU: its cgroup quota is reported); `value` / `cores`
    are the faster of the two, both are reported."""
    from tneq_qc_amd.circuits import config_task

    t = config_task(circ_cfg)
    n_sl = 1
    ext = {}
    for term, op in zip(t.eq.split("->")[0].split(","), t.operands):
        for ch, e in zip(term, op.shape):
            ext[ch] = e
    for s in t.sliced:
        n_sl *= ext[s]
    host = os.cpu_count() or 1
    n_amp = t.n_amplitudes
    runs = []
    for th in sorted({host, min(16, host)}, reverse=True):
        _log(f"cpu baseline at {th} BLAS threads")
        job_s, sample, used = _cpu_sample(t, n_sl, min_seconds if th == host else min_seconds / 2, th)
        runs.append({"value": n_amp / job_s, "cores": used, "sample": sample})
    best = max(runs, key=lambda r: r["value"])
    return {
        "value": best["value"],
        "unit": "amplitudes/s",
        "cores": best["cores"],
        "kind": "port",
        "host_cpus": host,
        "host_cpus_affinity": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None,
        "cgroup_cpu_max": _cgroup_cpu_max(),
        "cpu_model": _cpu_model(),
        "by_threads": runs,
        "sample": (f"oracle = numpy pairwise transpose+matmul executor in complex64 (the GPU dtype) on "
                   f"the {circ_cfg} network, same path/cut/slicing, {n_amp} amplitudes, slice-invariant steps "
                   f"once per job (as the GPU plan hoists them); {n_sl} slices, at BLAS threads = every host core "
                   f"({host}) and = 16; value = the faster ({best['cores']} threads: {best['sample']})"),
    }


def permute_probe(dev, rank: int = 26, reps: int = 5):
    """tq_permute on a rank-`rank` binary-leg complex64 tensor (2^rank elements) with a seeded
    random permutation, through a one-op plan: HIP-event kernel time, algorithmic bytes
    2 * numel * 8 (north_star: "rocprof HBM GB/s on the permute")."""
    import numpy as np
    import torch
    from tneq_qc_amd import _lib
    from tneq_qc_amd.einsum import get_symbol
    from tneq_qc_amd.expression import HipContractExpression

    rng = np.random.default_rng(26)
    p = rng.permutation(rank)
    s = "".join(get_symbol(i) for i in range(rank))
    e = HipContractExpression(s + "->" + "".join(s[i] for i in p), (2,) * rank)
    x = torch.randn((2,) * rank, dtype=torch.complex64, device=dev)
    y = torch.empty((2,) * rank, dtype=torch.complex64, device=dev)
    e(x, out=y)
    plan = e.plan(torch.complex64)
    plan.profile(_lib.TQ_OP_PERMUTE)
    for _ in range(reps):
        e(x, out=y)
    torch.cuda.synchronize()
    r = plan.profile_read(_lib.TQ_OP_PERMUTE)
    plan.profile(None)
    ok = bool(torch.equal(y.cpu(), x.cpu().permute(*p.tolist()).contiguous()))
    gbs = r["bytes"] / (r["ms"] / 1e3) / 1e9
    del x, y
    return {"rank": rank, "numel": 2 ** rank, "dtype": "c64", "perm": [int(v) for v in p],
            "avg_launch_ms": r["ms"] / r["launches"], "GBps": gbs, "frac": gbs / PEAK_HBM_GBS,
            "bit_exact": ok}


def c5_train(with_cpu: bool = True, steps: int = 20, warmup: int = 5, port: int = 0, rank: int = 0):
    """Secondary line (BASELINE.json configs[4], C5): the symmetry-breaking training step —
    8 pruning candidates x (split/merge core-only forward, fidelity loss, reverse-mode backward,
    SGDG) in complex128, each candidate on its own stream; on N ranks candidate k runs on rank
    k mod N (every rank of this bench runs its share) — next to the same step on the host CPU.
    Runs scripts/c5_bench.py in a child process per rank (started without exec, inheriting
    RANK / WORLD_SIZE / LOCAL_RANK): a fresh caching allocator, so the candidates' buffers (and
    the hipGraphs keyed on their pointers) settle during the warmup instead of inheriting the C4
    run's pool."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "c5_bench.py"), "--steps", str(steps),
           "--warmup", str(warmup), "--cpu-steps", "1" if with_cpu else "0", "--port", str(port)]
    # stdout carries the child's JSON line; its stderr (progress) passes through
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=300)
    if rank != 0:
        return None
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    out = {"metric": "candidate training steps/s (forward + backward + SGDG), C5 ansatz, 8 candidates",
           "value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"], "steps": steps,
           "warmup": warmup, "n_gpus": d.get("n_gpus", 1), "candidates_per_rank": d.get("candidates_per_rank"),
           "dtype": d["dtype"], "cores_per_candidate": d["cores_per_candidate"],
           "streams": d.get("streams", 1), "forward": d.get("forward"),
           "amplitudes_per_forward": d["amplitudes_per_forward"],
           "host_issue_ms_per_step": d.get("host_issue_ms_per_step"),
           "wall_ms_per_step_per_rank": d.get("wall_ms_per_step_per_rank"),
           "step_graphs": d.get("step_graphs"),
           "bound": "latency (2^16-element tensors; ~100 dependent pairwise launches per candidate-step, "
                    "forward + loss + backward replayed as one hipGraph per candidate, SGDG eager; a rank's "
                    "candidates overlap on their own streams)",
           "launches_per_candidate_step": d.get("launches_per_candidate_step"),
           "algorithmic_bytes_per_candidate_step": d.get("algorithmic_bytes_per_candidate_step")}
    ab = d.get("algorithmic_bytes_per_candidate_step")
    if ab:
        gbs = ab * d["value"] / 1e9
        out["roofline"] = {"bound": "hbm", "kernel": "every native launch of the training step (aggregate)",
                           "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                           "achieved_definition": "algorithmic bytes of the step's plans (tq_plan bytes_moved) x "
                                                  "candidate-steps/s",
                           "traffic": None}
        pm_src = "pmc_c5_r06.json" if _profile_json("pmc_c5_r06.json", "C5") else "pmc_c5_r05.json"
        pm = _profile_json(pm_src, "C5")
        if pm and pm.get("hbm_bytes_per_candidate_step"):
            # HBM bytes per candidate-step (2*FETCH_SIZE + WRITE_SIZE over every kernel of a
            # c5_bench run / its SGDG dispatches; rocprofv3 PMC passes, scripts/pmc_traffic.sh)
            out["roofline"]["traffic"] = pm["hbm_bytes_per_candidate_step"]
            out["roofline"]["traffic_unit"] = "bytes per candidate-step"
            out["roofline"]["traffic_vs_algorithmic"] = pm["hbm_bytes_per_candidate_step"] / ab
            out["roofline"]["traffic_source"] = f"profiles/{pm_src}"
    tr = _profile_json("c5_trace_r04.json", "C5")
    if tr:
        out["gpu_busy_frac"] = tr.get("gpu_busy_frac")
        out["trace_launches_per_candidate_step"] = tr.get("launches_per_candidate_step")
        out["trace_source"] = "profiles/c5_trace_r04.json"
    if "cpu_baseline" in d:
        out["cpu_baseline"] = dict(d["cpu_baseline"], cpu_model=_cpu_model())
    return out


def _child_details(cmd, env=None) -> dict:
    """Run a child bench.py (no exec) and return its full result (its --details file)."""
    import subprocess
    import tempfile
    fd, path = tempfile.mkstemp(suffix=".json", prefix="bench_child_")
    os.close(fd)
    try:
        r = subprocess.run(cmd + ["--details", path], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise RuntimeError(f"child bench rc {r.returncode}: {r.stderr[-400:]}")
        with open(path) as f:
            return json.load(f)
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass


def alt_gemm(args, envs: dict, desc: str, cfg: str):
    """Config `cfg` with another complex64 boundary-GEMM kernel (library switches in `envs`,
    read once per process: a child process, started without exec)."""
    import subprocess
    env = dict(os.environ, **envs)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg, "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--no-cpu-baseline", "--no-c5", "--no-alt", "--no-other"]
    d = _child_details(cmd, env)
    return {"config": cfg, "value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"],
            "gemm": f"{desc} ({' '.join(f'{k}={v}' for k, v in envs.items())})", "roofline": d["roofline"]}


def other_config(args, cfg: str):
    """BASELINE.json's other amplitude configs (C2: 30q depth-14, one amplitude, no slicing;
    C3: 40q depth-16, 64 slices) timed the same way on the same box, in a child process (each
    builds its own plan and arena); the headline stays C4."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", cfg, "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--no-c5", "--no-alt", "--no-other",
           "--cpu-seconds", str(args.other_cpu_seconds)]
    if args.no_cpu_baseline:
        cmd.append("--no-cpu-baseline")
    d = _child_details(cmd)
    return {k: d[k] for k in ("value", "unit", "ms_per_step", "config", "roofline", "hbm_kernels", "cpu_baseline",
                              "plan") if k in d}


def launch_ranks(args, argv) -> int:
    """`--gpus N` without a launcher: start the N ranks as child processes (no exec, and nothing
    in this parent touches the GPU), rank 0's output passed through; exit status = the worst
    rank's."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--devices", default=None,
                    help="comma list: the GPU of each local rank (default: local rank i on cuda:i)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group backend for N > 1 (nccl = RCCL over xGMI)")
    ap.add_argument("--save-out", default=None, help="rank 0 saves the last step's amplitudes (.npy)")
    ap.add_argument("--steps", type=int, default=50)   # steady state with four blocks in flight (10: +10 % per step)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="C4", choices=["C2", "C3", "C4", "C3d", "C4g", "C4x4"],
                    help="C4g: C4 on the big-boundary-GEMM path (each half swept whole); "
                         "C3d: C3 with deferred sweep tails; C4x4: 4 C4 blocks per contraction "
                         "(circuits.config_task)")
    ap.add_argument("--shard", default="bitstrings", choices=["bitstrings", "slices"],
                    help="N > 1: bitstrings = rank r contracts its own amplitude block (circuits."
                         "with_batch: other fixed bits, same plan), no collective (weak scaling); "
                         "slices = one block, its slices sharded over the ranks + one RCCL all-reduce "
                         "(strong scaling; also measured as `slices_strong` in bitstrings mode)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="bitstring sharding: blocks in flight per GPU -- M plans (own arenas), step k "
                         "on plan k %% M's stream (each step one whole block; the sweeps are latency-"
                         "bound, so other blocks fill the idle CUs: 2 / 3 / 4 in flight 0.468 / 0.416 / 0.411 ms per "
                         "block); 1 = one stream")
    ap.add_argument("--group", type=int, default=1,
                    help="bitstring sharding: blocks per lockstep group (blocks as lanes: every sweep level "
                         "of the group's blocks is one launch, tq_plan_execute_group); a step is still one "
                         "block, a group is launched when its last block is enqueued")
    ap.add_argument("--batch", type=int, default=0,
                    help="bitstring sharding: rank r contracts block batch + r (tests: a 1-rank run of "
                         "another rank's block)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 training-step line")
    ap.add_argument("--no-alt", action="store_true",
                    help="skip the f32-MFMA GEMM headline (TQ_GEMM_BF16=0, a child process)")
    ap.add_argument("--no-other", action="store_true",
                    help="skip the C2 / C3 secondary lines (child processes, N=1 only)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="CPU-baseline sample budget (seconds of oracle work at every host core)")
    ap.add_argument("--details", default=None,
                    help="write the full result (every secondary section) to this JSON file; stdout's "
                         "last line is the compact headline either way")
    ap.add_argument("--other-cpu-seconds", type=float, default=4.0,
                    help="CPU-baseline budget of the C2 / C3 secondary lines")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using the world size", file=sys.stderr)
    dev_id = int(args.devices.split(",")[local_rank]) if args.devices else local_rank

    import torch
    import torch.distributed as dist
    import tneq_qc_amd
    from tneq_qc_amd import _lib
    from tneq_qc_amd.circuits import config_task
    from tneq_qc_amd.expression import HipContractExpression

    torch.cuda.set_device(dev_id)
    dev = torch.device("cuda", dev_id)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from tneq_qc_amd.circuits import with_batch
    from tneq_qc_amd.distributed import SlicedContraction

    t_plan0 = time.perf_counter()
    base = config_task(args.config)
    bitstrings = args.shard == "bitstrings"
    inflight = max(1, args.inflight) if bitstrings else 1
    group = max(1, args.group) if bitstrings else 1
    pipe = None
    if bitstrings:
        # bitstring sharding (sampling.BlockPipeline): rank r contracts blocks batch + r + N k, k =
        # 0, 1, ... (a window of >= 64 distinct blocks, cycled) -- the same network with other
        # fixed bits -- `group` blocks per lockstep group (one launch per sweep level for all of
        # them), `inflight` groups on their own streams and plans
        from tneq_qc_amd.sampling import BlockPipeline
        pipe = BlockPipeline(base, [args.batch + rank + world * k for k in range(max(64, inflight * group))],
                             inflight=inflight, group=group, device=dev)
        task = with_batch(base, args.batch + rank)
        expr, bound0, out = pipe.expr, pipe.slots[0].bound[0], pipe.slots[0].outs[0]
        ops = list(bound0.tensors)
        pipe.step()   # slot 0 member 0's projector buffer holds block batch + r (the latency / profiled passes)
        pipe.reset()
        pipe.synchronize()
        plan = bound0.plan
    else:
        task = with_batch(base, args.batch) if args.batch else base
        expr = HipContractExpression(task.eq, *task.shapes, optimize=task.path, slices=task.sliced)
        ops = [torch.from_numpy(o).to(dev, torch.complex64) for o in task.operands]
        out = torch.empty(expr.out_shape, dtype=torch.complex64, device=dev)
        plan = expr.plan(torch.complex64)

    n_slices = plan.n_slices
    t_plan = time.perf_counter() - t_plan0

    def slices_job():
        """One block's slices rank, rank+N, ... + one RCCL all-reduce (SUM).  N > 1: consecutive
        steps alternate two output buffers and leave their all-reduce in flight (async): step k's
        RCCL reduce overlaps step k + 1's contraction, a buffer is reused only after its reduce has
        been waited for; the timed region still ends with a device synchronize."""
        job = SlicedContraction(expr)
        ops0 = ops if not bitstrings else [torch.from_numpy(o).to(dev, torch.complex64) for o in base.operands]
        bufs = [out, torch.empty_like(out)] if world > 1 else [out]
        works = [None] * len(bufs)
        nstep = [0]

        def step():
            i = nstep[0] % len(bufs)
            if world > 1:
                if works[i] is not None:
                    works[i].wait()
                _, works[i] = job(*ops0, out=bufs[i], async_reduce=True)
            else:
                job(*ops0, out=out)
            nstep[0] += 1

        def last():
            for w in works:
                if w is not None:
                    w.wait()
            return bufs[(nstep[0] - 1) % len(bufs)]
        return step, last

    def step1():
        """One block on the current stream (slot 0 member 0's plan): the latency pass and the
        profiled passes."""
        if bitstrings:
            bound0.run(out)
        else:
            expr(*ops, out=out)

    if bitstrings:
        def step():
            pipe.step()

        def last_out():
            # block batch + r again on slot 0 (the saved block is deterministic per rank)
            pipe.synchronize()
            pipe.reset()
            o = pipe.step()
            pipe.synchronize()
            return o
    else:
        step, last_out = slices_job()

    def timed(k: int, fn=None) -> float:
        fn = fn or step
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        if pipe is not None:
            pipe.flush()   # a partially filled group is launched inside the timed region
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    _log(f"plan compiled in {t_plan:.1f} s ({n_slices} slices); warmup")
    for _ in range(args.warmup):
        step()
    # ---- headline: production path (hipGraph replay per step, no events)
    dt = max_over_ranks(timed(args.steps))
    graphs = plan.query("graph_launches")
    if args.save_out:
        res = last_out()
        import numpy as np
        if rank == 0:
            np.save(args.save_out, res.cpu().numpy())
        elif bitstrings:   # every rank's own block (tests check each against the 1-rank blocks)
            root, ext = os.path.splitext(args.save_out)
            np.save(f"{root}.rank{rank}{ext}", res.cpu().numpy())
    slices_strong = None
    if bitstrings and world > 1:
        # the same ranks on ONE block, its slices sharded + the RCCL all-reduce (strong scaling)
        s_step, s_last = slices_job()
        for _ in range(args.warmup):
            s_step()
        dts = max_over_ranks(timed(args.steps, s_step))
        res_s = s_last()
        if args.save_out and rank == 0:
            import numpy as np
            root, ext = os.path.splitext(args.save_out)
            np.save(f"{root}.slices{ext}", res_s.cpu().numpy())
        slices_strong = {"value": base.n_amplitudes * args.steps / dts, "unit": "amplitudes/s",
                         "ms_per_step": dts / args.steps * 1e3, "scaling": "strong",
                         "parallelism": f"slices{world}", "slices_per_rank": len(range(rank, n_slices, world)),
                         "collective": f"RCCL all-reduce (SUM) of the {base.n_amplitudes}-amplitude partials"
                                       if args.dist_backend == "nccl" else "gloo all-reduce (SUM)"}
        _log(f"slices (strong) on one block: {dts / args.steps * 1e3:.2f} ms/step")

    _log(f"headline: {dt / args.steps * 1e3:.2f} ms/step ({inflight} groups of {group} in flight)")
    # ---- one block at a time (one stream): the latency of a step
    dt_lat = max_over_ranks(timed(args.steps, step1)) if inflight * group > 1 else dt
    # ---- dominant kernel: the same K steps launched eagerly (one stream) with HIP events around
    # every GEMM
    plan.profile(_lib.TQ_OP_GEMM)
    dt_prof = timed(args.steps, step1)
    gemm = plan.profile_read(_lib.TQ_OP_GEMM)
    plan.profile(None)

    # ---- one profiled step for the HBM-bound kernels (evidence for DESIGN.md)
    plan.profile(-1)
    step1()
    torch.cuda.synchronize()
    kinds = {k: plan.profile_read(getattr(_lib, f"TQ_OP_{k}")) for k in ("APPLY", "SWEEP", "PERMUTE", "GEMM")}
    plan.profile(None)

    n_amp = task.n_amplitudes * (world if bitstrings else 1)   # amplitudes of the whole job per step
    L = _lib.lib()
    g3m = bool(L.tq_library_query(b"gemm_3m") == 1)
    bf16 = bool(L.tq_library_query(b"gemm_bf16") == 1)
    f16 = bf16 and bool(L.tq_library_query(b"gemm_f16") == 1)
    f16_g3 = f16 and L.tq_library_query(b"gemm_f16_var") in (2, 5, 6, 7, 8, 9)   # Gauss 3M on the f16 terms
    planes = plan.query("planes_active") == 1   # the pre-split boundary GEMM (tq_gemmp.hip)
    value = n_amp * args.steps / dt
    nl = max(1, gemm["launches"])
    avg_gemm_s = gemm["ms"] / 1e3 / nl
    alg_flops = gemm["flops"] / nl                      # 8*M*N*K complex GEMM flops per launch
    # MFMA work executed per launch: f16 split = 4 real products x 3 term products = 24*M*N*K;
    # bf16 split = 4 x 6 = 48*M*N*K; f32 3M = 6*M*N*K, f32 4M = 8*M*N*K
    exe_flops = alg_flops * (2.25 if (planes or f16_g3) else 3.0 if f16 else 6.0 if bf16 else (0.75 if g3m else 1.0))
    peak = PEAK_BF16_MFMA_TFLOPS if bf16 else PEAK_FP32_MFMA_TFLOPS
    achieved = exe_flops / avg_gemm_s / 1e12 if avg_gemm_s > 0 else 0.0
    alg_rate = alg_flops / avg_gemm_s / 1e12 if avg_gemm_s > 0 else 0.0
    if planes:
        peak = PEAK_BF16_MFMA_TFLOPS
        pmc_b = _profile_json("pmc_gemm_planes_r05.json", args.config)
        pmc_t = pmc_b
        kdesc = ("boundary GEMM on pre-split operands (complex64: the dense producers store each operand as six "
                 "f16 term planes of its power-of-two-scaled re, im, re+im; Gauss's 3 real products x 3 term "
                 "products (hh, hl, lh) on v_mfma_f32_16x16x32_f16, f32 accumulation, LDS-DMA staged 256x256 "
                 "tiles, split-K partials + one combine pass that also sums the slice lanes)")
        exe_def = ("executed f16 MFMA flops per launch (3 real products (Gauss) x 3 term products = 18*M*N*K) / "
                   "avg launch time of the GEMM + combine")
    elif f16:
        pmc_b = (_profile_json("pmc_gemm_f16_r06.json", args.config) or _profile_json("pmc_gemm_f16_r04g.json", args.config)
                 if f16_g3 else _profile_json("pmc_gemm_f16_r02.json", args.config))
        pmc_t = pmc_b
        kdesc = ("boundary GEMM (complex64 on v_mfma_f32_32x32x16_f16: every f32 operand scaled by a power of two "
                 "(operand max from its producer sweep) and split into 2 f16 terms, 3 term products kept, f32 "
                 "accumulation; " + ("Gauss's 3 real products per complex product: P1 = Ar Br, P2 = Ai Bi, "
                                     "P3 = (Ar + Ai)(Br + Bi)" if f16_g3 else "4 real products per complex product")
                 + ")")
        exe_def = ("executed f16 MFMA flops per launch (" + ("3 real products (Gauss) x 3 term products = 18*M*N*K"
                   if f16_g3 else "4 real products x 3 term products = 24*M*N*K") + ") / avg launch time")
    elif bf16:
        pmc_b = _profile_json("pmc_gemm_bf16_r02.json", args.config)
        pmc_t = pmc_b
        kdesc = ("boundary GEMM (complex64 on v_mfma_f32_32x32x16_bf16: every f32 operand split exactly into "
                 "3 bf16 terms, 6 term products kept, f32 accumulation; 4 real products per complex product)")
        exe_def = "executed bf16 MFMA flops per launch (4 real products x 6 term products = 48*M*N*K) / avg launch time"
    else:
        pmc_t = _profile_json("pmc_gemm.json", args.config)
        pmc_b = _profile_json("pmc_gemm_busy_r02.json", args.config)
        kdesc = ("boundary GEMM (complex64, LDS-DMA fed v_mfma_f32_32x32x2_f32, "
                 + ("Gauss 3M: 3 real f32 MFMA GEMMs per complex GEMM" if g3m
                    else "4 real f32 MFMA GEMMs per complex GEMM") + ")")
        exe_def = "executed MFMA flops per launch (3M: 6*M*N*K, 4M: 8*M*N*K real) / avg launch time"
    # the GEMM's clock: measured inside the kernel (s_memtime / s_memrealtime, scripts/kernel_clock.py,
    # profiles/kclock_r06.json), not GRBM_GUI_ACTIVE / 8 / duration (unphysical for short dispatches)
    kcl = _kernel_clock()
    clk = None
    if kcl:
        kname = "gemm_planes_kernel" if planes else "gemm_c64_kouter_split_kernel"
        for sect in kcl.values():
            if isinstance(sect, dict) and isinstance(sect.get(kname), dict):
                clk = sect[kname].get("clock_GHz_median")
    gemm_rp = None
    if planes and args.config == "C4g":
        # rocprofv3 average of the same launch (GEMM + combine) from the committed kernel stats of
        # this path's bench command (r05, when it was the C4 default)
        g_ns = _rocprof_avg_ns("rocprof_r05_bench_kernel_stats.csv", "gemm_planes_kernel")
        c_ns = _rocprof_avg_ns("rocprof_r05_bench_kernel_stats.csv", "planes_combine_kernel")
        if g_ns and c_ns:
            gemm_rp = (g_ns + c_ns) / 1e6
    apply_ = kinds["APPLY"]
    sweep_ = kinds["SWEEP"]
    perm_ = kinds["PERMUTE"]
    res = {
        "metric": "amplitudes/sec + achieved MFMA TFLOP/s, 53q depth-20 RQC",
        "value": value,
        "unit": "amplitudes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak" if args.shard == "bitstrings" else "strong",
        "vs_baseline": None,
        "dtype": "c64",
        "data": "synthetic (Haar-random 2-qubit cores, seeded; |0> inputs; seeded fixed bits)",
        "config": {
            "workload": (f"{args.config}: {task.circuit.n_qubits}q depth-{task.circuit.depth} brick-wall RQC, "
                         f"{task.n_amplitudes} correlated amplitudes per block ({len(task.open_qubits)} open), "
                         f"cut {task.cut}, {n_slices} slices ({len(task.sliced)} sliced cut legs); "
                         + (f"{world} GPU(s), one block per rank (bitstring sharding, no collective)" if bitstrings
                            else f"{world} GPU(s), slices sharded, RCCL all-reduce")),
            "n_qubits": task.circuit.n_qubits,
            "depth": task.circuit.depth,
            "amplitudes_per_step": n_amp,
            "amplitudes_per_block": task.n_amplitudes,
            "blocks_per_step": world if bitstrings else 1,
            "slices": n_slices,
            "parallelism": f"bitstrings{world}" if bitstrings else f"slices{world}",
            "slices_per_rank": n_slices if bitstrings else len(range(rank, n_slices, world)),
        },
        "timing": {
            "headline": ("hipGraph replay of the whole plan per step (production path), no events"
                         + (f"; {group} blocks per lockstep group (blocks as lanes), {inflight} groups in flight "
                            f"per GPU on their own streams (each step one whole block)" if inflight * group > 1 else "")),
            "graph_launches_timed": graphs,
            "eager_profiled_ms_per_step": dt_prof / args.steps * 1e3,
            "inflight": inflight,
            "group": group,
            "latency_ms_per_step": dt_lat / args.steps * 1e3,
            "latency_definition": "the same K steps one block at a time on one stream (no overlap of steps)",
        },
        "roofline": {
            "bound": "mfma",
            "kernel": kdesc,
            "achieved": achieved,
            "peak": peak,
            "unit": "TFLOP/s",
            "frac": achieved / peak,
            "achieved_definition": exe_def + " (HIP events on the GEMM's stream, eager pass)",
            "clock_GHz_in_kernel": clk,
            "frac_at_measured_clock": (achieved / (peak * clk / PEAK_CLOCK_GHZ)) if clk else None,
            "algorithmic_tflops": alg_rate,
            "algorithmic_definition": "complex-GEMM flops 8*M*N*K per launch / avg launch time",
            "mfma_busy_pmc": (pmc_b or {}).get("mfma_busy_frac"),
            "traffic": (pmc_t or {}).get("hbm_bytes_per_launch"),
            "avg_launch_ms": avg_gemm_s * 1e3,
            "avg_launch_ms_rocprof": gemm_rp,
            "frac_rocprof": (exe_flops / (gemm_rp / 1e3) / 1e12 / peak) if gemm_rp else None,
            "flops_per_launch_algorithmic": alg_flops,
            "flops_per_launch_executed": exe_flops,
            "launches_timed": gemm["launches"],
        },
        "hbm_kernels": {
            "apply_GBps": (apply_["bytes"] / (apply_["ms"] / 1e3) / 1e9) if apply_["ms"] else None,
            "apply_ms_per_step": apply_["ms"],
            "sweep_GBps": (sweep_["bytes"] / (sweep_["ms"] / 1e3) / 1e9) if sweep_["ms"] else None,
            "sweep_ms_per_step": sweep_["ms"],
            "sweep_launches_per_step": sweep_["launches"],
            "permute_ms_per_step": perm_["ms"],
            "gemm_ms_per_step": kinds["GEMM"]["ms"],
            "peak_GBps": PEAK_HBM_GBS,
        },
        "plan": {
            "compile_s": t_plan,
            "kernels_per_slice": plan.query("n_kernels"),
            "hoisted_kernels": plan.query("n_ops_once"),
            "launches_once": plan.query("n_launch_once"),
            "launches_per_slice": plan.query("n_launch_slice"),
            "arena_GiB": plan.query("arena_bytes") / 2 ** 30,
        },
    }
    # the dominant kernel by time: on C4 the boundary GEMM; on the latency-bound small configs
    # (C2: no GEMM at all, C3: 64 small slices) the sweeps, priced against HBM
    if sweep_["ms"] > kinds["GEMM"]["ms"]:
        gbps = sweep_["bytes"] / (sweep_["ms"] / 1e3) / 1e9 if sweep_["ms"] else 0.0
        res["roofline_gemm"] = res["roofline"]
        res["roofline"] = {
            "bound": "hbm",
            "kernel": "sweep2 (fused multi-gate butterfly sweeps; the dominant kernel of this config by time)",
            "achieved": gbps,
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": gbps / PEAK_HBM_GBS,
            "achieved_definition": "algorithmic bytes (numel(X) + numel(Y)) * 8 over every sweep launch of one "
                                   "profiled step / their summed HIP-event time",
            "traffic": None,
            "launches_timed": sweep_["launches"],
            "ms_per_step": sweep_["ms"],
            "algorithmic_bytes_per_step": sweep_["bytes"],
        }
        if sweep_["ms"] and sweep_["flops"]:
            # the same launches against the FP32 vector roof: the gate arithmetic (complex MACs x 8
            # flops, tq_plan.cpp emit_s2) over the same event time; arithmetic intensity vs the
            # ridge point says which roof binds (above the ridge: VALU, below: HBM)
            tf = sweep_["flops"] / (sweep_["ms"] / 1e3) / 1e12
            ai = sweep_["flops"] / max(1.0, sweep_["bytes"])
            ridge = PEAK_FP32_MFMA_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)
            attain = min(PEAK_FP32_MFMA_TFLOPS, ai * PEAK_HBM_GBS / 1e3)   # TFLOP/s
            res["roofline"].update({
                "flops_per_step_algorithmic": sweep_["flops"],
                "achieved_tflops": tf,
                "valu_fp32_peak_tflops": PEAK_FP32_MFMA_TFLOPS,
                "frac_valu": tf / PEAK_FP32_MFMA_TFLOPS,
                "arith_intensity_flop_per_byte": ai,
                "ridge_flop_per_byte": ridge,
                "frac_of_attainable": tf / attain,
                "attainable_definition": "min(FP32 vector peak, intensity x 8 TB/s): the roof that binds "
                                         "at this arithmetic intensity (sweep2 is latency-bound under both)",
            })
        # rocprofv3 kernel stats of the default bench command (scripts/prof_round.sh r05f): the
        # average sweep2 launch there, priced with this step's algorithmic bytes per launch
        st = _rocprof_avg_ns(ROCPROF_STATS, "sweep2_kernel") if args.config == "C4" else None
        if st and sweep_["launches"]:
            per_launch = sweep_["bytes"] / sweep_["launches"]
            res["roofline"]["avg_launch_us_events"] = sweep_["ms"] / sweep_["launches"] * 1e3
            res["roofline"]["avg_launch_us_rocprof"] = st / 1e3
            res["roofline"]["achieved_rocprof"] = per_launch / (st / 1e9) / 1e9
            res["roofline"]["frac_rocprof"] = res["roofline"]["achieved_rocprof"] / PEAK_HBM_GBS
            res["roofline"]["rocprof_source"] = f"profiles/{ROCPROF_STATS} (sweep2_kernel, all forms)"
        pmc_s = None
        for tag in ("r06", "r05", "r04"):
            src = f"pmc_{args.config.lower()}_{tag}.json"
            pmc_s = _profile_json(src, args.config)
            if pmc_s:
                break
        if pmc_s and not pmc_s.get("sweep_dispatches") and pmc_s.get("groups"):
            # a scripts/prof_round.sh summary: per launch shape, the average HBM bytes of a dispatch
            g2 = [g for g in pmc_s["groups"] if g.get("family") == "sweep2" and g.get("hbm_bytes") is not None]
            nd = sum(g["dispatches"] for g in g2)
            if nd:
                pmc_s = dict(pmc_s, sweep_dispatches=nd,
                             sweep_hbm_bytes=sum(g["hbm_bytes"] * g["dispatches"] for g in g2))
        if pmc_s and pmc_s.get("sweep_dispatches"):
            # HBM bytes of the sweep launches (2*FETCH_SIZE + WRITE_SIZE, rocprofv3 PMC passes of
            # this command), per launch x this step's launches
            per = pmc_s["sweep_hbm_bytes"] / pmc_s["sweep_dispatches"]
            res["roofline"]["traffic"] = per * sweep_["launches"]
            res["roofline"]["traffic_unit"] = "bytes per step (sweep launches)"
            res["roofline"]["traffic_vs_algorithmic"] = per * sweep_["launches"] / max(1.0, sweep_["bytes"])
            res["roofline"]["traffic_source"] = f"profiles/{src}"
        # the concurrency-aware rate of the headline: the step's algorithmic sweep bytes over the
        # measured time per step WITH the blocks in flight (several launches overlap: the
        # per-launch `achieved` is the one-launch-at-a-time rate)
        agg = sweep_["bytes"] / (dt / args.steps) / 1e9 if dt > 0 else 0.0
        res["roofline"]["aggregate_GBps"] = agg
        res["roofline"]["aggregate_frac"] = agg / PEAK_HBM_GBS
        res["roofline"]["aggregate_definition"] = ("algorithmic sweep bytes per step / ms_per_step of the headline "
                                                   "(blocks in flight overlap their launches)")
        if kcl and isinstance(kcl.get("C4_headline_regime", {}).get("sweep2_kernel"), dict):
            res["roofline"]["clock_GHz_in_kernel"] = kcl["C4_headline_regime"]["sweep2_kernel"].get("clock_GHz_median")
    if slices_strong:
        res["slices_strong"] = slices_strong
    if rank == 0:
        _log("permute probe")
        try:
            res["permute"] = permute_probe(dev)
        except Exception as e:  # the probe must never hide the headline
            res["permute"] = {"error": repr(e)}
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        _log("cpu baseline")
        try:
            res["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        except Exception as e:  # the baseline must never hide the GPU number
            res["cpu_baseline"] = {"error": repr(e)}
    if world == 1 and rank == 0 and f16 and not args.no_alt and args.config in ("C4", "C4g"):
        # the other boundary-GEMM kernels on the big-GEMM path's operands (C4g; no producer-written
        # planes: the GEMM splits its operands itself)
        for key, envs, desc in (
                ("alt_f16_gemm_side_split", {"TQ_GEMM_PLANES": "0"},
                 "f16 split inside the GEMM, Gauss 3M on v_mfma_f32_32x32x16_f16 (the r04 default)"),
                ("alt_bf16_split", {"TQ_GEMM_PLANES": "0", "TQ_GEMM_F16": "0"},
                 "bf16 3-term split, v_mfma_f32_32x32x16_bf16"),
                ("alt_f32_mfma", {"TQ_GEMM_PLANES": "0", "TQ_GEMM_BF16": "0"}, "v_mfma_f32_32x32x2_f32")):
            _log(f"alternate GEMM headline: {desc}")
            try:
                res[key] = alt_gemm(args, envs, desc, "C4g")
            except Exception as e:  # the alternate lines must never hide the headline
                res[key] = {"error": repr(e)}
    if world == 1 and rank == 0 and args.config == "C4" and not args.no_other:
        # C4g: the same amplitudes on the big-boundary-GEMM path (the planes GEMM's roofline)
        # C4x4: 4 blocks of C4 in one contraction (2^22 amplitudes; a larger correlated batch)
        for cfg in ("C2", "C3", "C4g", "C4x4"):
            _log(f"secondary config {cfg}")
            try:
                res[f"config_{cfg}"] = other_config(args, cfg)
            except Exception as e:  # the secondary lines must never hide the headline
                res[f"config_{cfg}"] = {"error": repr(e)}
    if not args.no_c5:   # every rank runs its share of the candidates
        if rank == 0:
            _log("C5 training line")
        try:
            port = int(os.environ.get("MASTER_PORT", "29500")) + 7
            c5 = c5_train(with_cpu=world == 1 and not args.no_cpu_baseline, port=port, rank=rank)
            if rank == 0:
                res["c5_train"] = c5
        except Exception as e:  # the secondary line must never hide the headline
            res["c5_train"] = {"error": repr(e)}
    if rank == 0:
        emit(res, args.details or os.environ.get("TQ_BENCH_DETAILS"))
    if world > 1:
        dist.destroy_process_group()


# ---- output: the driver parses the LAST stdout line (its tail holds a few KB), so that line is
# the compact headline; every secondary section goes to stderr as one `[bench-detail]` line each
# and, with --details / TQ_BENCH_DETAILS, the full result to a JSON file
HEADLINE_MAX_BYTES = 2048   # well inside the driver's stdout tail
SECONDARY_KEYS = ("config_C2", "config_C3", "config_C4g", "config_C4x4", "config_C3d", "c5_train",
                  "alt_f16_gemm_side_split", "alt_bf16_split", "alt_f32_mfma")


def _short(s, n: int):
    s = "" if s is None else str(s)
    return s if len(s) <= n else s[: n - 3] + "..."


def _sig(x, n: int = 5):
    """A float rounded to n significant digits (the compact line's secondary numbers)."""
    if not isinstance(x, float) or x == 0.0 or x != x:
        return x
    return float(f"{x:.{n}g}")


def _pick(d, keys):
    d = d or {}
    return {k: d[k] for k in keys if k in d}


def headline(res: dict) -> dict:
    """The compact headline object (the last stdout line): the contract keys, the dominant
    kernel's roofline, the CPU baseline and one [value, ms, frac] triple per secondary line."""
    h = _pick(res, ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                    "scaling", "vs_baseline", "dtype", "data"))
    cfg = dict(res.get("config") or {})
    if "workload" in cfg:
        cfg["workload"] = _short(cfg["workload"], 160)
    h["config"] = _rounded(cfg)
    t = res.get("timing") or {}
    h["timing"] = _rounded(_pick(t, ("inflight", "group", "latency_ms_per_step", "eager_profiled_ms_per_step")))
    rf = res.get("roofline") or {}
    r = _rounded(_pick(rf, ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_vs_algorithmic",
                            "frac_rocprof", "avg_launch_us_events", "avg_launch_us_rocprof", "launches_timed",
                            "algorithmic_bytes_per_step", "aggregate_GBps", "aggregate_frac",
                            "clock_GHz_in_kernel")))
    r["kernel"] = _short(rf.get("kernel"), 60)
    for k in ("traffic_source", "rocprof_source"):
        if k in rf:
            r[k] = _short(rf[k], 60)
    h["roofline"] = r
    if res.get("roofline_gemm"):
        h["roofline_gemm"] = _rounded(_pick(res["roofline_gemm"], ("achieved", "peak", "unit", "frac")))
    cb = res.get("cpu_baseline")
    if cb:
        h["cpu_baseline"] = _rounded(_pick(cb, ("value", "unit", "cores", "kind", "cpu_model", "error")))
        if "sample" in cb:
            h["cpu_baseline"]["sample"] = _short(cb["sample"], 100)
    sec = {}
    for k in SECONDARY_KEYS:
        v = res.get(k)
        if not v:
            continue
        # [value, ms per step, roofline frac] (units: the section's, in the --details file)
        e = [_sig(v.get("value")), _sig(v.get("ms_per_step")),
             _sig((v.get("roofline") or {}).get("frac") if isinstance(v.get("roofline"), dict) else None)]
        if "error" in v:
            e = {"error": _short(v["error"], 60)}
        sec[k.replace("config_", "").replace("alt_", "")] = e
    p = res.get("permute")
    if p:
        sec["permute"] = [_sig(p.get("GBps")), _sig(p.get("frac")), p.get("bit_exact")]
    if res.get("slices_strong"):
        ss = res["slices_strong"]
        sec["slices_strong"] = [_sig(ss.get("value")), _sig(ss.get("ms_per_step")), ss.get("parallelism")]
    if sec:
        h["secondary"] = sec
    return h


def _rounded(d: dict) -> dict:
    return {k: _sig(v) for k, v in d.items()}


def headline_line(res: dict) -> str:
    """`headline(res)` as one JSON line of at most HEADLINE_MAX_BYTES (secondary numbers, then
    long strings dropped if it would not fit)."""
    h = headline(res)
    s = json.dumps(h, separators=(",", ":"))
    if len(s) > HEADLINE_MAX_BYTES:
        h.pop("secondary", None)
        s = json.dumps(h, separators=(",", ":"))
    if len(s) > HEADLINE_MAX_BYTES:
        for sect in (h, h.get("roofline", {}), h.get("timing", {}), h.get("cpu_baseline", {}), h.get("config", {})):
            for k, v in list(sect.items()):
                if isinstance(v, str) and len(v) > 60 and k not in ("metric", "unit"):
                    sect[k] = _short(v, 60)
        s = json.dumps(h, separators=(",", ":"))
    return s


def emit(res: dict, details_path=None) -> None:
    """Secondary sections -> stderr (one line each), full result -> `details_path` (optional),
    the compact headline -> the last stdout line."""
    for k, v in res.items():
        if isinstance(v, dict) and k not in ("config", "timing"):
            print(f"[bench-detail] {k} {json.dumps(v, separators=(',', ':'))}", file=sys.stderr, flush=True)
    if details_path:
        try:
            d = os.path.dirname(os.path.abspath(details_path))
            os.makedirs(d, exist_ok=True)
            with open(details_path, "w") as f:
                json.dump(res, f, indent=1)
        except OSError as e:
            print(f"[bench] could not write {details_path}: {e!r}", file=sys.stderr, flush=True)
    sys.stderr.flush()
    print(headline_line(res), flush=True)


if __name__ == "__main__":
    main()
