#!/usr/bin/env python3
"""Throughput of the §8(f) measurement-data path on one MI355X: the Hermite feature / Mx
generator (HBM-bound; algorithmic bytes = n * (8 + (K + K^2) * sizeof)), the inverse-CDF draw
(bytes = S * G * sizeof + G * sizeof + S * (4 + sizeof)), and whole EngineSiamese.sample calls
(grid contraction + draws) on a small brick wall.  Prints one JSON object."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import tneq_qc_amd  # noqa: F401
from tneq_qc_amd import ops
from tneq_qc_amd.core.engine_siamese import EngineSiamese

dev = torch.device("cuda:0")


def gpu_time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


res = {}

import math
k = np.arange(129, dtype=np.float64)
W = np.exp(-0.5 * (0.5 * math.log(2 * math.pi) + np.array([math.lgamma(int(v) + 1) for v in k])))
for dt, K, n in [(torch.complex64, 16, 1 << 20), (torch.complex128, 16, 1 << 20), (torch.float32, 16, 1 << 20),
                 (torch.complex64, 2, 1 << 24), (torch.complex64, 64, 1 << 16)]:
    x = torch.randn(n, dtype=torch.float64, device=dev)
    esz = torch.empty(0, dtype=dt).element_size()
    t = gpu_time(lambda: ops.hermite_features(x, K, W, dt))
    b = n * (8 + (K + K * K) * esz)
    res[f"hermite_{str(dt).split('.')[-1]}_K{K}_n{n}"] = {"us": t * 1e6, "GBps": b / t / 1e9}
for dt in (torch.float64, torch.float32):
    S, G = 1 << 16, 1000
    d = torch.rand(S, G, dtype=dt, device=dev)
    g = torch.linspace(-5, 5, G, dtype=dt, device=dev)
    u = torch.rand(S, dtype=torch.float32, device=dev)
    t = gpu_time(lambda: ops.inverse_cdf_sample(d, g, u))
    esz = d.element_size()
    b = S * G * esz + G * esz + S * (4 + esz)
    res[f"icdf_{str(dt).split('.')[-1]}_S{S}_G{G}"] = {"us": t * 1e6, "GBps": b / t / 1e9}
from tneq_qc_amd.backends import BackendFactory
from tneq_qc_amd.circuits import build_brick_wall_IM, incidence_to_graph, random_unitary_cores
from tneq_qc_amd.core import QCTN
for n_q, S, G in [(4, 256, 1000), (8, 64, 1000)]:
    eng = EngineSiamese(BackendFactory.create_backend("hip", device="cuda:0", dtype="complex128"), "balanced")
    q = QCTN(incidence_to_graph(build_brick_wall_IM(n_q, 2)))
    cores = random_unitary_cores(q, 5)
    q.cores_weights = {c: torch.from_numpy(cores[c]).to(dev) for c in q.cores}
    states = [torch.tensor([1.0, 0.0], dtype=torch.complex128, device=dev) for _ in range(n_q)]
    eng.sample(q, states, S, 2, bounds=[-4, 4], grid_size=G)   # compile + warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.sample(q, states, S, 2, bounds=[-4, 4], grid_size=G)
    torch.cuda.synchronize()
    dt_ = time.perf_counter() - t0
    res[f"sample_{n_q}q_S{S}_G{G}"] = {"s": dt_, "samples_per_s": S / dt_, "grid_points_per_s": S * G * n_q / dt_}
# §8(f) row 2: one training step of the symmetry-breaking loop shape (C5: 8-qubit 5-cell masked
# ansatz, complex128 core-only contraction, fidelity loss against a target, backward through the
# HIP expression = one more contraction per core, one Stiefel SGDG step)
from tneq_qc_amd.circuits import ansatz_qctn
from tneq_qc_amd.contractor import EinsumStrategy
be = BackendFactory.create_backend("hip", device="cuda:0", dtype="complex128")
bw = ansatz_qctn()
q = bw.qctn
eq, shapes = EinsumStrategy.build_core_only_expression(q)
expr = EinsumStrategy.create_contract_expression(eq, shapes)
tgt = expr(*[be.convert_to_tensor(bw.cores[c]) for c in q.cores]).detach().reshape(-1)
rng = np.random.default_rng(3)
params = [be.convert_to_tensor(bw.cores[c] + 0.1 * (rng.standard_normal(bw.cores[c].shape)
                                                     + 1j * rng.standard_normal(bw.cores[c].shape)))
          for c in q.cores]
state = {}


def train_step():
    global params, state
    ps = [p.detach().requires_grad_(True) for p in params]
    out = expr(*ps).reshape(-1)
    loss = 1.0 - torch.vdot(tgt, out).abs() ** 2 / (torch.vdot(tgt, tgt).real * torch.vdot(out, out).real)
    grads = torch.autograd.grad(loss, ps)
    params, state = be.optimizer_update(ps, list(grads), state, "sgdg", {"learning_rate": 0.01})
    return loss


for _ in range(3):
    train_step()
torch.cuda.synchronize()
t0 = time.perf_counter()
steps = 20
for _ in range(steps):
    loss = train_step()
torch.cuda.synchronize()
dt_ = (time.perf_counter() - t0) / steps
res["train_step_C5_ansatz"] = {"ms_per_step": dt_ * 1e3, "cores": len(q.cores), "loss": float(loss.detach())}
print(json.dumps(res))
