#!/usr/bin/env python3
"""The bench headline phase ALONE (C4 BlockPipeline: --group blocks per lockstep group,
--inflight groups on their own streams, `warmup` + `steps` blocks), for a rocprofv3 kernel trace
of exactly the regime the headline runs in:
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 scripts/headline_trace.py
A 100-ms idle gap separates the warmup from the timed steps, so scripts/regime_summary.py can
cut the trace there.  Prints one JSON line (ms per block by the host clock)."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import tneq_qc_amd  # noqa: F401
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.sampling import BlockPipeline

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C4")
ap.add_argument("--group", type=int, default=1)
ap.add_argument("--inflight", type=int, default=4)
ap.add_argument("--steps", type=int, default=48)
ap.add_argument("--warmup", type=int, default=16)
a = ap.parse_args()
dev = torch.device("cuda:0")
pipe = BlockPipeline(config_task(a.config), list(range(max(64, a.group * a.inflight))), inflight=a.inflight,
                     group=a.group, device=dev)
for _ in range(a.warmup):
    pipe.step()
pipe.synchronize()
time.sleep(0.1)
t0 = time.perf_counter()
for _ in range(a.steps):
    pipe.step()
pipe.synchronize()
dt = time.perf_counter() - t0
print(json.dumps({"config": a.config, "group": a.group, "inflight": a.inflight, "steps": a.steps,
                  "ms_per_block": dt / a.steps * 1e3}))
