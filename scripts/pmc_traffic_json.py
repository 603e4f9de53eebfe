#!/usr/bin/env python3
"""Summarize scripts/pmc_traffic.sh <tag> into profiles/pmc_c2_<tag>.json, pmc_c3_<tag>.json (the sweep
launches' HBM bytes, the schema bench.py reads for the C2 / C3 roofline traffic) and
pmc_c5_<tag>.json (every kernel of the C5 training step, per candidate-step = per SGDG dispatch).
Bytes = 2 * FETCH_SIZE + WRITE_SIZE (kB x 1024; the gfx950 FETCH_SIZE correction of
MI355X_MICROARCH.md).
    python3 scripts/pmc_traffic_json.py gpurun_out/t<tag> <tag>"""
import csv, glob, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tr05"
TAG = sys.argv[2] if len(sys.argv) > 2 else "r05"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")


def counter(cfg, c):
    """(sum of the counter over dispatches in kB, dispatches, SGDG dispatches)"""
    tot, disp, sgdg = 0.0, set(), set()
    for f in glob.glob(os.path.join(root, f"{cfg}_{c}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != c:
                continue
            tot += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
            if "sgdg" in r["Kernel_Name"].lower():
                sgdg.add(r["Dispatch_Id"])
    return tot, len(disp), len(sgdg)


for cfg in ("C2", "C3", "C4", "C4x4"):
    fk, fd, _ = counter(cfg, "FETCH_SIZE")
    wk, wd, _ = counter(cfg, "WRITE_SIZE")
    if not fd:
        continue
    d = {"config": cfg,
         "command": f"rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) --kernel-include-regex sweep -- "
                    f"python3 bench.py --config {cfg} --no-cpu-baseline --no-c5 --no-alt --no-other --steps 2 --warmup 1",
         "definition": "sweep_hbm_bytes = sum over the sweep dispatches of (2*FETCH_SIZE + WRITE_SIZE) * 1024",
         "sweep_dispatches": fd, "write_dispatches": wd, "sweep_hbm_bytes": (2 * fk + wk) * 1024,
         "fetch_kB_total": fk, "write_kB_total": wk}
    json.dump(d, open(os.path.join(OUT, f"pmc_{cfg.lower()}_{TAG}.json"), "w"), indent=1)
    print(cfg, fd, "dispatches", round(d["sweep_hbm_bytes"] / fd), "B per dispatch")
fk, fd, fs = counter("C5", "FETCH_SIZE")
wk, wd, ws = counter("C5", "WRITE_SIZE")
if fd and fs:
    per = (2 * fk + wk) * 1024 / fs
    d = {"config": "C5",
         "command": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) -- python3 scripts/c5_bench.py --steps 2 "
                    "--warmup 1 --cpu-steps 0",
         "definition": "hbm_bytes_per_candidate_step = (2*FETCH_SIZE + WRITE_SIZE) * 1024 over every kernel of the "
                       "run / SGDG dispatches (one per candidate-step); includes torch's own kernels of the step "
                       "(loss reductions, copies) and the run's setup",
         "dispatches": fd, "sgdg_dispatches": fs, "hbm_bytes_total": (2 * fk + wk) * 1024,
         "hbm_bytes_per_candidate_step": per}
    json.dump(d, open(os.path.join(OUT, f"pmc_c5_{TAG}.json"), "w"), indent=1)
    print("C5", fs, "candidate-steps", round(per), "B per candidate-step")
