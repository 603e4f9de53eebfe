#!/usr/bin/env python3
"""Summarize scripts/prof_r04_small.sh into profiles/pmc_c2_r04.json, profiles/pmc_c3_r04.json
(the sweep launches' HBM bytes: 2*FETCH_SIZE + WRITE_SIZE, kB x 1024, the gfx950 FETCH_SIZE
correction of MI355X_MICROARCH.md; bench.py reads them for the C2 / C3 roofline `traffic`) and
profiles/c5_trace_r04.json (the C5 training bench's kernel trace: launches per candidate-step and
the GPU-busy fraction over the timed steps)."""
import collections, csv, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/p04s"


def per_dispatch(path):
    v = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        v[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return v


os.makedirs("profiles", exist_ok=True)
for cfg in ("C2", "C3"):
    try:
        f = per_dispatch(f"{root}/{cfg}_f/run_counter_collection.csv")
        w = per_dispatch(f"{root}/{cfg}_w/run_counter_collection.csv")
    except FileNotFoundError:
        continue
    res = {"config": cfg,
           "command": f"rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate passes) --kernel-include-regex sweep "
                      f"-- python3 bench.py --config {cfg} --no-cpu-baseline --no-c5 --no-alt --no-other "
                      f"--steps 2 --warmup 1",
           "definition": "sweep_hbm_bytes = sum over the sweep dispatches of (2*FETCH_SIZE + WRITE_SIZE) * 1024",
           "sweep_dispatches": len(f),
           "sweep_hbm_bytes": (2 * sum(f.values()) + sum(w.values()) * len(f) / max(1, len(w))) * 1024,
           "fetch_kB_total": sum(f.values()), "write_kB_total": sum(w.values()), "write_dispatches": len(w)}
    json.dump(res, open(f"profiles/pmc_{cfg.lower()}_r04.json", "w"), indent=1)
    print(cfg, res["sweep_dispatches"], res["sweep_hbm_bytes"])

try:
    rows = list(csv.DictReader(open(f"{root}/c5/run_kernel_trace.csv")))
except FileNotFoundError:
    rows = []
if rows:
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    sg = [k for k in ks if "sgdg_kernel" in k[2]]
    steps, cands = 10, 8
    timed = sg[-steps * cands:]
    t0 = sg[-steps * cands - 1][1]          # the last warmup step's optimizer launch ended
    t1 = timed[-1][1]
    win = [k for k in ks if t0 < k[0] <= t1]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    fam = collections.Counter(n.split("<")[0].split("(")[0] for _, _, n in win)
    res = {"config": "C5",
           "command": "rocprofv3 --kernel-trace -- python3 scripts/c5_bench.py --steps 10 --warmup 3 --cpu-steps 0",
           "window": "from the end of the last warmup step's SGDG launch to the end of the last timed one",
           "window_ms": (t1 - t0) / 1e6, "kernels_in_window": len(win),
           "launches_per_candidate_step": len(win) / (steps * cands),
           "gpu_busy_frac": busy / max(1, t1 - t0),
           "definition": "gpu_busy_frac = union of kernel intervals in the window / window length (traced run)",
           "kernel_families": dict(fam.most_common(12))}
    json.dump(res, open("profiles/c5_trace_r04.json", "w"), indent=1)
    print("C5", res["launches_per_candidate_step"], res["gpu_busy_frac"])
