#!/usr/bin/env python3
"""Summarize scripts/prof_round.sh <tag>: per kernel family (boundary GEMM, dense sweep, sweep2) and launch
shape (grid size), the average counters per dispatch over the PMC passes, the trace duration, the
HBM bytes (2*FETCH_SIZE + WRITE_SIZE, kB; the gfx950 FETCH correction of MI355X_MICROARCH.md), the
effective shader clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), the MFMA busy fraction and the
wave-cycle shares.  Writes profiles/pmc_c4_<tag>.json, profiles/pmc_gemm_f16_<tag>.json (the
schema bench.py reads for the roofline) and profiles/rocprof_<tag>_bench_kernel_stats.csv.
    python3 scripts/prof_round_json.py gpurun_out/p<tag> <tag>"""
import collections, csv, json, os, shutil, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/p04"
TAG = sys.argv[2] if len(sys.argv) > 2 else "r04"
FAM = {"gemm_f16_split": "split_kernel", "gemm_planes": "gemm_planes_kernel", "dense_sweep": "sweepd_kernel",
       "sweep2": "sweep2_kernel"}


def fam_of(name):
    for f, frag in FAM.items():
        if frag in name:
            return f
    return None


def dispatches(path, value_col=True):
    """{(family, grid): [per-dispatch dict in dispatch order]}"""
    per = collections.OrderedDict()
    meta = {}
    for r in csv.DictReader(open(path)):
        f = fam_of(r["Kernel_Name"])
        if f is None:
            continue
        d = int(r["Dispatch_Id"])
        if value_col:
            per.setdefault(d, collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
        else:
            per[d] = {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])}
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or ""
        meta[d] = (f, g)
    out = collections.defaultdict(list)
    for d in sorted(per):
        out[meta[d]].append(per[d])
    return out


trace = dispatches(f"{root}/k0/run_kernel_trace.csv", value_col=False)
passes = [dispatches(f"{root}/p{i}/run_counter_collection.csv") for i in (1, 2, 3, 4)]
res = {"config": "C4",
       "command": f"scripts/prof_round.sh {TAG}: rocprofv3 --pmc <set> --kernel-include-regex "
                  "'split_kernel|gemm_planes_kernel|sweepd_kernel|sweep2_kernel' -- python3 bench.py --no-cpu-baseline --no-c5 "
                  "--no-alt --steps 2 --warmup 1 (4 counter passes + a kernel-trace pass of the same command)",
       "definitions": {
           "hbm_bytes": "2*FETCH_SIZE + WRITE_SIZE (kB x 1024; gfx950 FETCH_SIZE correction)",
           "effective_clock_GHz": "GRBM_GUI_ACTIVE / 8 XCDs / trace duration, null when > 2.4 GHz (unphysical for "
                                  "short dispatches); the in-kernel clock: profiles/kclock_*.json",
           "mfma_busy_frac": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 256 CUs * 4 SIMDs)",
           "wait_frac": "SQ_WAIT_ANY / SQ_WAVE_CYCLES (share of resident wave cycles spent waiting)",
           "wait_lds_frac": "SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES"},
       "groups": []}
for key in sorted(trace, key=lambda k: (k[0], -len(trace[k]))):
    fam, grid = key
    ns = [x["ns"] for x in trace[key]]
    avg_ns = sum(ns) / len(ns)
    c = collections.defaultdict(list)
    for p in passes:
        for disp in p.get(key, []):
            for k, v in disp.items():
                c[k].append(v)
    c = {k: sum(v) / len(v) for k, v in c.items()}
    g = {"family": fam, "grid": grid, "dispatches": len(ns), "avg_ns": avg_ns, "counters_avg": c}
    if "GRBM_GUI_ACTIVE" in c and avg_ns > 0:
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        # GRBM_GUI_ACTIVE / 8 / duration is not a clock for short dispatches (r05: 2.8-10.8 GHz):
        # kept only when physical (<= 2.4 GHz); the in-kernel clock is scripts/kernel_clock.py's
        clk = cyc / avg_ns
        g["effective_clock_GHz"] = clk if clk <= 2.4 else None
        g["mfma_busy_frac"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (cyc * 256 * 4)
    if c.get("SQ_WAVE_CYCLES"):
        g["wait_frac"] = c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"]
        g["wait_inst_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
        g["wait_lds_frac"] = c.get("SQ_WAIT_INST_LDS", 0) / c["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        hb = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        g["hbm_bytes"] = hb
        g["hbm_GBps"] = hb / avg_ns
    res["groups"].append(g)
os.makedirs("profiles", exist_ok=True)
json.dump(res, open(f"profiles/pmc_c4_{TAG}.json", "w"), indent=1)

# the boundary GEMM in the schema bench.py reads (pmc_gemm_f16_r0N.json)
gg = [g for g in res["groups"] if g["family"] == "gemm_f16_split"]
if gg:
    g = max(gg, key=lambda x: x["dispatches"])
    batch, M, N, K = 4, 1024, 1024, 65536
    g3 = os.environ.get("TQ_GEMM_F16_VAR", "6") in ("2", "5", "6")   # Gauss 3M: 9 MFMAs per tile-step
    n_mfma = batch * (9 if g3 else 12) * (M // 32) * (N // 32) * (K // 16)
    c = g["counters_avg"]
    gem = {"config": "C4",
           "kernel": ("gemm_c64_kouter_split_kernel<TileH8G3, SplitF16> (complex64 via 2-term f16 split of the "
                      "power-of-two-scaled operands, Gauss 3M" if g3 else
                      "gemm_c64_kouter_split_kernel<TileH, SplitF16> (complex64 via 2-term f16 split of the "
                      "power-of-two-scaled operands, 4M") +
                     ", M=N=1024, K=65536 per slice, block 128x128, batch 4 (slice lanes), split-K 1)",
           "command": res["command"],
           "launches": g["dispatches"],
           "counters_avg_per_launch": c,
           "expected_mfma_per_launch": n_mfma,
           "busy_cycles_per_mfma": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / n_mfma,
           "avg_launch_ns_trace": g["avg_ns"],
           "effective_clock_GHz": g.get("effective_clock_GHz"),
           "mfma_busy_frac": g.get("mfma_busy_frac"),
           "wait_frac": g.get("wait_frac"),
           "wait_lds_frac": g.get("wait_lds_frac"),
           "FETCH_SIZE_kB_per_launch": c.get("FETCH_SIZE"),
           "WRITE_SIZE_kB_per_launch": c.get("WRITE_SIZE"),
           "hbm_bytes_per_launch": g.get("hbm_bytes"),
           "batch": batch, "splits": 1,
           "algorithmic_bytes_per_launch": batch * ((M * K + N * K) * 8 + M * N * 8),
           "definition": res["definitions"]["mfma_busy_frac"] + "; " + res["definitions"]["hbm_bytes"]
                         + "; algorithmic bytes = batch x (A + B once + C written)"}
    json.dump(gem, open(f"profiles/pmc_gemm_f16_{TAG}.json", "w"), indent=1)
# the pre-split boundary GEMM (tq_gemmp.hip, default since r05) in the same schema
gp = [g for g in res["groups"] if g["family"] == "gemm_planes"]
if gp:
    g = max(gp, key=lambda x: x["dispatches"])
    batch, M, N, K = 4, 1024, 1024, 65536
    n_mfma = batch * 3 * 3 * (M // 16) * (N // 16) * (K // 32)   # v_mfma_f32_16x16x32_f16
    c = g["counters_avg"]
    gem = {"config": "C4",
           "kernel": ("gemm_planes_kernel (complex64 from six f16 term planes per operand stored by the dense "
                      "producers; Gauss 3M x 3 term products on v_mfma_f32_16x16x32_f16, 256x256 tiles, "
                      "LDS-DMA staged planes, M=N=1024, K=65536 per slice, batch 4 (slice lanes), split-K 4)"),
           "command": res["command"],
           "launches": g["dispatches"],
           "counters_avg_per_launch": c,
           "expected_mfma_per_launch": n_mfma,
           "busy_cycles_per_mfma": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / n_mfma,
           "avg_launch_ns_trace": g["avg_ns"],
           "effective_clock_GHz": g.get("effective_clock_GHz"),
           "mfma_busy_frac": g.get("mfma_busy_frac"),
           "wait_frac": g.get("wait_frac"),
           "wait_lds_frac": g.get("wait_lds_frac"),
           "FETCH_SIZE_kB_per_launch": c.get("FETCH_SIZE"),
           "WRITE_SIZE_kB_per_launch": c.get("WRITE_SIZE"),
           "hbm_bytes_per_launch": g.get("hbm_bytes"),
           "batch": batch, "splits": 4,
           "algorithmic_bytes_per_launch": batch * ((M * K + N * K) * 8 + M * N * 8),
           "plane_bytes_per_launch": batch * (M * K + N * K) * 12,
           "definition": res["definitions"]["mfma_busy_frac"] + "; " + res["definitions"]["hbm_bytes"]
                         + "; algorithmic bytes = batch x (complex64 A + B once + C written); the planes are "
                           "12 B per operand element (1.5x the complex64 bytes)"}
    json.dump(gem, open(f"profiles/pmc_gemm_planes_{TAG}.json", "w"), indent=1)
st = f"{root}/kt/run_kernel_stats.csv"
if os.path.exists(st):
    shutil.copy(st, f"profiles/rocprof_{TAG}_bench_kernel_stats.csv")
for g in res["groups"]:
    print(g["family"], g["grid"], g["dispatches"], f"{g['avg_ns']/1e3:.1f}us",
          {k: (round(g[k], 3) if g[k] is not None else None) for k in ("effective_clock_GHz", "mfma_busy_frac", "wait_frac", "wait_lds_frac")
           if g.get(k) is not None}, f"{g.get('hbm_GBps', 0):.0f} GB/s")
