#!/usr/bin/env python3
"""Summarize the PMC passes of scripts/pmc_gemm_bf16.sh (or pmc_gemm_f16.sh: 4th argument "f16")
into profiles/pmc_gemm_{bf16,f16}_r02.json: MFMA busy fraction of the split boundary GEMM
(SQ_VALU_MFMA_BUSY_CYCLES advances 32 cycles per v_mfma_f32_32x32x16_bf16 / _f16), the effective shader clock (GRBM_GUI_ACTIVE summed over the 8
XCDs / kernel duration), and HBM bytes per launch (FETCH_SIZE doubled per the gfx950 correction
in MI355X_MICROARCH.md's HBM section, + WRITE_SIZE)."""
import collections, csv, json, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_gemm_bf16_r02.json"
kind = sys.argv[3] if len(sys.argv) > 3 else "bf16"
# slices per launch (the plan's slice lanes: one batched launch per batch) and split-K count
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 1
splits = int(sys.argv[5]) if len(sys.argv) > 5 else 4
F16 = kind == "f16"
frag = "SplitF16" if F16 else "SplitBF16"
pre = "pmcf" if F16 else "pmcx"
kt = "ktf" if F16 else "ktx"


def passes(d):
    agg = collections.defaultdict(list)
    n = set()
    for r in csv.DictReader(open(f"{root}/{d}/run_counter_collection.csv")):
        if frag not in r["Kernel_Name"]:
            continue
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        n.add(r["Dispatch_Id"])
    return {k: sum(v) / len(v) for k, v in agg.items()}, len(n)


c1, n1 = passes(pre + "1")
c2, _ = passes(pre + "2")
c3, _ = passes(pre + "3")
# kernel duration from the kernel-trace pass (same command, no counters)
dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f"{root}/{kt}/run_kernel_trace.csv"))
       if frag in r["Kernel_Name"]]
avg_ns = sum(dur) / len(dur)
M = N = 1024
K = 65536
n_mfma = batch * (12 if F16 else 24) * (M // 32) * (N // 32) * (K // 16)  # 4M x (3 | 6) term products per tile-step
cyc_xcd = c1["GRBM_GUI_ACTIVE"] / 8
res = {
    "config": "C4",
    "kernel": ("gemm_c64_kouter_split_kernel<TileH, SplitF16> (complex64 via 2-term f16 split of the "
               "power-of-two-scaled operands, 4M, " if F16 else
               "gemm_c64_kouter_split_kernel<TileX, SplitBF16> (complex64 via exact 3-term bf16 split, 4M, ")
              + f"M=N=1024, K=65536 per slice, block 128x128, batch {batch} (slice lanes), split-K {splits})",
    "command": f"scripts/pmc_gemm_{kind}.sh (rocprofv3 --pmc ... --kernel-include-regex gemm_c64 -- python3 bench.py "
               "--no-cpu-baseline --no-c5 --steps 2 --warmup 1; FETCH_SIZE and WRITE_SIZE in separate passes; "
               "durations from a --kernel-trace pass)",
    "launches": n1,
    "counters_avg_per_launch": c1,
    "expected_mfma_per_launch": n_mfma,
    "busy_cycles_per_mfma": c1["SQ_VALU_MFMA_BUSY_CYCLES"] / n_mfma,
    "avg_launch_ns_trace": avg_ns,
    "cycles_per_xcd": cyc_xcd,
    "effective_clock_GHz": cyc_xcd / avg_ns if cyc_xcd / avg_ns <= 2.4 else None,   # null: unphysical (short dispatch)
    "mfma_busy_frac": c1["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc_xcd * 256 * 4),
    "FETCH_SIZE_kB_per_launch": c2.get("FETCH_SIZE"),
    "WRITE_SIZE_kB_per_launch": c3.get("WRITE_SIZE"),
    "hbm_bytes_per_launch": (2 * c2.get("FETCH_SIZE", 0) + c3.get("WRITE_SIZE", 0)) * 1024,
    "batch": batch,
    "splits": splits,
    "algorithmic_bytes_per_launch": batch * ((M * K + N * K) * 8 + splits * M * N * 8),
    "definition": "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 XCDs * 256 CUs * 4 SIMDs); "
                  "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (kB, gfx950 FETCH correction); algorithmic bytes = "
                  "batch x (A + B once + the split-K partial slabs, or C, written)",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
