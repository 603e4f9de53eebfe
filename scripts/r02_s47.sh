#!/bin/bash
# Round-2 GPU session 47: timing of the pre-split f16 GEMM form (terms regrouped, no split
# arithmetic; gemm_f16_var 3 on raw complex64 bits: a timing diagnostic) vs the default split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "g47a 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g47a -o run -- python3 scripts/gemm_c64_bench.py --bench-shape --reps=20" \
  "g47b 200 env TQ_GEMM_F16_VAR=3 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/g47b -o run -- python3 scripts/gemm_c64_bench.py --bench-shape --reps=20"
for d in g47a g47b; do echo "== $d"; grep -i "split_kernel\|absmax" gpurun_out/$d/run_kernel_stats.csv | cut -c1-250; done
