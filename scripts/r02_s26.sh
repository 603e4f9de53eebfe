#!/bin/bash
# Round-2 GPU session 26: f16 split GEMM memory-path diagnostics (DG 5 = loads only, fully consumed)
# with the clock from GRBM_GUI_ACTIVE.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "d5 100 env TQ_GEMM_DIAG=5 python scripts/gemm_c64_bench.py --bench-shape" \
  "p5 120 env TQ_GEMM_DIAG=5 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES TCP_TCC_READ_REQ_sum --kernel-include-regex split_kernel --output-format csv -d gpurun_out/p5 -o run -- python3 scripts/gemm_c64_bench.py --bench-shape" \
  "p0 120 env TQ_GEMM_DIAG=0 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES TCP_TCC_READ_REQ_sum --kernel-include-regex split_kernel --output-format csv -d gpurun_out/p0 -o run -- python3 scripts/gemm_c64_bench.py --bench-shape" \
  "p1 120 env TQ_GEMM_DIAG=1 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --kernel-include-regex split_kernel --output-format csv -d gpurun_out/p1 -o run -- python3 scripts/gemm_c64_bench.py --bench-shape"
