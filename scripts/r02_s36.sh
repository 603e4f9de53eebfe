#!/bin/bash
# Round-2 GPU session 36: f16 split GEMM diagnostics on the 4-wave tile (timing only): 3 = no
# MFMAs, 4 = no global loads; clock counters for each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
R="--kernel-include-regex split_kernel --output-format csv"
scripts/gpu_check.sh \
  "v3 100 env TQ_GEMM_F16_VAR=3 python scripts/gemm_c64_bench.py --bench-shape" \
  "v4 100 env TQ_GEMM_F16_VAR=4 python scripts/gemm_c64_bench.py --bench-shape" \
  "q0 100 env TQ_GEMM_F16_VAR=0 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY $R -d gpurun_out/q0 -o run -- python3 scripts/gemm_c64_bench.py --bench-shape" \
  "q3 100 env TQ_GEMM_F16_VAR=3 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY $R -d gpurun_out/q3 -o run -- python3 scripts/gemm_c64_bench.py --bench-shape" \
  "q4 100 env TQ_GEMM_F16_VAR=4 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY $R -d gpurun_out/q4 -o run -- python3 scripts/gemm_c64_bench.py --bench-shape"
