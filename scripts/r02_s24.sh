#!/bin/bash
# Round-2 GPU session 24: f16 split GEMM diagnostic variants (timing only; 1 no MFMA, 2 no split,
# 3 no global loads, 4 no barrier) at the bench shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "d0 100 env TQ_GEMM_DIAG=0 python scripts/gemm_c64_bench.py --bench-shape" \
  "d1 100 env TQ_GEMM_DIAG=1 python scripts/gemm_c64_bench.py --bench-shape" \
  "d2 100 env TQ_GEMM_DIAG=2 python scripts/gemm_c64_bench.py --bench-shape" \
  "d3 100 env TQ_GEMM_DIAG=3 python scripts/gemm_c64_bench.py --bench-shape" \
  "d4 100 env TQ_GEMM_DIAG=4 python scripts/gemm_c64_bench.py --bench-shape" \
  "p24 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex split_kernel --output-format csv -d gpurun_out/p24 -o run -- python3 scripts/gemm_c64_bench.py --bench-shape" \
  "q24 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC --kernel-include-regex split_kernel --output-format csv -d gpurun_out/q24 -o run -- python3 scripts/gemm_c64_bench.py --bench-shape"
