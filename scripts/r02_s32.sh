#!/bin/bash
# Round-2 GPU session 31/32: row-pair swizzle + padded term planes of the split GEMM (store conflicts),
# sweep2 store loop split by producer tracking: parity + bench + kernel stats + conflicts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k32 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_gpu.py tests/test_contract_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "b32 400 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "kt32 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt32 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "c32 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-include-regex split_kernel --output-format csv -d gpurun_out/c32 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt --steps 2 --warmup 1"
