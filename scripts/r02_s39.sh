#!/bin/bash
# Round-2 GPU session 39: f16 split GEMM, Gauss 3M variant (TQ_GEMM_F16_VAR=2): parity + timing
# vs the default and the 4-wave 4M tile; fullsize slice parity and bench on the 3M variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k39 300 env TQ_GEMM_F16_VAR=2 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf -k 'gemm_c64 and f16' --timeout 120 --timeout-method thread" \
  "v2 100 env TQ_GEMM_F16_VAR=2 python scripts/gemm_c64_bench.py" \
  "v0 100 env TQ_GEMM_F16_VAR=0 python scripts/gemm_c64_bench.py --bench-shape" \
  "f39 300 env TQ_GEMM_F16_VAR=2 python -u -m pytest tests/test_fullsize_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "b39 300 env TQ_GEMM_F16_VAR=2 python bench.py --no-cpu-baseline --no-c5 --no-alt"
