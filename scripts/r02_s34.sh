#!/bin/bash
# Round-2 GPU session 34: f16 split GEMM with 3 staging sets (unroll 6) and fragment reads in
# MFMA-pair order: kernel parity + timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k34 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf -k gemm_c64 --timeout 120 --timeout-method thread" \
  "h34 100 python scripts/gemm_c64_bench.py --bench-shape" \
  "b34 100 env TQ_GEMM_F16=0 python scripts/gemm_c64_bench.py --bench-shape"
