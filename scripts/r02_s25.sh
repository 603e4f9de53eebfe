#!/bin/bash
# Round-2 GPU session 25: f16 split GEMM (fma_mix split, saddr loads): parity + timing, bf16 timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k25 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf -k gemm_c64 --timeout 120 --timeout-method thread" \
  "d0 100 env TQ_GEMM_DIAG=0 python scripts/gemm_c64_bench.py --bench-shape" \
  "d1 100 env TQ_GEMM_DIAG=1 python scripts/gemm_c64_bench.py --bench-shape" \
  "d2 100 env TQ_GEMM_DIAG=2 python scripts/gemm_c64_bench.py --bench-shape" \
  "d3 100 env TQ_GEMM_DIAG=3 python scripts/gemm_c64_bench.py --bench-shape" \
  "b25 100 env TQ_GEMM_F16=0 python scripts/gemm_c64_bench.py --bench-shape"
