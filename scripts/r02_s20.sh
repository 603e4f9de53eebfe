#!/bin/bash
# Round-2 GPU session 20: boundary-GEMM 3M tile variants (TQ_GEMM_VARIANT 0..3): parity + timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "gv0 120 env TQ_GEMM_VARIANT=0 python scripts/gemm_bench.py" \
  "gv1 120 env TQ_GEMM_VARIANT=1 python scripts/gemm_bench.py" \
  "gv2 120 env TQ_GEMM_VARIANT=2 python scripts/gemm_bench.py" \
  "gv3 120 env TQ_GEMM_VARIANT=3 python scripts/gemm_bench.py" \
  "gt1 200 env TQ_GEMM_VARIANT=1 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k gemm --timeout 120 --timeout-method thread" \
  "gt2 200 env TQ_GEMM_VARIANT=2 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k gemm --timeout 120 --timeout-method thread" \
  "gt3 200 env TQ_GEMM_VARIANT=3 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -k gemm --timeout 120 --timeout-method thread"
