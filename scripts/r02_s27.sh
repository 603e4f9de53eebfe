#!/bin/bash
# Round-2 GPU session 27: split GEMMs with 16-B staging loads: parity + timing (f16, bf16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k27 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf -k gemm_c64 --timeout 120 --timeout-method thread" \
  "h27 100 python scripts/gemm_c64_bench.py" \
  "b27 100 env TQ_GEMM_F16=0 python scripts/gemm_c64_bench.py --bench-shape"
