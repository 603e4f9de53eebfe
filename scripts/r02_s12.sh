#!/bin/bash
# Round-2 GPU session 12: generic MFMA GEMM (f64 / c128 / f32 / c64) vs torch.matmul + kernel tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "ktests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_contract_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "g64 300 python scripts/gemm64_bench.py f64 f32"
