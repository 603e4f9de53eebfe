#!/bin/bash
# Round-2 GPU session 23: f16 2-term split complex64 GEMM: kernel parity, timing vs bf16 split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k23 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf -k gemm_c64 --timeout 120 --timeout-method thread" \
  "g23h 200 python scripts/gemm_c64_bench.py" \
  "g23b 200 env TQ_GEMM_F16=0 python scripts/gemm_c64_bench.py --bench-shape" \
  "f23 300 python -u -m pytest tests/test_fullsize_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread"
