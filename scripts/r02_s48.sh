#!/bin/bash
# Round-2 GPU session 48: pre-split boundary-GEMM operands (producers store f16 terms, GEMM
# regroups them): parity, window fallback, C4 bench, kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "p48 300 python -u -m pytest tests/test_presplit_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread" \
  "k48 400 python -u -m pytest tests/test_fullsize_gpu.py tests/test_contract_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "b48 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "kt48 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt48 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt"
