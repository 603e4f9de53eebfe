#!/bin/bash
# Round-2 GPU session 41: sweep2 16-B paired stores (complex64): sweep / contraction parity, bench,
# kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t41 600 python -u -m pytest tests/test_contract_gpu.py tests/test_fullsize_gpu.py tests/test_golden_gpu.py tests/test_strategy_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "b41 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "kt41 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt41 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt"
