#!/bin/bash
# Round-2 GPU session 45: sweep2 store-phase epilogue gate (last gate applied in registers while
# the tile leaves LDS): parity, C4 bench, kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k45 400 python -u -m pytest tests/test_contract_gpu.py tests/test_fullsize_gpu.py tests/test_strategy_gpu.py tests/test_golden_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "b45 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "kt45 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt45 -o run -- python3 bench.py --no-cpu-baseline --no-c5 --no-alt"
