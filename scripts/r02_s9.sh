#!/bin/bash
# Round-2 GPU session 9: reverse-mode autograd parity; C5 training-step bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "agrad 300 python -u -m pytest tests/test_autograd_gpu.py tests/test_strategy_gpu.py tests/test_data_gpu.py tests/test_optim_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "c5 300 python scripts/c5_bench.py --steps 10 --warmup 2 --cpu-steps 1"
