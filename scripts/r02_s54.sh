#!/bin/bash
# Round-2 GPU session 54: C5 candidates on separate streams: equality test, c5_bench one stream
# vs eight streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "t54 300 python -u -m pytest tests/test_c5_streams_gpu.py tests/test_autograd_gpu.py tests/test_optim_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "c5a 200 python scripts/c5_bench.py --one-stream --cpu-steps 0" \
  "c5b 200 python scripts/c5_bench.py --cpu-steps 0"
