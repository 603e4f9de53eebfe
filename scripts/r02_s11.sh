#!/bin/bash
# Round-2 GPU session 11: tree contraction (log2 W merge stages) on native plans.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "tree 400 python -u -m pytest tests/test_tree_gpu.py tests/test_distributed_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread"
