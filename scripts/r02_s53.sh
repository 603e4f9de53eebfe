#!/bin/bash
# Round-2 GPU session 53: slice lanes -- one batched GEMM launch per batch (uniform lane stride) and the lanes summed before one output permute: parity (incl. kernels, tree, strategy) + C3 bench + trace.
# compile with the lanes hint): C3 parity + bench + kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k53 600 python -u -m pytest tests/test_fullsize_gpu.py tests/test_distributed_gpu.py tests/test_presplit_gpu.py tests/test_contract_gpu.py tests/test_kernels_gpu.py tests/test_tree_gpu.py tests/test_strategy_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "c3_53 300 python bench.py --config C3 --no-cpu-baseline --no-c5 --no-alt" \
  "kt53 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt53 -o run -- python3 bench.py --config C3 --no-cpu-baseline --no-c5 --no-alt"
