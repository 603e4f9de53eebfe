#!/bin/bash
# Round-2 GPU session 51: slice lanes (C3: 8 slices per batch, sweep levels merged across lanes):
# parity (full-size, contract, distributed, tree, presplit), C3 / C4 bench, C3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k51 600 python -u -m pytest tests/test_fullsize_gpu.py tests/test_contract_gpu.py tests/test_distributed_gpu.py tests/test_presplit_gpu.py tests/test_tree_gpu.py -m gpu -x -q -rf --timeout 200 --timeout-method thread" \
  "c3_51 300 python bench.py --config C3 --no-cpu-baseline --no-c5 --no-alt" \
  "b51 300 python bench.py --no-cpu-baseline --no-c5 --no-alt" \
  "kt51 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt51 -o run -- python3 bench.py --config C3 --no-cpu-baseline --no-c5 --no-alt"
