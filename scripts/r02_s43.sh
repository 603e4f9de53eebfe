#!/bin/bash
# Round-2 GPU session 43: short-K split rule (>= 8 K-tiles per split): kernel tests, C3 / C2 / C4
# bench lines (dominant-kernel roofline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k43 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "c3 400 python bench.py --config C3 --no-c5 --no-alt" \
  "c2 400 python bench.py --config C2 --no-c5 --no-alt" \
  "c4 300 python bench.py --no-cpu-baseline --no-c5 --no-alt"
