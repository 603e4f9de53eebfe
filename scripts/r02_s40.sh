#!/bin/bash
# Round-2 GPU session 40: runtime f16 tile variants (gemm_f16_var): kernel tests on all complex64
# kernels, single-GPU projections of the per-rank time (rank_sim).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "k40 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -rf --timeout 120 --timeout-method thread" \
  "r40 300 python scripts/rank_sim.py C4"
