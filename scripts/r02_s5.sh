#!/bin/bash
# Round-2 GPU session 5: sweep2 chunk pipeline (stores drain under the next chunk's gates).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
scripts/gpu_check.sh \
  "ctests 300 python -u -m pytest tests/test_contract_gpu.py tests/test_fullsize_gpu.py tests/test_kernels_gpu.py -m gpu -q -rf --timeout 200 --timeout-method thread" \
  "bench 300 python bench.py --steps 10 --warmup 3" \
  "trace 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python3 scripts/rank_sim.py C4 1"
